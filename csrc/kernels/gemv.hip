// Decode GEMV family (T = 1): y = W x with W block-quantised (Q4_K/Q5_K/Q6_K/Q8_0,
// F16/F32) in the planar layout and x quantised to q8 in the kernel prologue.
//
// Replaces upstream MMVQ (`mul_mat_vec_q` + `quantize_q8_1`) and the
// ops it is chained with (RMSNorm K2, RoPE K5, KV store K6, SwiGLU K11, residual
// add K10) by ONE launch per projection:
//
//   prologue  : [RMSNorm(x)*w] -> per-32 int8 quantisation -> LDS (K B + K/8 B)
//   body      : each wave owns NR output rows; lane l streams chunks l, l+64, ...
//               (16 B of 4/6-bit weights per lane per chunk = 1 KiB per wave
//               instruction, non-temporal: weights are read once per token)
//   epilogue  : wave-reduce, then store / residual add / SwiGLU / RoPE+KV append
//
// Geometry: 256-thread blocks (4 waves), grid-stride over row groups with the
// grid capped at 4 blocks per CU so the prologue is amortised over many rows.
#include "kernels.h"
#include "qdot.h"

namespace lfk {

static constexpr int kMaxBlocks = 1024;  // 256 CUs x 4

template <bool NORM>
__device__ __forceinline__ void quantize_x(const float* __restrict__ x, const float* __restrict__ nw, float eps, int K,
                                           int8_t* xq, float* xd, float* red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float scale = 1.f;
  if constexpr (NORM) {
    float ss = 0.f;
    for (int i = tid * 4; i < K; i += 1024) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    scale = rsqrtf(tot / (float)K + eps);
  }
  for (int i = tid * 4; i < K; i += 1024) {
    float4 v = *reinterpret_cast<const float4*>(x + i);
    if constexpr (NORM) {
      float4 w = *reinterpret_cast<const float4*>(nw + i);
      v.x *= scale * w.x; v.y *= scale * w.y; v.z *= scale * w.z; v.w *= scale * w.w;
    }
    float amax = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    amax = fmaxf(amax, __shfl_xor(amax, 4));
    const float d = amax * (1.f / 127.f);
    const float id = d > 0.f ? 1.f / d : 0.f;
    const int q0 = __float2int_rn(v.x * id), q1 = __float2int_rn(v.y * id);
    const int q2 = __float2int_rn(v.z * id), q3 = __float2int_rn(v.w * id);
    *reinterpret_cast<int*>(xq + i) = (q0 & 0xFF) | ((q1 & 0xFF) << 8) | ((q2 & 0xFF) << 16) | ((q3 & 0xFF) << 24);
    if ((tid & 7) == 0) xd[i >> 5] = d;
  }
  __syncthreads();
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// NR rows of one matrix against the LDS-resident q8 x, K-slice `ks` of `wk`
// (chunks ks*64 + lane + 64*wk*j). Loads for two passes of all NR rows are
// issued before any math (2*NR independent 16-B loads per lane in flight);
// out-of-range chunks are clamped (loaded, then ignored).
template <int QT, int NR>
__device__ __forceinline__ void load_pair(WRaw<QT> (&w)[2][NR], const RowPtr (&R)[NR], int c0, int step, int nchunks,
                                          int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = min(c0 + step * u + lane, nchunks - 1);
#pragma unroll
    for (int r = 0; r < NR; ++r) wload<QT>(w[u][r], R[r], c);
  }
}

template <int QT, int NR>
__device__ __forceinline__ void dot_pair(const WRaw<QT> (&w)[2][NR], int c0, int step, int nchunks, const int8_t* xq,
                                         const float* xd, float (&acc)[NR], int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = c0 + step * u + lane;
    if (c < nchunks) {
      XChunk X;
      load_x<QT>(X, xq, xd, c);
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[r] += wdot<QT>(w[u][r], X, c);
    }
  }
}

template <int QT, int NR>
__device__ __forceinline__ void dot_rows(const RowPtr (&R)[NR], int nchunks, const int8_t* xq, const float* xd,
                                         float (&acc)[NR], int lane) {
  for (int c0 = 0; c0 < nchunks; c0 += 128) {
    WRaw<QT> w[2][NR];
    load_pair<QT, NR>(w, R, c0, 64, nchunks, lane);
    dot_pair<QT, NR>(w, c0, 64, nchunks, xq, xd, acc, lane);
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) acc[r] = wave_sum(acc[r]);
}

// rows per wave-item: enough independent loads in flight without dropping below
// 2 waves/SIMD (Q6_K carries 4 loads per chunk, F16/F32 8)
template <int QT>
constexpr int rows_per_item() { return (QT == T_Q4_K || QT == T_Q8_0 || QT == T_Q5_K) ? 4 : 2; }

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// pick acc[lane] for lanes < NR (every lane holds every reduced row)
template <int NR>
__device__ __forceinline__ float pick(const float (&acc)[NR], int lane) {
  float v = acc[0];
#pragma unroll
  for (int r = 1; r < NR; ++r) v = lane == r ? acc[r] : v;
  return v;
}

// K split over `wk` waves of the block (wk = 1, 2 or 4, chosen on the host so
// every wave has >= one full 64-chunk pass): a block holds 4/wk row groups;
// the wk partial sums of a group meet in LDS.
template <int EPI, int NR>
__device__ __forceinline__ void item_rows(const GemvArgs& a, int it, int groups, RowPtr (&R)[NR], int& slot, int& f0) {
  constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
  slot = it / groups;
  f0 = (it - slot * groups) * NF;
  const uint8_t* base = a.w.base;
  if (a.expert_ids) base += (size_t)a.expert_ids[slot] * a.w.expert_stride;
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    if constexpr (EPI == EPI_SWIGLU) {
      const int f = f0 + r;
      const unsigned gr = (unsigned)((f >> 5) * 64 + (f & 31));
      R[r] = row_ptr(base, a.w.P, gr);
      R[NF + r] = row_ptr(base, a.w.P, gr + 32);
    } else {
      R[r] = row_ptr(base, a.w.P, (unsigned)min(f0 + r, a.n_out - 1));
    }
  }
}

// One wave = one row group of NR rows (NF outputs); 4 waves per block; grid
// capped at 4 blocks/CU and strided over row groups. Measured on MI355X this
// simple form (115 VGPRs for Q4_K, 4 waves/SIMD) beat variants that prefetch
// across the prologue or split K across waves (170-200 VGPRs): occupancy wins.
template <int QT, int EPI, int NR, bool NORM>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs a, int /*unused*/) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = a.w.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + K);
  float* red = xd + (K >> 5);
  quantize_x<NORM>(a.x, a.norm_w, a.eps, K, xq, xd, red);
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int nchunks = K >> 5;
  constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
  const int groups = (a.n_out + NF - 1) / NF;
  const int total = groups * a.n_slots;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    RowPtr R[NR];
    int slot, f0;
    item_rows<EPI, NR>(a, item, groups, R, slot, f0);
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    dot_rows<QT, NR>(R, nchunks, xq, xd, acc, lane);
    if (lane < NF && f0 + lane < a.n_out) {
      float* o = a.out + (size_t)slot * a.out_slot_stride + f0 + lane;
      if constexpr (EPI == EPI_SWIGLU) {
        float g = acc[0], u = acc[NF];
#pragma unroll
        for (int r = 1; r < NF; ++r) {
          g = lane == r ? acc[r] : g;
          u = lane == r ? acc[NF + r] : u;
        }
        *o = silu(g) * u;
      } else {
        const float v = pick<NR>(acc, lane);
        if constexpr (EPI == EPI_STORE) *o = a.resid ? v + a.resid[f0 + lane] : v;
        else *o += v;
      }
    }
  }
}

QMat make_qmat(const void* base, int type, int rows, int K, size_t expert_stride) {
  QMat m;
  m.base = static_cast<const uint8_t*>(base);
  m.type = type;
  m.rows = rows;
  m.K = K;
  m.P = planes_of(type, rows, K);
  m.expert_stride = expert_stride;
  return m;
}

static inline int grid_for(int items, int per_block = 4) {
  int b = (items + per_block - 1) / per_block;
  return b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b);
}


template <int QT, int EPI>
static void launch_gemv(const GemvArgs& a, hipStream_t s) {
  constexpr int NR = rows_per_item<QT>();
  constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
  const size_t lds = a.w.K + (a.w.K / 32) * 4 + 32 + 4 * NR * 4 + 64;
  const int items = (a.n_out + NF - 1) / NF * a.n_slots;
  dim3 grid(grid_for(items)), block(256);
  const int wk = 1;
  if (a.norm_w) hipLaunchKernelGGL((gemv_kernel<QT, EPI, NR, true>), grid, block, lds, s, a, wk);
  else hipLaunchKernelGGL((gemv_kernel<QT, EPI, NR, false>), grid, block, lds, s, a, wk);
}

template <int QT>
static void gemv_t(const GemvArgs& a, int epi, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: launch_gemv<QT, EPI_STORE>(a, s); break;
    case EPI_ADD: launch_gemv<QT, EPI_ADD>(a, s); break;
    case EPI_SWIGLU: launch_gemv<QT, EPI_SWIGLU>(a, s); break;
    default: throw std::runtime_error("gemv: bad epilogue");
  }
}

void gemv(const GemvArgs& a, int epi, hipStream_t s) {
  if (epi == EPI_SWIGLU && (a.n_out % 32)) throw std::runtime_error("gemv: swiglu features must be a multiple of 32");
  if (a.w.K % 32) throw std::runtime_error("gemv: K must be a multiple of 32");
  if (a.n_out <= 0) return;
  switch (a.w.type) {
    case T_Q4_K: gemv_t<T_Q4_K>(a, epi, s); break;
    case T_Q5_K: gemv_t<T_Q5_K>(a, epi, s); break;
    case T_Q6_K: gemv_t<T_Q6_K>(a, epi, s); break;
    case T_Q8_0: gemv_t<T_Q8_0>(a, epi, s); break;
    case T_F16: gemv_t<T_F16>(a, epi, s); break;
    case T_F32: gemv_t<T_F32>(a, epi, s); break;
    default: throw std::runtime_error("gemv: unsupported weight type");
  }
}

// ------------------------------------------------------------------ QKV + RoPE + KV append
// One launch covers a run of Q/K/V segments that share a quant type (Q4_K_M:
// usually Q+K together, V separately when it is Q6_K). Items are 4 rows = two
// RoPE pairs, so the rotation happens between lanes (2j, 2j+1) after the reduce.
struct QkvSeg {
  const uint8_t* base;
  Planes P;
  int rows;
  int kind;  // 0 = Q, 1 = K, 2 = V
};
struct QkvLaunch {
  QkvSeg seg[3];
  int nseg;
  int K;
  const float* x;
  const float* norm_w;
  float eps;
  float* q_out;
  __half* k_cache;
  __half* v_cache;
  int n_ctx, head_dim;
  const int* pos;
  const float2* rope;
};

// One launch per run of Q/K/V segments sharing a quant type (measured: mixing
// two types in one kernel raised VGPRs past 200 and ran slower than 2 launches).
template <int QT>
__global__ __launch_bounds__(256) void gemv_qkv_kernel(QkvLaunch a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NR = rows_per_item<QT>();
  const int K = a.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + K);
  float* red = xd + (K >> 5);
  if (a.norm_w) quantize_x<true>(a.x, a.norm_w, a.eps, K, xq, xd, red);
  else quantize_x<false>(a.x, nullptr, a.eps, K, xq, xd, red);
  const int wave = wave_id(), lane = threadIdx.x & 63;
  int total = 0;
  for (int i = 0; i < a.nseg; ++i) total += a.seg[i].rows / NR;
  const int nchunks = K >> 5;
  const int hd = a.head_dim;
  const int pos = *a.pos;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    int it = item, si = 0;
    while (si < a.nseg - 1 && it >= a.seg[si].rows / NR) { it -= a.seg[si].rows / NR; ++si; }
    const QkvSeg& sg = a.seg[si];
    const int r0 = it * NR;
    RowPtr R[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) R[r] = row_ptr(sg.base, sg.P, (unsigned)(r0 + r));
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    dot_rows<QT, NR>(R, nchunks, xq, xd, acc, lane);
    float v = pick<NR>(acc, lane);
    const float partner = __shfl_xor(v, 1);
    if (lane < NR) {
      const int r = r0 + lane;
      const int dd = r % hd;
      if (sg.kind < 2) {
        const float2 cs = a.rope[(size_t)pos * (hd >> 1) + (dd >> 1)];
        v = (lane & 1) ? partner * cs.y + v * cs.x : v * cs.x - partner * cs.y;
      }
      if (sg.kind == 0) {
        a.q_out[r] = v;
      } else {
        __half* c = (sg.kind == 1 ? a.k_cache : a.v_cache) + ((size_t)(r / hd) * a.n_ctx + pos) * hd + dd;
        *c = __float2half(v);
      }
    }
  }
}

void gemv_qkv(const QkvArgs& a, hipStream_t s) {
  const int K = a.wq.K;
  if (K % 32 || a.wk.K != K || a.wv.K != K) throw std::runtime_error("gemv_qkv: K mismatch");
  if (a.wq.rows % 4 || a.wk.rows % 4) throw std::runtime_error("gemv_qkv: rows must be multiples of 4");
  const QMat* m[3] = {&a.wq, &a.wk, &a.wv};
  const size_t lds = K + (K / 32) * 4 + 64;
  for (int i = 0; i < 3;) {
    QkvLaunch L{};
    L.K = K; L.x = a.x; L.norm_w = a.norm_w; L.eps = a.eps; L.q_out = a.q_out; L.k_cache = a.k_cache;
    L.v_cache = a.v_cache; L.n_ctx = a.n_ctx; L.head_dim = a.head_dim; L.pos = a.pos; L.rope = a.rope;
    const int t = m[i]->type;
    int items = 0;
    while (i < 3 && m[i]->type == t) {
      L.seg[L.nseg] = QkvSeg{m[i]->base, m[i]->P, m[i]->rows, i};
      items += m[i]->rows / (t == T_Q4_K || t == T_Q5_K || t == T_Q8_0 ? 4 : 2);
      ++L.nseg;
      ++i;
    }
    dim3 grid(grid_for(items)), block(256);
    switch (t) {
      case T_Q4_K: hipLaunchKernelGGL(gemv_qkv_kernel<T_Q4_K>, grid, block, lds, s, L); break;
      case T_Q5_K: hipLaunchKernelGGL(gemv_qkv_kernel<T_Q5_K>, grid, block, lds, s, L); break;
      case T_Q6_K: hipLaunchKernelGGL(gemv_qkv_kernel<T_Q6_K>, grid, block, lds, s, L); break;
      case T_Q8_0: hipLaunchKernelGGL(gemv_qkv_kernel<T_Q8_0>, grid, block, lds, s, L); break;
      case T_F16: hipLaunchKernelGGL(gemv_qkv_kernel<T_F16>, grid, block, lds, s, L); break;
      case T_F32: hipLaunchKernelGGL(gemv_qkv_kernel<T_F32>, grid, block, lds, s, L); break;
      default: throw std::runtime_error("gemv_qkv: unsupported type");
    }
  }
}

// ------------------------------------------------------------------ MoE down projection
template <int QT>
__global__ __launch_bounds__(256) void gemv_moe_down_kernel(MoeDownArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NR = 2;
  const int K = a.w.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + (size_t)a.n_slots * K);
  float* red = xd + (size_t)a.n_slots * (K >> 5);
  for (int s = 0; s < a.n_slots; ++s)
    quantize_x<false>(a.h + (size_t)s * K, nullptr, 0.f, K, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), red);
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int nchunks = K >> 5;
  const int total = (a.w.rows + NR - 1) / NR;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    const int r0 = item * NR;
    float tot[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) tot[r] = 0.f;
    for (int s = 0; s < a.n_slots; ++s) {
      const uint8_t* base = a.w.base + (size_t)a.expert_ids[s] * a.w.expert_stride;
      RowPtr R[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) R[r] = row_ptr(base, a.w.P, (unsigned)min(r0 + r, a.w.rows - 1));
      float acc[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[r] = 0.f;
      dot_rows<QT, NR>(R, nchunks, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), acc, lane);
      const float ws = a.expert_w[s];
#pragma unroll
      for (int r = 0; r < NR; ++r) tot[r] += ws * acc[r];
    }
    if (lane < NR && r0 + lane < a.w.rows) a.out[r0 + lane] += pick<NR>(tot, lane);
  }
}

void gemv_moe_down(const MoeDownArgs& a, hipStream_t s) {
  const int K = a.w.K;
  const size_t lds = (size_t)a.n_slots * (K + (K / 32) * 4) + 64;
  dim3 grid(grid_for((a.w.rows + 1) / 2)), block(256);
  switch (a.w.type) {
    case T_Q4_K: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q4_K>, grid, block, lds, s, a); break;
    case T_Q5_K: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q5_K>, grid, block, lds, s, a); break;
    case T_Q6_K: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q6_K>, grid, block, lds, s, a); break;
    case T_Q8_0: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q8_0>, grid, block, lds, s, a); break;
    case T_F16: hipLaunchKernelGGL(gemv_moe_down_kernel<T_F16>, grid, block, lds, s, a); break;
    case T_F32: hipLaunchKernelGGL(gemv_moe_down_kernel<T_F32>, grid, block, lds, s, a); break;
    default: throw std::runtime_error("moe_down: unsupported type");
  }
}

// ------------------------------------------------------------------ MoE router (one wave)
__global__ void moe_route_kernel(const float* logits, int E, int k, int* ids, float* w) {
  const int lane = threadIdx.x;
  float v = lane < E ? logits[lane] : -INFINITY;
  const float m = wave_max(v);
  float p = lane < E ? __expf(v - m) : 0.f;
  const float sum = wave_sum(p);
  p /= sum;
  float sel_sum = 0.f, my_w = 0.f;
  int my_id = 0;
  float taken = lane < E ? p : -1.f;
  for (int j = 0; j < k; ++j) {
    // arg-max with the lowest index on ties (matches a stable descending sort)
    float best = taken;
    int bi = lane;
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == j) { my_id = bi; my_w = best; }
    sel_sum += best;
    if (lane == bi) taken = -1.f;
  }
  if (lane < k) {
    ids[lane] = my_id;
    w[lane] = my_w / sel_sum;
  }
}

void moe_route(const float* logits, int n_expert, int k, int* ids, float* w, hipStream_t s) {
  if (n_expert > 64 || k > n_expert) throw std::runtime_error("moe_route: n_expert must be <= 64");
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(64), 0, s, logits, n_expert, k, ids, w);
}

// ------------------------------------------------------------------ MoE prefill helpers
__global__ void moe_route_dense_kernel(const float* logits, int E, int k, float* wd) {
  const int t = blockIdx.x, lane = threadIdx.x;
  const float* lg = logits + (size_t)t * E;
  float v = lane < E ? lg[lane] : -INFINITY;
  const float m = wave_max(v);
  float p = lane < E ? __expf(v - m) : 0.f;
  p /= wave_sum(p);
  float taken = lane < E ? p : -1.f, sel = 0.f, mine = 0.f;
  for (int j = 0; j < k; ++j) {
    float best = taken;
    int bi = lane;
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    sel += best;
    if (lane == bi) { mine = best; taken = -1.f; }
  }
  if (lane < E) wd[(size_t)t * E + lane] = mine / sel;
}

void moe_route_dense(const float* logits, int T, int n_expert, int k, float* w_dense, hipStream_t s) {
  if (T <= 0) return;
  if (n_expert > 64) throw std::runtime_error("moe_route_dense: n_expert must be <= 64");
  hipLaunchKernelGGL(moe_route_dense_kernel, dim3(T), dim3(64), 0, s, logits, n_expert, k, w_dense);
}

__global__ void axpy_rows_kernel(float* acc, const float* y, const float* wd, int e, int E, int d) {
  const int t = blockIdx.x;
  const float w = wd[(size_t)t * E + e];
  if (w == 0.f) return;
  for (int i = threadIdx.x; i < d; i += blockDim.x) acc[(size_t)t * d + i] += w * y[(size_t)t * d + i];
}

void axpy_rows(float* acc, const float* y, const float* w_dense, int e, int E, int T, int d, hipStream_t s) {
  if (T <= 0) return;
  hipLaunchKernelGGL(axpy_rows_kernel, dim3(T), dim3(256), 0, s, acc, y, w_dense, e, E, d);
}

}  // namespace lfk
