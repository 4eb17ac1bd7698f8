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

template <int QT, int NR>
__device__ __forceinline__ void dot_rows(const uint8_t* base, const Planes& P, const size_t (&rows)[NR], int nchunks,
                                         const int8_t* xq, const float* xd, float (&acc)[NR], int lane) {
#pragma unroll 2
  for (int c = lane; c < nchunks; c += 64) {
    XChunk X;
    load_x<QT>(X, xq, xd, c);
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] += chunk_dot<QT>(base, P, rows[r], c, X);
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) acc[r] = wave_sum(acc[r]);
}

template <int QT, int EPI, int NR>
__device__ void gemv_body(const GemvArgs& a, const int8_t* xq, const float* xd) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunks = a.w.K >> 5;
  const int groups = (a.n_out + NR - 1) / NR;
  const int total = groups * a.n_slots;
  constexpr int NROW = (EPI == EPI_SWIGLU) ? 2 * NR : NR;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    const int slot = item / groups;
    const int g = item - slot * groups;
    const uint8_t* base = a.w.base;
    if (a.expert_ids) base += (size_t)a.expert_ids[slot] * a.w.expert_stride;
    size_t rows[NROW];
    const int f0 = g * NR;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if constexpr (EPI == EPI_SWIGLU) {
        const int f = f0 + r;
        rows[r] = (size_t)((f >> 5) * 64 + (f & 31));
        rows[NR + r] = rows[r] + 32;
      } else {
        rows[r] = (size_t)min(f0 + r, a.n_out - 1);
      }
    }
    float acc[NROW];
#pragma unroll
    for (int r = 0; r < NROW; ++r) acc[r] = 0.f;
    dot_rows<QT, NROW>(base, a.w.P, rows, nchunks, xq, xd, acc, lane);
    if (lane < NR && f0 + lane < a.n_out) {
      float v = acc[0];
#pragma unroll
      for (int r = 1; r < NR; ++r) if (lane == r) v = acc[r];
      float* o = a.out + (size_t)slot * a.out_slot_stride + f0 + lane;
      if constexpr (EPI == EPI_STORE) {
        *o = a.resid ? v + a.resid[f0 + lane] : v;
      } else if constexpr (EPI == EPI_ADD) {
        *o += v;
      } else {
        float u = acc[NR];
#pragma unroll
        for (int r = 1; r < NR; ++r) if (lane == r) u = acc[NR + r];
        *o = silu(v) * u;
      }
    }
  }
}

template <int EPI, int NR, bool NORM>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = a.w.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + K);
  float* red = xd + (K >> 5);
  quantize_x<NORM>(a.x, a.norm_w, a.eps, K, xq, xd, red);
  LFK_DISPATCH_TYPE(a.w.type, gemv_body<QT, EPI, NR>(a, xq, xd));
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

static inline int grid_for(int items) {
  int b = (items + 3) / 4;
  return b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b);
}

void gemv(const GemvArgs& a, int epi, hipStream_t s) {
  constexpr int NR = 2;
  if (epi == EPI_SWIGLU && (a.n_out % 32)) throw std::runtime_error("gemv: swiglu features must be a multiple of 32");
  if (a.w.K % 32) throw std::runtime_error("gemv: K must be a multiple of 32");
  if (a.n_out <= 0) return;
  const size_t lds = a.w.K + (a.w.K / 32) * 4 + 64;
  const int items = (a.n_out + NR - 1) / NR * a.n_slots;
  dim3 grid(grid_for(items)), block(256);
  const bool norm = a.norm_w != nullptr;
#define LAUNCH(E, N)                                                                         \
  if (norm) hipLaunchKernelGGL((gemv_kernel<E, NR, true>), grid, block, lds, s, a);          \
  else hipLaunchKernelGGL((gemv_kernel<E, NR, false>), grid, block, lds, s, a);
  switch (epi) {
    case EPI_STORE: LAUNCH(EPI_STORE, NR); break;
    case EPI_ADD: LAUNCH(EPI_ADD, NR); break;
    case EPI_SWIGLU: LAUNCH(EPI_SWIGLU, NR); break;
    default: throw std::runtime_error("gemv: bad epilogue");
  }
#undef LAUNCH
}

// ------------------------------------------------------------------ QKV + RoPE + KV append
template <int QT>
__device__ __forceinline__ void qkv_pair(const QMat& w, size_t row, int nchunks, const int8_t* xq, const float* xd,
                                         float& a0, float& a1, int lane) {
  size_t rows[2] = {row, row + 1};
  float acc[2] = {0.f, 0.f};
  dot_rows<QT, 2>(w.base, w.P, rows, nchunks, xq, xd, acc, lane);
  a0 = acc[0];
  a1 = acc[1];
}

__global__ __launch_bounds__(256) void gemv_qkv_kernel(QkvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = a.wq.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + K);
  float* red = xd + (K >> 5);
  if (a.norm_w) quantize_x<true>(a.x, a.norm_w, a.eps, K, xq, xd, red);
  else quantize_x<false>(a.x, nullptr, a.eps, K, xq, xd, red);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nq = a.wq.rows, nkv = a.wk.rows;
  const int total = (nq + 2 * nkv) >> 1;
  const int nchunks = K >> 5;
  const int hd = a.head_dim;
  const int pos = *a.pos;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    int r = item * 2;
    int seg;
    const QMat* w;
    if (r < nq) { seg = 0; w = &a.wq; }
    else if (r < nq + nkv) { seg = 1; r -= nq; w = &a.wk; }
    else { seg = 2; r -= nq + nkv; w = &a.wv; }
    float a0 = 0.f, a1 = 0.f;
    LFK_DISPATCH_TYPE(w->type, qkv_pair<QT>(*w, (size_t)r, nchunks, xq, xd, a0, a1, lane));
    if (lane == 0) {
      const int dd = r % hd;
      float y0 = a0, y1 = a1;
      if (seg < 2) {
        const float2 cs = a.rope[(size_t)pos * (hd >> 1) + (dd >> 1)];
        y0 = a0 * cs.x - a1 * cs.y;
        y1 = a0 * cs.y + a1 * cs.x;
      }
      if (seg == 0) {
        a.q_out[r] = y0;
        a.q_out[r + 1] = y1;
      } else {
        const int kvh = r / hd;
        __half* c = (seg == 1 ? a.k_cache : a.v_cache) + ((size_t)kvh * a.n_ctx + pos) * hd + dd;
        c[0] = __float2half(y0);
        c[1] = __float2half(y1);
      }
    }
  }
}

void gemv_qkv(const QkvArgs& a, hipStream_t s) {
  const int K = a.wq.K;
  if (K % 32 || a.wk.K != K || a.wv.K != K) throw std::runtime_error("gemv_qkv: K mismatch");
  const size_t lds = K + (K / 32) * 4 + 64;
  const int items = (a.wq.rows + 2 * a.wk.rows) / 2;
  hipLaunchKernelGGL(gemv_qkv_kernel, dim3(grid_for(items)), dim3(256), lds, s, a);
}

// ------------------------------------------------------------------ MoE down projection
template <int QT>
__device__ void moe_down_body(const MoeDownArgs& a, const int8_t* xq, const float* xd) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int K = a.w.K, nchunks = K >> 5;
  const int total = a.w.rows >> 1;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    size_t rows[2] = {(size_t)item * 2, (size_t)item * 2 + 1};
    float tot0 = 0.f, tot1 = 0.f;
    for (int s = 0; s < a.n_slots; ++s) {
      const uint8_t* base = a.w.base + (size_t)a.expert_ids[s] * a.w.expert_stride;
      float acc[2] = {0.f, 0.f};
      dot_rows<QT, 2>(base, a.w.P, rows, nchunks, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), acc, lane);
      const float ws = a.expert_w[s];
      tot0 += ws * acc[0];
      tot1 += ws * acc[1];
    }
    if (lane == 0) {
      a.out[rows[0]] += tot0;
      a.out[rows[1]] += tot1;
    }
  }
}

__global__ __launch_bounds__(256) void gemv_moe_down_kernel(MoeDownArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = a.w.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + (size_t)a.n_slots * K);
  float* red = xd + (size_t)a.n_slots * (K >> 5);
  for (int s = 0; s < a.n_slots; ++s)
    quantize_x<false>(a.h + (size_t)s * K, nullptr, 0.f, K, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), red);
  LFK_DISPATCH_TYPE(a.w.type, moe_down_body<QT>(a, xq, xd));
}

void gemv_moe_down(const MoeDownArgs& a, hipStream_t s) {
  const int K = a.w.K;
  const size_t lds = (size_t)a.n_slots * (K + (K / 32) * 4) + 64;
  hipLaunchKernelGGL(gemv_moe_down_kernel, dim3(grid_for(a.w.rows / 2)), dim3(256), lds, s, a);
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
