// MoE prefill routing for grouped expert GEMMs (Mixtral).
//
// Upstream ggml-cuda's mul_mat_id copies the expert ids to the host, syncs, and
// runs one matmul per expert over gathered rows. Here everything stays on the
// device: one routing kernel builds, per expert, the list of (token, weight)
// rows routed to it (ascending token order: deterministic), their offsets in a
// gathered buffer and each token's k positions in it. The expert GEMMs then
// read their row count and offset from device memory (GemmArgs::rows_dev), so
// only the rows routed to an expert are multiplied - top-2 of 8 experts costs
// 2/8 of the dense loop - and no host round trip is needed.
#include <algorithm>

#include "gemv_dev.h"
#include "moe_route_dev.h"

namespace lfk {

// One block. sel/selw: [T*k] scratch; cnt_off: [E+1] (offsets, off[E] = T*k);
// tok/gw: [T*k] gathered row -> token / routing weight; pos: [T*k] token slot -> row.
__global__ __launch_bounds__(256) void moe_route_group_kernel(const float* __restrict__ logits, int T, int E, int k,
                                                              int* sel, float* selw, int* cnt_off, int* tok,
                                                              float* gw, int* pos) {
  __shared__ int s_cnt[65];
  // A: per token softmax + top-k (lowest index on ties), renormalised over the selected
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    const float* lg = logits + (size_t)t * E;
    float m = -INFINITY;
    for (int e = 0; e < E; ++e) m = fmaxf(m, lg[e]);
    float p[64];
    float sum = 0.f;
    for (int e = 0; e < E; ++e) { p[e] = __expf(lg[e] - m); sum += p[e]; }
    float selsum = 0.f;
    unsigned long long taken = 0ull;
    for (int j = 0; j < k; ++j) {
      int bi = -1;
      float best = -1.f;
      for (int e = 0; e < E; ++e)
        if (!((taken >> e) & 1ull) && p[e] > best) { best = p[e]; bi = e; }
      taken |= 1ull << bi;
      sel[t * k + j] = bi;
      selw[t * k + j] = best / sum;
      selsum += best / sum;
    }
    for (int j = 0; j < k; ++j) selw[t * k + j] /= selsum;
  }
  __syncthreads();
  // B: per-expert counts, C: offsets
  if (threadIdx.x < E) {
    int c = 0;
    for (int i = 0; i < T * k; ++i) c += sel[i] == (int)threadIdx.x;
    s_cnt[threadIdx.x] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int o = 0;
    for (int e = 0; e < E; ++e) { const int c = s_cnt[e]; s_cnt[e] = o; cnt_off[e] = o; o += c; }
    cnt_off[E] = o;
  }
  __syncthreads();
  // D: fill each expert's rows in ascending token order
  if (threadIdx.x < E) {
    int p = s_cnt[threadIdx.x];
    for (int i = 0; i < T * k; ++i)
      if (sel[i] == (int)threadIdx.x) {
        tok[p] = i / k;
        gw[p] = selw[i];
        pos[i] = p;
        ++p;
      }
  }
}

void moe_route_group(const float* logits, int T, int n_expert, int k, int* sel, float* selw, int* cnt_off, int* tok,
                     float* gw, int* pos, hipStream_t s) {
  if (T <= 0) return;
  if (n_expert > 64 || k > n_expert) throw std::runtime_error("moe_route_group: n_expert must be <= 64");
  hipLaunchKernelGGL(moe_route_group_kernel, dim3(1), dim3(256), 0, s, logits, T, n_expert, k, sel, selw, cnt_off,
                     tok, gw, pos);
}

// dst[r][:] = src[tok[r]][:] (bf16 rows, 16 B per thread)
__global__ void gather_rows_bf16_kernel(const __hip_bfloat16* __restrict__ src, const int* __restrict__ tok, int d,
                                        __hip_bfloat16* __restrict__ dst) {
  const int r = blockIdx.x;
  const uint4* s = reinterpret_cast<const uint4*>(src + (size_t)tok[r] * d);
  uint4* o = reinterpret_cast<uint4*>(dst + (size_t)r * d);
  for (int i = threadIdx.x; i < d / 8; i += blockDim.x) o[i] = s[i];
}

void gather_rows_bf16(const __hip_bfloat16* src, const int* tok, int n_rows, int d, __hip_bfloat16* dst,
                      hipStream_t s) {
  if (n_rows <= 0) return;
  if (d % 8) throw std::runtime_error("gather_rows_bf16: d must be a multiple of 8");
  hipLaunchKernelGGL(gather_rows_bf16_kernel, dim3(n_rows), dim3(256), 0, s, src, tok, d, dst);
}

// acc[t][:] += sum_j gw[pos[t*k+j]] * y[pos[t*k+j]][:]   (fixed slot order: deterministic)
__global__ void moe_scatter_add_kernel(float* __restrict__ acc, const float* __restrict__ y,
                                       const int* __restrict__ pos, const float* __restrict__ gw, int k, int d) {
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    float v = 0.f;
    for (int j = 0; j < k; ++j) {
      const int r = pos[t * k + j];
      v += gw[r] * y[(size_t)r * d + i];
    }
    acc[(size_t)t * d + i] += v;
  }
}

void moe_scatter_add(float* acc, const float* y, const int* pos, const float* gw, int T, int k, int d,
                     hipStream_t s) {
  if (T <= 0) return;
  hipLaunchKernelGGL(moe_scatter_add_kernel, dim3(T), dim3(256), 0, s, acc, y, pos, gw, k, d);
}

// ------------------------------------------------------------------ decode: fused router
// logits = W_r (F32 [E][d]) . (RMSNorm(x) * w_norm), softmax over E, top-k, renormalise.
// One block of 1024 threads: replaces the router GEMV launch + the routing launch
// (two kernel boundaries per MoE layer). The router stays in f32 end to end.
static constexpr int kRouterMaxE = 16;

// (batched rows: block b routes row b - x + b * ldx - and writes the dense weight row
// wd + b * ld_dense instead of ids / wout)
template <int EM>
__global__ __launch_bounds__(1024) void moe_router_fused_kernel(const float* __restrict__ x, const float* __restrict__ nw,
                                                                float eps, const float* __restrict__ W, int d, int E,
                                                                int k, float* logits, int* ids, float* wout, int ldx,
                                                                float* wd, int ld_dense) {
  __shared__ float red[16][EM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  x += (size_t)blockIdx.x * ldx;
  float ss = 0.f, acc[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = 0.f;
  for (int i = tid * 4; i < d; i += 4096) {
    const float4 xv = *reinterpret_cast<const float4*>(x + i);
    const float4 wv = *reinterpret_cast<const float4*>(nw + i);
    ss += xv.x * xv.x + xv.y * xv.y + xv.z * xv.z + xv.w * xv.w;
    const float4 n = make_float4(xv.x * wv.x, xv.y * wv.y, xv.z * wv.z, xv.w * wv.w);
    // every row load unconditional (clamped row, result masked): a load under a
    // runtime `e < E` branch makes hipcc drain vmcnt per row (E dependent round trips)
    float4 r[EM];
#pragma unroll
    for (int e = 0; e < EM; ++e) r[e] = *reinterpret_cast<const float4*>(W + (size_t)min(e, E - 1) * d + i);
#pragma unroll
    for (int e = 0; e < EM; ++e)
      acc[e] += e < E ? n.x * r[e].x + n.y * r[e].y + n.z * r[e].z + n.w * r[e].w : 0.f;
  }
  ss = wave_sum_fast(ss);
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = e < E ? wave_sum_fast(acc[e]) : 0.f;
  if (lane == 0) {
    red[wave][EM] = ss;
#pragma unroll
    for (int e = 0; e < EM; ++e) red[wave][e] = acc[e];
  }
  __syncthreads();
  if (wave != 0) return;
  // softmax + top-k (lowest index on ties) + renormalise (moe_route_dev.h, shared with the
  // routed SwiGLU GEMV)
  int my_id;
  float my_w, sel_sum, v;
  moe_route_finish<EM, 16>(red, E, k, d, eps, lane, my_id, my_w, sel_sum, v);
  if (logits && lane < E) logits[lane] = v;
  if (wd) {
    // dense row: lane e < E finds its own weight among the k picks (lanes 0..k-1 hold them)
    float* row = wd + (size_t)blockIdx.x * ld_dense;
    float mine = 0.f;
    for (int j = 0; j < k; ++j) {
      const int id = __shfl(my_id, j);
      const float w = __shfl(my_w, j);
      if (id == lane) mine = w / sel_sum;
    }
    if (lane < E) row[lane] = mine;
    return;
  }
  if (lane < k) {
    ids[lane] = my_id;
    wout[lane] = my_w / sel_sum;
  }
}

bool moe_router_fused_ok(int router_type, int E, int d) {
  return router_type == T_F32 && E <= kRouterMaxE && E >= 1 && d % 4 == 0;
}

void moe_router_fused(const float* x, const float* nw, float eps, const float* W, int d, int E, int k, float* logits,
                      int* ids, float* w, hipStream_t s) {
  if (E > kRouterMaxE || k > E || d % 4) throw std::runtime_error("moe_router_fused: unsupported shape");
  if (E <= 8)  // rows padded to EM are loaded (clamped) and masked: size EM to the expert count
    hipLaunchKernelGGL(moe_router_fused_kernel<8>, dim3(1), dim3(1024), 0, s, x, nw, eps, W, d, E, k, logits, ids, w,
                       0, nullptr, 0);
  else
    hipLaunchKernelGGL(moe_router_fused_kernel<16>, dim3(1), dim3(1024), 0, s, x, nw, eps, W, d, E, k, logits, ids, w,
                       0, nullptr, 0);
}

void moe_router_rows(const float* x, int ldx, int B, const float* nw, float eps, const float* W, int d, int E, int k,
                     float* wd, int ld, hipStream_t s) {
  if (E > kRouterMaxE || k > E || d % 4 || B < 1 || ld < E || ldx % 4) throw std::runtime_error("moe_router_rows: unsupported shape");
  if (E <= 8)
    hipLaunchKernelGGL(moe_router_fused_kernel<8>, dim3(B), dim3(1024), 0, s, x, nw, eps, W, d, E, k, nullptr, nullptr,
                       nullptr, ldx, wd, ld);
  else
    hipLaunchKernelGGL(moe_router_fused_kernel<16>, dim3(B), dim3(1024), 0, s, x, nw, eps, W, d, E, k, nullptr, nullptr,
                       nullptr, ldx, wd, ld);
}

// ------------------------------------------------------------------ decode: grouped down, split-K
// out[r] += sum_s w_s * dot(W_{e_s}[r, :], h_s), as the dense down projection's EARLY
// split-K GEMV (gemv.hip): one 1024-thread block per CU (LDS request > half the CU),
// contiguous item ranges, the first weight loads issued before the h prologue's wait.
// Items = (slot, 64-chunk part, 4-row group), part-major; the two slots' h vectors are
// quantised as ONE vector of n_slots*K (slot boundaries fall on q8 blocks).
static constexpr size_t kMoeOnePerCuLds = 80 * 1024 + 256;

template <int QT>
__global__ __launch_bounds__(1024) void moe_down_splitk_kernel(MoeDownArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NR = 4, WPB = 16;
  const int K = a.w.K, S = a.n_slots, nch = K >> 5;
  const int kps = (nch + 63) / 64;
  const int RG = (a.w.rows + NR - 1) / NR;
  const int total = RG * S * kps;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + (size_t)S * K);
  float* red = xd + (size_t)S * (K >> 5);
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int per = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = min(total, (int)blockIdx.x * per), i1 = min(total, i0 + per);
  XPrologue<false, 1024> xp;
  xp.load(a.h, nullptr, S * K);
  RowPtr R[NR];
  WStream<QT, NR, 1> ws;
  int item = i0 + wave, s = 0, kpl = 0, rg = 0;
  auto locate = [&](int it) {
    const int p = it / RG;
    rg = it - p * RG;
    s = p / kps;
    kpl = p - s * kps;
    const uint8_t* base = a.w.base + (size_t)a.expert_ids[s] * a.w.expert_stride;
#pragma unroll
    for (int r = 0; r < NR; ++r) R[r] = row_ptr(base, a.w.P, (unsigned)min(rg * NR + r, a.w.rows - 1));
  };
  locate(min(item, total - 1));  // unconditional: no control-flow join before the h wait
  ws.load(R, kpl * 64, nch, lane);
  xp.finish(a.h, nullptr, 0.f, S * K, xq, xd, red);
  while (item < i1) {
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    ws.dot(kpl * 64, nch, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), acc, lane);
    const int cs = s, crg = rg;
    const int next = item + WPB;
    if (next < i1) {
      locate(next);
      ws.load(R, kpl * 64, nch, lane);
    }
    const float wsl = a.expert_w[cs];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] *= wsl;
    const float v = reduce_rows<NR>(acc, lane);
    if (lane < NR && crg * NR + lane < a.w.rows) atomicAdd(a.out + crg * NR + lane, v);
    item = next;
  }
}

bool moe_down_splitk(const MoeDownArgs& a, hipStream_t s) {
  const int K = a.w.K;
  if (K % 256 || a.n_slots < 1 || a.n_slots * (size_t)K > 64 * 1024) return false;
  const size_t lds = std::max((size_t)a.n_slots * (K + (K / 32) * 4) + 128, kMoeOnePerCuLds);
  static int cus = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return c > 0 ? c : 256;
  }();
  switch (a.w.type) {
    case T_Q4_K: hipLaunchKernelGGL(moe_down_splitk_kernel<T_Q4_K>, dim3(cus), dim3(1024), lds, s, a); return true;
    case T_Q5_K: hipLaunchKernelGGL(moe_down_splitk_kernel<T_Q5_K>, dim3(cus), dim3(1024), lds, s, a); return true;
    case T_Q6_K: hipLaunchKernelGGL(moe_down_splitk_kernel<T_Q6_K>, dim3(cus), dim3(1024), lds, s, a); return true;
    case T_Q8_0: hipLaunchKernelGGL(moe_down_splitk_kernel<T_Q8_0>, dim3(cus), dim3(1024), lds, s, a); return true;
    default: return false;  // F16/F32 experts: the per-slot kernel (gemv.hip)
  }
}

}  // namespace lfk
