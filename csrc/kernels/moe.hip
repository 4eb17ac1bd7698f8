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
#include "kernels.h"

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

}  // namespace lfk
