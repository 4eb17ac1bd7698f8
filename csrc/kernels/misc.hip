// Small kernels: embedding gather (on the GPU, not the CPU),
// RMSNorm->bf16 for the prefill GEMMs (K2), prefill RoPE + KV append (K5/K6),
// helpers, and the on-device synthetic weight generator.
#include <algorithm>
#include <hip/hip_bf16.h>

#include "kernels.h"
#include "qdot.h"

namespace lfk {

template <int QT>
__device__ void embed_row(const QMat& e, int token, int t, float* x) {
  // clamped: a token id can only come from the host (validated) or the sampler, but a
  // corrupted id must not turn into an out-of-bounds read that faults the GPU
  const size_t row = (size_t)min(max(token, 0), e.rows - 1);
  const int nq = e.K >> 5;
  for (int q = threadIdx.x; q < nq; q += blockDim.x) {
    float v[32];
    dequant32<QT>(e.base, e.P, row, q, v);
    float4* dst = reinterpret_cast<float4*>(x + (size_t)t * e.K + 32 * q);
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  }
}
template <int QT>
__device__ void embed_body(const QMat& e, const int* tokens, int T, float* x) {
  embed_row<QT>(e, tokens[blockIdx.x], blockIdx.x, x);
}

// side job: zero [zero, zero + zero_n) ints (the decode step's done counters, attn_wo1)
__global__ __launch_bounds__(128) void embed_kernel(QMat e, const int* tokens, int T, float* x, int* zero, int zero_n) {
  for (int i = blockIdx.x * 128 + threadIdx.x; i < zero_n; i += gridDim.x * 128) zero[i] = 0;
  LFK_DISPATCH_TYPE(e.type, embed_body<QT>(e, tokens, T, x));
}

void embed_rows(const QMat& emb, const int* tokens, int T, float* x, hipStream_t s, int* zero, int zero_n) {
  if (T <= 0) return;
  hipLaunchKernelGGL(embed_kernel, dim3(T), dim3(128), 0, s, emb, tokens, T, x, zero, zero ? zero_n : 0);
}

template <bool F16SW>
__global__ __launch_bounds__(256) void rmsnorm_bf16_kernel(const float* x, const float* w, float eps, int d,
                                                          __hip_bfloat16* y, float* zero, int zero_ld) {
  const int t = blockIdx.x, tid = threadIdx.x;
  const float* xr = x + (size_t)t * d;
  __shared__ float red[4];
  float ss = 0.f;
  for (int i = tid * 4; i < d; i += 1024) {
    float4 v = *reinterpret_cast<const float4*>(xr + i);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (zero) {  // the next GEMM's split-K partials meet in this row by atomic add
    float4* zr = reinterpret_cast<float4*>(zero + (size_t)t * zero_ld);
    for (int i = tid; i < zero_ld / 4; i += 256) zr[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float sc = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)d + eps);
  for (int i = tid * 4; i < d; i += 1024) {
    float4 v = *reinterpret_cast<const float4*>(xr + i);
    float4 g = *reinterpret_cast<const float4*>(w + i);
    if constexpr (F16SW) {  // 4-group order (0, 2, 1, 3): the pairs (0, 2) and (1, 3)
      const __half2 p0 = __floats2half2_rn(v.x * sc * g.x, v.z * sc * g.z);
      const __half2 p1 = __floats2half2_rn(v.y * sc * g.y, v.w * sc * g.w);
      *reinterpret_cast<uint2*>(y + (size_t)t * d + i) =
          make_uint2(__builtin_bit_cast(unsigned, p0), __builtin_bit_cast(unsigned, p1));
    } else {
      *reinterpret_cast<uint2*>(y + (size_t)t * d + i) =
          make_uint2(pk_bf16_pair(v.x * sc * g.x, v.y * sc * g.y), pk_bf16_pair(v.z * sc * g.z, v.w * sc * g.w));
    }
  }
}

void rmsnorm_bf16(const float* x, const float* w, float eps, int T, int d, __hip_bfloat16* y, hipStream_t s,
                  float* zero, int zero_ld, bool f16sw) {
  if (T <= 0) return;
  if (zero && (zero_ld % 4 || reinterpret_cast<uintptr_t>(zero) % 16))
    throw std::runtime_error("rmsnorm_bf16: zeroed rows must be float4 aligned");
  if (f16sw) hipLaunchKernelGGL(rmsnorm_bf16_kernel<true>, dim3(T), dim3(256), 0, s, x, w, eps, d, y, zero, zero_ld);
  else hipLaunchKernelGGL(rmsnorm_bf16_kernel<false>, dim3(T), dim3(256), 0, s, x, w, eps, d, y, zero, zero_ld);
}

__global__ void to_bf16_kernel(const float* x, int n, __hip_bfloat16* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = __float2bfloat16(x[i]);
}

void to_bf16(const float* x, int n, __hip_bfloat16* y, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(to_bf16_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, n, y);
}

__global__ __launch_bounds__(256) void rope_kv_prefill_kernel(const float* qkv, int pos0, int n_q, int n_kv, int hd,
                                                              int n_ctx, const float2* rope, float* q_out,
                                                              __half* kc, __half* vc, const int* pos_arr,
                                                              const int* slot_arr, size_t slot_stride) {
  const int t = blockIdx.x;
  const int pos = pos_arr ? min(max(pos_arr[t], 0), n_ctx - 1) : pos0 + t;
  if (slot_arr) {
    kc += (size_t)slot_arr[t] * slot_stride;
    vc += (size_t)slot_arr[t] * slot_stride;
  }
  const int ncol = n_q + 2 * n_kv;
  const float* row = qkv + (size_t)t * ncol;
  for (int p = threadIdx.x; p < ncol / 2; p += blockDim.x) {
    int c = 2 * p;
    float a0 = row[c], a1 = row[c + 1];
    if (c < n_q + n_kv) {
      const int dd = (c < n_q ? c : c - n_q) % hd;
      const float2 cs = rope[(size_t)pos * (hd >> 1) + (dd >> 1)];
      const float y0 = a0 * cs.x - a1 * cs.y, y1 = a0 * cs.y + a1 * cs.x;
      a0 = y0;
      a1 = y1;
    }
    if (c < n_q) {
      q_out[(size_t)t * n_q + c] = a0;
      q_out[(size_t)t * n_q + c + 1] = a1;
    } else {
      const bool isk = c < n_q + n_kv;
      const int r = isk ? c - n_q : c - n_q - n_kv;
      const int kvh = r / hd, dd = r % hd;
      __half* dst = (isk ? kc : vc) + ((size_t)kvh * n_ctx + pos) * hd + dd;
      dst[0] = __float2half(a0);
      dst[1] = __float2half(a1);
    }
  }
}

void rope_kv_prefill(const float* qkv, int T, int pos0, int n_q, int n_kv, int head_dim, int n_ctx, const float2* rope,
                     float* q_out, __half* k_cache, __half* v_cache, hipStream_t s, const int* pos_arr,
                     const int* slot_arr, size_t slot_stride) {
  if (T <= 0) return;
  if ((pos_arr == nullptr) != (slot_arr == nullptr)) throw std::runtime_error("rope_kv_prefill: pos/slot arrays");
  hipLaunchKernelGGL(rope_kv_prefill_kernel, dim3(T), dim3(256), 0, s, qkv, pos0, n_q, n_kv, head_dim, n_ctx, rope,
                     q_out, k_cache, v_cache, pos_arr, slot_arr, slot_stride);
}

__global__ void batch_gather_kernel(const int* slots, int B, const int* state, int* tok, int* pos, int* zero,
                                    int zero_n, int zero_stride) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    const int* st = state + (size_t)slots[b] * S_NSTATE;
    tok[b] = st[S_TOKEN];
    pos[b] = st[S_POS];
  }
  if (b < zero_n) zero[(size_t)b * zero_stride] = 0;
}
// (+ zero zero[i * zero_stride], i < zero_n: the step's in-launch chain counters)
void batch_gather(const int* slots, int B, const int* state, int* tok, int* pos, hipStream_t s, int* zero,
                  int zero_n, int zero_stride) {
  if (B <= 0) return;
  const int n = std::max(B, zero ? zero_n : 0);
  hipLaunchKernelGGL(batch_gather_kernel, dim3((n + 63) / 64), dim3(64), 0, s, slots, B, state, tok, pos, zero,
                     zero ? zero_n : 0, zero_stride);
}

// batched decode step head: block b gathers row b's token / position from its slot's state and
// embeds that token (one launch instead of batch_gather + embed_rows)
__global__ __launch_bounds__(128) void batch_embed_kernel(QMat e, const int* slots, const int* state, int* tok, int* pos,
                                                          float* x, int* zero, int zero_n, int zero_stride) {
  const int b = blockIdx.x;
  for (int i = b * 128 + threadIdx.x; i < zero_n; i += gridDim.x * 128) zero[(size_t)i * zero_stride] = 0;
  const int* st = state + (size_t)slots[b] * S_NSTATE;
  const int token = st[S_TOKEN];
  if (threadIdx.x == 0) {
    tok[b] = token;
    pos[b] = st[S_POS];
  }
  LFK_DISPATCH_TYPE(e.type, embed_row<QT>(e, token, b, x));
}
void batch_gather_embed(const int* slots, int B, const int* state, int* tok, int* pos, const QMat& emb, float* x,
                        hipStream_t s, int* zero, int zero_n, int zero_stride) {
  if (B <= 0) return;
  hipLaunchKernelGGL(batch_embed_kernel, dim3(B), dim3(128), 0, s, emb, slots, state, tok, pos, x, zero,
                     zero ? zero_n : 0, zero_stride);
}

__global__ void add_inplace_kernel(float* x, const float* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += y[i];
}
void add_inplace(float* x, const float* y, int n, hipStream_t s) {
  hipLaunchKernelGGL(add_inplace_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, y, n);
}

__global__ void set_i32_kernel(int* p, int v) { *p = v; }
void set_i32(int* p, int v, hipStream_t s) { hipLaunchKernelGGL(set_i32_kernel, dim3(1), dim3(1), 0, s, p, v); }

// ---------------------------------------------------------------- synthetic weights on device
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_bytes_kernel(uint32_t* p, size_t nwords, unsigned long long seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwords; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)mix64(seed ^ (i * 0xD1B54A32D192ED03ull));
}

__device__ __forceinline__ float u01(unsigned long long h) { return (float)(h >> 40) * (1.f / 16777216.f); }

// Overwrite the scale fields of each block with finite values matching gguf/quants.py:random_blocks.
__global__ void fix_scales_kernel(uint8_t* base, int type, size_t nblocks, Planes P, float std, unsigned long long seed) {
  for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < nblocks; b += (size_t)gridDim.x * blockDim.x) {
    const float jit = 0.5f + u01(mix64(seed * 31 + b));
    if (type == T_Q4_K || type == T_Q5_K) {
      const float nmax = type == T_Q4_K ? 15.f : 31.f;
      const float var_sq = (63.f * 127.f / 6.f) * (nmax * (2.f * nmax + 1.f) / 6.f) - (31.5f * nmax / 2.f) * (31.5f * nmax / 2.f);
      const float var = var_sq + (nmax / 2.f) * (nmax / 2.f) * (64.f * 64.f - 1.f) / 12.f;
      const float d = std / sqrtf(var) * jit;
      // meta record b (16 B): d, dmin
      uint8_t* meta = base + (type == T_Q4_K ? P.p1 : P.p2) + 16 * b;
      reinterpret_cast<__half*>(meta)[0] = __float2half(d);
      reinterpret_cast<__half*>(meta)[1] = __float2half(d * nmax * 0.5f);
    } else if (type == T_Q6_K) {
      reinterpret_cast<__half*>(base + P.p3)[b] = __float2half(std / (73.9f * 18.5f) * jit);
    } else if (type == T_Q8_0) {
      reinterpret_cast<__half*>(base + P.p1)[b] = __float2half(std / 73.9f * jit);
    } else if (type == T_F32) {
      // uniform in [-sqrt(3) std, sqrt(3) std]
      const float u = u01(mix64(seed ^ (b * 0x9E37ull)));
      reinterpret_cast<float*>(base)[b] = (2.f * u - 1.f) * 1.7320508f * std;
    } else if (type == T_F16) {
      const float u = u01(mix64(seed ^ (b * 0x9E37ull)));
      reinterpret_cast<__half*>(base)[b] = __float2half((2.f * u - 1.f) * 1.7320508f * std);
    }
  }
}

void fill_random_planar(uint8_t* base, int type, size_t rows, size_t K, float std, unsigned long long seed,
                        hipStream_t s) {
  const size_t bytes = qbytes(type, rows, K);
  const Planes P = planes_of(type, rows, K);
  hipLaunchKernelGGL(fill_bytes_kernel, dim3(2048), dim3(256), 0, s, reinterpret_cast<uint32_t*>(base), bytes / 4, seed);
  size_t nblocks;
  if (type == T_Q4_K || type == T_Q5_K || type == T_Q6_K) nblocks = rows * (K / 256);
  else if (type == T_Q8_0) nblocks = rows * (K / 32);
  else nblocks = rows * K;
  hipLaunchKernelGGL(fix_scales_kernel, dim3(2048), dim3(256), 0, s, base, type, nblocks, P, std, seed + 1);
}

}  // namespace lfk

namespace lfk {
// Clock probe (microbenchmarks): a dependent FMA chain timed in shader cycles
// (clock64) and in constant-rate wall ticks (wall_clock64, 100 MHz), so the
// ratio gives the shader clock the GPU actually ran at.
__global__ void clock_probe_kernel(long long* out, int iters) {
  const long long w0 = wall_clock64(), c0 = clock64();
  float x = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) x = fmaf(x, 0.999f, 0.5f);
  const long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
    out[2] = (long long)x;
  }
}
void clock_probe(long long* out, int iters, hipStream_t s) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, out, iters);
}
}  // namespace lfk

namespace lfk {
// ---------------------------------------------------------------- launch-shape probe (microbenchmarks)
// A trivial kernel of the given geometry: every thread spins `iters` dependent
// FMAs, one lane per block writes. Timing a graph chain of these separates the
// per-launch cost of a workgroup shape (256 vs 1024 threads, LDS request) from
// any real kernel body.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void launch_probe_kernel(float* out, int iters) {
  extern __shared__ float lds_probe[];
  float v = (float)threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 0.5f;
  if (threadIdx.x == 0) {
    lds_probe[0] = v;
    out[blockIdx.x & 1023] = lds_probe[0];
  }
}
void launch_probe(int threads, int blocks, size_t lds, int iters, float* out, hipStream_t s) {
  if (threads == 1024) hipLaunchKernelGGL(launch_probe_kernel<1024>, dim3(blocks), dim3(1024), lds, s, out, iters);
  else if (threads == 512) hipLaunchKernelGGL(launch_probe_kernel<512>, dim3(blocks), dim3(512), lds, s, out, iters);
  else hipLaunchKernelGGL(launch_probe_kernel<256>, dim3(blocks), dim3(256), lds, s, out, iters);
}
}  // namespace lfk
