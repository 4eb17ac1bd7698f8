// GPU sampler: the upstream chain - repetition/frequency/presence
// penalties over the last-n window -> top-k -> top-p -> min-p -> temperature ->
// draw - runs on the device, so only a 4-byte token id ever crosses to the host
// (upstream copies 501 KiB of logits per token and samples on the CPU).
//
// Stage 1 (one block per ~1K-logit slice): penalties on the slice, then the
// slice's top-K by an exact 32-step bisection on order-preserving integer keys.
// Stage 2 (one block): exact global top-K of the stage-1 candidates, a 64-lane
// bitonic sort, then top-p / min-p / temperature / draw on <= 64 survivors and
// the device-state update (token, position, RNG step, penalty ring).
//
// The uniform draw is SplitMix64(seed ^ step*C) >> 40 - identical to
// engine/sampling.py:philox_uniform and the CPU backend.
#include <cfloat>

#include "kernels.h"
#include "qdot.h"

namespace lfk {

static constexpr int KMAX = 64;
static constexpr int SLICE = 1024;  // logits per stage-1 block (4 per thread)


__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// block-wide count of keys >= cand (each thread holds NE keys); ping-pong LDS slots
template <int NE>
__device__ __forceinline__ int block_count_ge(const unsigned (&keys)[NE], unsigned cand, int* slots, int parity) {
  int c = 0;
#pragma unroll
  for (int j = 0; j < NE; ++j) c += __popcll(__ballot(keys[j] >= cand));
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) slots[parity * 4 + wave] = c;
  __syncthreads();
  return slots[parity * 4 + 0] + slots[parity * 4 + 1] + slots[parity * 4 + 2] + slots[parity * 4 + 3];
}

// exact K-th largest key among the block's keys (keys < 1 are padding)
template <int NE>
__device__ unsigned kth_largest(const unsigned (&keys)[NE], int K, int* slots) {
  unsigned tau = 0;
  for (int bit = 31; bit >= 0; --bit) {
    const unsigned cand = tau | (1u << bit);
    if (block_count_ge<NE>(keys, cand, slots, bit & 1) >= K) tau = cand;
  }
  return tau;
}

template <int NE>
__device__ int compact_topk(const unsigned (&keys)[NE], const int (&idx)[NE], unsigned tau, int K, unsigned* okey,
                            int* oidx, int* counter) {
  if (threadIdx.x == 0) { counter[0] = 0; counter[1] = 0; }
  __syncthreads();
  int n_gt = 0;
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    if (keys[j] > tau) {
      const int p = atomicAdd(&counter[0], 1);
      okey[p] = keys[j];
      oidx[p] = idx[j];
    }
  }
  __syncthreads();
  n_gt = counter[0];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    if (keys[j] == tau && tau != 0) {
      const int p = atomicAdd(&counter[1], 1);
      if (n_gt + p < K) {
        okey[n_gt + p] = keys[j];
        oidx[n_gt + p] = idx[j];
      }
    }
  }
  __syncthreads();
  return min(K, n_gt + counter[1]);
}

__global__ __launch_bounds__(256) void sample_stage1(SamplerArgs a) {
  __shared__ float sl[SLICE];
  __shared__ int win[64];
  __shared__ int slots[8];
  __shared__ int counter[2];
  __shared__ unsigned okey[KMAX];
  __shared__ int oidx[KMAX];
  const int tid = threadIdx.x;
  const int lo = blockIdx.x * SLICE;
  const int n = min(SLICE, a.V - lo);
  for (int i = tid; i < SLICE; i += 256) sl[i] = i < n ? a.logits[lo + i] : -FLT_MAX;
  // penalty window (the last min(ring_len, last_n) sampled/prompt tokens)
  const int rlen = a.state[S_RING_LEN], rhead = a.state[S_RING_HEAD];
  const SamplerParamsDev& P = *a.p;
  const int wn = min(rlen, P.last_n);
  if (tid < 64) win[tid] = tid < wn ? a.ring[(rhead - wn + tid + 64) & 63] : -1;
  __syncthreads();
  if (tid < wn) {
    const int t = win[tid];
    bool first = true;
    int cnt = 0;
    for (int j = 0; j < wn; ++j) {
      if (win[j] == t) { cnt++; if (j < tid) first = false; }
    }
    if (first && t >= lo && t < lo + n) {
      float l = sl[t - lo];
      l = l <= 0.f ? l * P.repeat_penalty : l / P.repeat_penalty;
      l -= (float)cnt * P.freq_penalty + P.presence_penalty;
      sl[t - lo] = l;
    }
  }
  __syncthreads();
  unsigned keys[4];
  int idx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = tid + 256 * j;
    keys[j] = i < n ? fkey(sl[i]) : 0u;
    idx[j] = lo + i;
  }
  const int K = P.top_k;
  const unsigned tau = kth_largest<4>(keys, K, slots);
  const int m = compact_topk<4>(keys, idx, tau, K, okey, oidx, counter);
  if (tid < K) {
    a.cand_val[blockIdx.x * KMAX + tid] = tid < m ? kfloat(okey[tid]) : -FLT_MAX;
    a.cand_idx[blockIdx.x * KMAX + tid] = tid < m ? oidx[tid] : -1;
  }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  unsigned long long z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void sample_stage2(SamplerArgs a, int nb) {
  __shared__ int slots[8];
  __shared__ int counter[2];
  __shared__ unsigned okey[KMAX];
  __shared__ int oidx[KMAX];
  constexpr int NE = 32;  // up to 256*32 = 8192 candidates (128 blocks x 64)
  const int tid = threadIdx.x;
  const SamplerParamsDev& P = *a.p;
  const int K = P.top_k;
  const int ncand = nb * KMAX;
  unsigned keys[NE];
  int idx[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int i = tid + 256 * j;
    const bool ok = i < ncand && (i % KMAX) < K && a.cand_idx[i] >= 0;
    keys[j] = ok ? fkey(a.cand_val[i]) : 0u;
    idx[j] = ok ? a.cand_idx[i] : 0x7fffffff;
  }
  const unsigned tau = kth_largest<NE>(keys, K, slots);
  const int m = compact_topk<NE>(keys, idx, tau, K, okey, oidx, counter);
  if (tid >= 64) return;
  // ---- one wave: bitonic sort (descending value, ascending index) of <= 64 candidates
  const int lane = tid;
  float v = lane < m ? kfloat(okey[lane]) : -FLT_MAX;
  int id = lane < m ? oidx[lane] : 0x7fffffff;
  for (int size = 2; size <= 64; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float ov = __shfl_xor(v, stride);
      const int oi = __shfl_xor(id, stride);
      const bool up = ((lane & size) == 0);          // this sub-sequence sorted descending
      const bool lower = ((lane & stride) == 0);
      const bool other_better = (ov > v) || (ov == v && oi < id);
      const bool take = (lower == up) ? other_better : !other_better;
      if (take && !(ov == v && oi == id)) { v = ov; id = oi; }
    }
  }
  int tok;
  if (P.greedy || m <= 1) {
    tok = __shfl(id, 0);
  } else {
    const float v0 = __shfl(v, 0);
    // top-p on temperature-1 probabilities
    const float e = lane < m ? __expf(v - v0) : 0.f;
    float cum = e;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(cum, o);
      if (lane >= o) cum += t;
    }
    const float tot = __shfl(cum, 63);
    int n1 = m;
    if (P.top_p < 1.f) {
      const unsigned long long reach = __ballot(lane < m && cum >= P.top_p * tot);
      if (reach) n1 = min(m, (int)__ffsll((long long)reach));  // first index reaching p, inclusive
    }
    int n2 = n1;
    if (P.min_p > 0.f) {
      const float thr = v0 + __logf(P.min_p);
      n2 = max(1, (int)__popcll(__ballot(lane < n1 && v >= thr)));
    }
    const float w = lane < n2 ? __expf((v - v0) / P.temp) : 0.f;
    float cw = w;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(cw, o);
      if (lane >= o) cw += t;
    }
    const float wt = __shfl(cw, 63);
    const int step = a.state[S_STEP];
    const unsigned long long h = splitmix64(P.seed ^ ((unsigned long long)step * 0xD1B54A32D192ED03ull));
    const float u = (float)(h >> 40) * (1.f / 16777216.f);
    const unsigned long long over = __ballot(lane < n2 && cw > u * wt);
    const int pick = over ? (int)__ffsll((long long)over) - 1 : n2 - 1;
    tok = __shfl(id, pick);
  }
  if (lane == 0) {
    int* st = a.state;
    st[S_TOKEN] = tok;
    const int head = st[S_RING_HEAD];
    a.ring[head & 63] = tok;
    st[S_RING_HEAD] = (head + 1) & 63;
    st[S_RING_LEN] = min(st[S_RING_LEN] + 1, 64);
    if (a.out_tokens) a.out_tokens[st[S_NOUT] % a.out_cap] = tok;
    st[S_NOUT] += 1;
    st[S_STEP] += 1;
    if (a.advance_pos) st[S_POS] += 1;
  }
}

int sampler_blocks(int V) { return (V + SLICE - 1) / SLICE; }

void sample(const SamplerArgs& a, hipStream_t s) {
  const int nb = sampler_blocks(a.V);
  if (nb * KMAX > 256 * 32) throw std::runtime_error("GPU sampler: vocabulary too large");
  hipLaunchKernelGGL(sample_stage1, dim3(nb), dim3(256), 0, s, a);
  hipLaunchKernelGGL(sample_stage2, dim3(1), dim3(256), 0, s, a, nb);
}

}  // namespace lfk
