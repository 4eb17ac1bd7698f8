// GPU sampler: the upstream chain - repetition/frequency/presence
// penalties over the last-n window -> top-k -> top-p -> min-p -> temperature ->
// draw - runs on the device, so only a 4-byte token id ever crosses to the host
// (upstream copies 501 KiB of logits per token and samples on the CPU).
//
// Penalties: one wave patches the <= 64 penalised logits in place.
// Stage 1 (one WAVE per 1K-logit slice, no LDS, no barrier): the slice's top-K
// by an exact 32-step bisection on order-preserving integer keys (ballots).
// Stage 2 (one block): candidates below the largest slice threshold are dropped
// (they cannot be in the global top-K), the rest are selected exactly by one
// wave, bitonic-sorted, then top-p / min-p / temperature / draw, and the device
// state (token, position, RNG step, penalty ring) is updated.
//
// The uniform draw is SplitMix64(seed ^ step*C) >> 40 - identical to
// engine/sampling.py:philox_uniform and the CPU backend.
#include <cfloat>

#include "kernels.h"
#include "qdot.h"

namespace lfk {

static constexpr int KMAX = 64;
static constexpr int SLICE = 1024;  // logits per stage-1 wave (16 per lane)
static constexpr int NE1 = SLICE / 64;

__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}

// Penalties, in place on the logits buffer (rewritten by the lm_head every step).
// Lane i owns window entry i; only the first occurrence of a token applies it.
__global__ __launch_bounds__(64) void sample_penalties(SamplerArgs a) {
  const SamplerParamsDev& P = *a.p;
  const int lane = threadIdx.x;
  const int rlen = a.state[S_RING_LEN], rhead = a.state[S_RING_HEAD];
  const int wn = min(rlen, P.last_n);
  const int t = lane < wn ? a.ring[(rhead - wn + lane + 64) & 63] : -1;
  int cnt = 0;
  bool first = true;
  for (int j = 0; j < 64; ++j) {
    const int tj = __shfl(t, j);
    if (tj == t) {
      ++cnt;
      if (j < lane) first = false;
    }
  }
  if (t >= 0 && t < a.V && first) {
    float l = a.logits[t];
    l = l <= 0.f ? l * P.repeat_penalty : l / P.repeat_penalty;
    l -= (float)cnt * P.freq_penalty + P.presence_penalty;
    a.logits[t] = l;
  }
}

// Superset selection by value bisection: find T with K <= count(v >= T) <= 64
// (or the best effort after 40 halvings, ties), then every element >= T is a
// candidate. A superset of the top-K is exact for the final selection: stage 2
// sorts <= 64 survivors and keeps the first K. Typically 5-8 halvings.
template <int NE>
__device__ __forceinline__ float wave_superset_threshold(const float (&v)[NE], int K) {
  float lo = FLT_MAX, hi = -FLT_MAX;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    if (v[e] > -FLT_MAX) lo = fminf(lo, v[e]);
    hi = fmaxf(hi, v[e]);
  }
  lo = -wave_max(-lo);
  hi = wave_max(hi);
  // invariant: count(>= T) >= K (T starts at the minimum); hi only ever lowers
  float T = lo;
  int cT = 0;
#pragma unroll
  for (int e = 0; e < NE; ++e) cT += v[e] >= T;
  cT = (int)wave_sum((float)cT);
  for (int it = 0; it < 40 && cT > KMAX; ++it) {
    const float mid = 0.5f * (T + hi);
    if (!(mid > T) || !(mid < hi)) break;
    int cm = 0;
#pragma unroll
    for (int e = 0; e < NE; ++e) cm += v[e] >= mid;
    cm = (int)wave_sum((float)cm);
    if (cm >= K) { T = mid; cT = cm; } else { hi = mid; }
  }
  return T;
}

// wave-ordered compaction of the values >= T (at most `cap` kept)
template <int NE>
__device__ __forceinline__ int wave_collect(const float (&v)[NE], const int (&idx)[NE], float T, int cap, float* ov,
                                            int* oi) {
  const int lane = threadIdx.x & 63;
  int base = 0;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const bool f = v[e] >= T && v[e] > -FLT_MAX;
    const unsigned long long m = __ballot(f);
    if (f) {
      const int p = base + lanes_below(m);
      if (p < cap) { ov[p] = v[e]; oi[p] = idx[e]; }
    }
    base += __popcll(m);
  }
  return min(base, cap);
}

__global__ __launch_bounds__(64) void sample_stage1(SamplerArgs a) {
  const int lane = threadIdx.x;
  const int lo = blockIdx.x * SLICE;
  const int K = a.p->top_k;
  float v[NE1];
  int idx[NE1];
#pragma unroll
  for (int e = 0; e < NE1; ++e) {
    const int i = lo + 64 * e + lane;
    v[e] = i < a.V ? a.logits[i] : -FLT_MAX;
    idx[e] = i;
  }
  const float T = wave_superset_threshold<NE1>(v, K);
  float* ov = a.cand_val + blockIdx.x * KMAX;
  int* oi = a.cand_idx + blockIdx.x * KMAX;
  const int m = wave_collect<NE1>(v, idx, T, KMAX, ov, oi);
  if (lane >= m) {
    ov[lane] = -FLT_MAX;
    oi[lane] = -1;
  }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  unsigned long long z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Stage 2 (one 256-thread block): superset threshold over all stage-1
// candidates (block-wide counts), collect <= 64 into LDS, then one wave sorts
// (value desc, index asc), keeps K, applies top-p / min-p / temperature, draws,
// and updates the device state.
__device__ __forceinline__ int block_count(int c, int* red, int parity) {
  c = (int)wave_sum((float)c);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[parity * 4 + wave] = c;
  __syncthreads();
  return red[parity * 4] + red[parity * 4 + 1] + red[parity * 4 + 2] + red[parity * 4 + 3];
}

template <int NE2>
__global__ __launch_bounds__(256) void sample_stage2(SamplerArgs a, int nb) {
  __shared__ float tval[KMAX];
  __shared__ int tidx[KMAX];
  __shared__ int red[8];
  __shared__ float redf[8];
  __shared__ int ncol;
  const int tid = threadIdx.x;
  const SamplerParamsDev& P = *a.p;
  const int K = P.top_k;
  float v[NE2];
  int idx[NE2];
#pragma unroll
  for (int e = 0; e < NE2; ++e) {
    const int i = 256 * e + tid;
    const bool ok = i < nb * KMAX;
    const int id = ok ? a.cand_idx[i] : -1;
    v[e] = (ok && id >= 0) ? a.cand_val[i] : -FLT_MAX;
    idx[e] = id;
  }
  // block min / max of the valid candidates
  float lo = FLT_MAX, hi = -FLT_MAX;
#pragma unroll
  for (int e = 0; e < NE2; ++e) {
    if (v[e] > -FLT_MAX) lo = fminf(lo, v[e]);
    hi = fmaxf(hi, v[e]);
  }
  lo = -wave_max(-lo);
  hi = wave_max(hi);
  if ((tid & 63) == 0) { redf[tid >> 6] = lo; redf[4 + (tid >> 6)] = hi; }
  if (tid == 0) ncol = 0;
  __syncthreads();
  lo = fminf(fminf(redf[0], redf[1]), fminf(redf[2], redf[3]));
  hi = fmaxf(fmaxf(redf[4], redf[5]), fmaxf(redf[6], redf[7]));
  float T = lo;
  int c = 0;
#pragma unroll
  for (int e = 0; e < NE2; ++e) c += v[e] >= T && v[e] > -FLT_MAX;
  int cT = block_count(c, red, 0);
  for (int it = 0; it < 40 && cT > KMAX; ++it) {
    const float mid = 0.5f * (T + hi);
    if (!(mid > T) || !(mid < hi)) break;
    c = 0;
#pragma unroll
    for (int e = 0; e < NE2; ++e) c += v[e] >= mid;
    const int cm = block_count(c, red, (it + 1) & 1);
    if (cm >= K) { T = mid; cT = cm; } else { hi = mid; }
  }
#pragma unroll
  for (int e = 0; e < NE2; ++e) {
    if (v[e] >= T && v[e] > -FLT_MAX) {
      const int p = atomicAdd(&ncol, 1);
      if (p < KMAX) { tval[p] = v[e]; tidx[p] = idx[e]; }
    }
  }
  __syncthreads();
  if (tid >= 64) return;
  const int lane = tid;
  int m = min(ncol, KMAX);
  // ---- bitonic sort (descending value, ascending index) of <= 64 candidates
  float vv = lane < m ? tval[lane] : -FLT_MAX;
  int id = lane < m ? tidx[lane] : 0x7fffffff;
  for (int size = 2; size <= 64; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float ov = __shfl_xor(vv, stride);
      const int oi = __shfl_xor(id, stride);
      const bool up = ((lane & size) == 0);
      const bool lower = ((lane & stride) == 0);
      const bool other_better = (ov > vv) || (ov == vv && oi < id);
      const bool take = (lower == up) ? other_better : !other_better;
      if (take && !(ov == vv && oi == id)) { vv = ov; id = oi; }
    }
  }
  m = min(m, K);
  const float v_ = vv;
  int tok;
  if (P.greedy || m <= 1) {
    tok = __shfl(id, 0);
  } else {
    const float v0 = __shfl(v_, 0);
    // top-p on temperature-1 probabilities
    const float e = lane < m ? expf(v_ - v0) : 0.f;
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
      const float thr = v0 + logf(P.min_p);
      n2 = max(1, (int)__popcll(__ballot(lane < n1 && v_ >= thr)));
    }
    const float w = lane < n2 ? expf((v_ - v0) / P.temp) : 0.f;
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
  hipLaunchKernelGGL(sample_penalties, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(sample_stage1, dim3(nb), dim3(64), 0, s, a);
  const int ncand = nb * KMAX;
  if (ncand <= 256 * 8) hipLaunchKernelGGL(sample_stage2<8>, dim3(1), dim3(256), 0, s, a, nb);
  else if (ncand <= 256 * 32) hipLaunchKernelGGL(sample_stage2<32>, dim3(1), dim3(256), 0, s, a, nb);
  else throw std::runtime_error("GPU sampler: vocabulary too large (max 131072)");
}

}  // namespace lfk
