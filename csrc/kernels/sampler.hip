// GPU sampler: the upstream chain - repetition/frequency/presence
// penalties over the last-n window -> top-k -> top-p -> min-p -> temperature ->
// draw - runs on the device, so only a 4-byte token id ever crosses to the host
// (upstream copies 501 KiB of logits per token and samples on the CPU).
//
// Stage 1 (one WAVE per 1K-logit slice): penalties of the window tokens that
// fall in the slice, then a top-K superset of the slice by an 8-way threshold
// search (DPP reductions, ballots), plus the slice's lower bound of the global
// K-th value.
// Stage 2 (one block): candidates below the largest slice bound are dropped
// (they cannot be in the global top-K), the survivors are compacted in LDS and
// one wave selects, bitonic-sorts, applies top-p / min-p / temperature, draws,
// and updates the device state (token, position, RNG step, penalty ring).
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
  lo = -wave_max_fast(-lo);
  hi = wave_max_fast(hi);
  // invariant: count(>= T) >= K (T starts at the minimum); hi only ever lowers.
  // 8-way search per round (counts above 8 thresholds at once, DPP reductions).
  float T = lo;
  int cT = 0;
#pragma unroll
  for (int e = 0; e < NE; ++e) cT += v[e] >= T;
  cT = (int)wave_sum_fast((float)cT);
  for (int it = 0; it < 16 && cT > KMAX; ++it) {
    const float step = (hi - T) * (1.f / 9.f);
    if (!(step > 0.f) || !(T + step > T)) break;
    int best = -1, cbest = cT;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = T + step * (float)(j + 1);
      int cm = 0;
#pragma unroll
      for (int e = 0; e < NE; ++e) cm += v[e] >= t;
      cm = (int)wave_sum_fast((float)cm);
      if (cm >= K) { best = j; cbest = cm; }
    }
    const float newT = best >= 0 ? T + step * (float)(best + 1) : T;
    hi = best < 7 ? T + step * (float)(best + 2) : hi;
    T = newT;
    cT = cbest;
  }
  return T;
}

// wave-ordered compaction of the values >= T (at most `cap` kept)
template <int NE>
__device__ __forceinline__ int wave_collect(const float (&v)[NE], const int (&idx)[NE], float T, int cap, float* ov,
                                            int* oi) {
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

// Batched mode: row b of the launch (blockIdx.y in stage 1, blockIdx.x in stage 2)
// works on its own logits row and the sampling state of its KV slot; every pointer is
// re-based here so the stage bodies are the single-row code.
__device__ __forceinline__ void batch_row(SamplerArgs& a, int b) {
  if (a.batch <= 0) return;
  const int slot = a.slots[b];
  a.logits += (size_t)b * a.logits_ld;
  a.p += slot;
  a.ring += 64 * slot;
  a.state += (size_t)S_NSTATE * slot;
}

__host__ __device__ __forceinline__ size_t cand_words(int nb) { return (size_t)nb * (2 * KMAX + 2); }

// Stage 1: one wave per 1024-logit slice. The repetition/frequency/presence
// penalties of ring tokens that fall in this slice are applied here (the wave
// stages its slice in LDS, lanes owning a first occurrence patch their entry),
// then the slice's top-K superset is selected without LDS or barriers.
__global__ __launch_bounds__(64) void sample_stage1_kernel(SamplerArgs a) {
  batch_row(a, blockIdx.y);
  const int nb = gridDim.x;
  unsigned* blk = a.cand + (size_t)blockIdx.y * cand_words(nb);
  float* cand_val = reinterpret_cast<float*>(blk);
  int* cand_idx = reinterpret_cast<int*>(blk) + nb * KMAX;
  unsigned* cand_tau = blk + 2 * nb * KMAX;
  __shared__ float sl[SLICE];
  const int lane = threadIdx.x;
  const int lo = blockIdx.x * SLICE;
  const SamplerParamsDev& P = *a.p;
  const int K = P.top_k;
  float v[NE1];
  int idx[NE1];
#pragma unroll
  for (int e = 0; e < NE1; ++e) {
    const int i = lo + 64 * e + lane;
    v[e] = i < a.V ? a.logits[i] : -FLT_MAX;
    idx[e] = a.vocab_off + i;
  }
  // window / bias tokens are global ids; this slice holds [g0, g0 + SLICE) of them
  const int g0 = a.vocab_off + lo, gend = a.vocab_off + a.V;
  // ---- logit bias (lane j holds entry j; distinct tokens), then the penalties
  // (window = last min(ring_len, last_n) tokens) on the biased values
  const int nbias = P.n_bias;
  const int bt = lane < nbias ? P.bias_tok[lane] : -1;
  const bool bmine = bt >= g0 && bt < g0 + SLICE && bt < gend;
  const int rlen = a.state[S_RING_LEN], rhead = a.state[S_RING_HEAD];
  const int wn = min(rlen, P.last_n);
  const int t = lane < wn ? a.ring[(rhead - wn + lane + 64) & 63] : -1;
  const bool mine = t >= g0 && t < g0 + SLICE && t < gend;
  if (__ballot(mine) | __ballot(bmine)) {  // wave-uniform: a window or bias token lies in this slice
#pragma unroll
    for (int e = 0; e < NE1; ++e) sl[64 * e + lane] = v[e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (bmine) sl[bt - g0] += P.bias_val[lane];
    int cnt = 0;
    bool first = true;
    for (int j = 0; j < wn; ++j) {
      const int tj = __builtin_amdgcn_readlane(t, j);
      if (tj == t) {
        ++cnt;
        if (j < lane) first = false;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (mine && first) {
      float l = sl[t - g0];
      l = l <= 0.f ? l * P.repeat_penalty : l / P.repeat_penalty;
      l -= (float)cnt * P.freq_penalty + P.presence_penalty;
      sl[t - g0] = l;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int e = 0; e < NE1; ++e) v[e] = sl[64 * e + lane];
  }
  // ---- top-K superset of the slice
  const float T = wave_superset_threshold<NE1>(v, K);
  float* ov = cand_val + blockIdx.x * KMAX;
  int* oi = cand_idx + blockIdx.x * KMAX;
  const int m = wave_collect<NE1>(v, idx, T, KMAX, ov, oi);
  if (lane >= m) {
    ov[lane] = -FLT_MAX;
    oi[lane] = -1;
  }
  // this slice alone holds >= K values >= T, so the global K-th largest is >= T:
  // stage 2 drops every candidate below the largest such slice bound
  float vmax = -FLT_MAX;
#pragma unroll
  for (int e = 0; e < NE1; ++e) vmax = fmaxf(vmax, v[e]);
  vmax = wave_max_fast(vmax);
  if (lane == 0) {
    const int nvalid = min(SLICE, a.V - lo);
    cand_tau[blockIdx.x] = __float_as_uint(m >= K && nvalid >= K ? T : -FLT_MAX);
    cand_tau[nb + blockIdx.x] = __float_as_uint(vmax);
  }
}

// inclusive wave prefix sum (64 lanes)
__device__ __forceinline__ float wave_scan(float x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(x, o);
    if (lane >= o) x += t;
  }
  return x;
}

// Tail-free (llama_sample_tail_free, min_keep 1) on m > 2 candidates held one per
// lane, sorted by descending logit: normalised |second derivative| of the
// temperature-1 probabilities; keep the first i tokens where i >= 1 is the first
// index whose running sum exceeds z.
__device__ __forceinline__ int tail_free_cut(float v, int m, float z) {
  const int lane = threadIdx.x & 63;
  const float v0 = __shfl(v, 0);
  const float e = lane < m ? expf(v - v0) : 0.f;
  const float p = e / wave_sum_fast(e);
  const float p1 = __shfl(p, min(lane + 1, 63));
  const float d1 = p - p1;                       // valid for lane < m-1
  const float d1n = __shfl(d1, min(lane + 1, 63));
  const bool ok = lane < m - 2;
  float d2 = ok ? fabsf(d1 - d1n) : 0.f;
  const float s = wave_sum_fast(d2);
  d2 = ok ? (s > 1e-6f ? d2 / s : 1.f / (float)(m - 2)) : 0.f;
  const float cum = wave_scan(d2);
  const unsigned long long hit = __ballot(ok && lane >= 1 && cum > z);
  return hit ? (int)__ffsll((long long)hit) - 1 : m;
}

// Locally typical (llama_sample_typical, min_keep 1): rank the m candidates by
// |surprise - entropy| (ties by position), keep them in that order until the
// kept mass exceeds tp; the kept set is compacted back into descending-logit
// order in lanes [0, new m). Returns the new m.
__device__ __forceinline__ int typical_keep(float& v, int& id, int m, float tp) {
  const int lane = threadIdx.x & 63;
  const float v0 = __shfl(v, 0);
  const float e = lane < m ? expf(v - v0) : 0.f;
  const float p = e / wave_sum_fast(e);
  const float lp = lane < m ? logf(fmaxf(p, 1e-30f)) : 0.f;
  const float ent = -wave_sum_fast(lane < m ? p * lp : 0.f);
  const float sh = lane < m ? fabsf(-lp - ent) : FLT_MAX;
  float before = 0.f;  // mass of the candidates ranked ahead of this one
  for (int j = 0; j < m; ++j) {
    const float sj = __shfl(sh, j);
    const float pj = __shfl(p, j);
    if (sj < sh || (sj == sh && j < lane)) before += pj;
  }
  const unsigned long long keep = __ballot(lane < m && before <= tp);
  const int kept = __popcll(keep);
  const bool k = (keep >> lane) & 1ull;
  const int dst = k ? lanes_below(keep) : kept + lanes_below(~keep);
  v = __int_as_float(__builtin_amdgcn_ds_permute(dst << 2, __float_as_int(v)));
  id = __builtin_amdgcn_ds_permute(dst << 2, id);
  return max(kept, 1);
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

// Stage 2 (one 256-thread block): drop candidates below the largest slice
// bound, compact the survivors into LDS (typically < 100), then ONE wave selects
// a top-K superset of <= 64 from them (8-way threshold search, no barriers),
// sorts (value desc, index asc), keeps K, applies top-p / min-p / temperature,
// draws and updates the device state.
static constexpr int CAP2 = 2048;  // survivors above the bounds (typically < 200)
// The candidate blocks of one row: `world` of them (one per vocabulary shard), nb_l slices
// each; slice g of the row is slice g % nb_l of block g / nb_l.
struct CandRow {
  const unsigned* base;
  size_t rank_stride;   // words between two ranks' blocks of this row
  int nb_l;
  __device__ __forceinline__ const unsigned* blk(int r) const { return base + (size_t)r * rank_stride; }
  __device__ __forceinline__ void cand(int i, float& v, int& id) const {
    const int per = nb_l * KMAX, r = i / per, j = i - r * per;
    const unsigned* b = blk(r);
    v = __uint_as_float(b[j]);
    id = (int)b[per + j];
  }
  __device__ __forceinline__ float bound(int g) const {
    const int r = g / nb_l;
    return __uint_as_float(blk(r)[2 * nb_l * KMAX + (g - r * nb_l)]);
  }
  __device__ __forceinline__ float smax(int g) const {
    const int r = g / nb_l;
    return __uint_as_float(blk(r)[2 * nb_l * KMAX + nb_l + (g - r * nb_l)]);
  }
};

// one wave: the <= KMAX top-K superset of the n survivors in LDS, compacted into tval / tidx
template <int NW>
__device__ __forceinline__ int top_superset(int n, int K, const float* cval, const int* cidx, float* tval, int* tidx) {
  const int lane = threadIdx.x & 63;
  float w[NW];
  int wi[NW];
#pragma unroll
  for (int e = 0; e < NW; ++e) {
    const int i = 64 * e + lane;
    w[e] = i < n ? cval[i] : -FLT_MAX;
    wi[e] = i < n ? cidx[i] : 0x7fffffff;
  }
  const float T = n > KMAX ? wave_superset_threshold<NW>(w, K) : -FLT_MAX;
  return wave_collect<NW>(w, wi, T, KMAX, tval, tidx);
}

template <int NE2, bool TL = false>
__global__ __launch_bounds__(256) void sample_stage2_kernel(SamplerArgs a, int nb_l) {
  const int brow = blockIdx.x;
  batch_row(a, brow);
  const int rows = a.batch > 0 ? a.batch : 1;
  const int nb = nb_l * a.world;   // slices of the whole vocabulary
  CandRow cr;
  cr.nb_l = nb_l;
  cr.rank_stride = (size_t)rows * cand_words(nb_l);
  cr.base = (a.cand_all ? a.cand_all : a.cand) + (size_t)brow * cand_words(nb_l);
  long long t0 = 0;
  if constexpr (TL) t0 = wall_clock64();
#define LFK_ST(i) do { if constexpr (TL) { if (threadIdx.x == 0) a.dbg_clk[i] = wall_clock64() - t0; } } while (0)
  __shared__ float cval[CAP2];
  __shared__ int cidx[CAP2];
  __shared__ float tval[KMAX];
  __shared__ int tidx[KMAX];
  __shared__ float redf[4];
  __shared__ int ncol;
  const int tid = threadIdx.x;
  const SamplerParamsDev& P = *a.p;
  const int K = P.top_k;
  if (tid == 0) ncol = 0;
  // Two lower bounds of the global K-th largest value: (a) each slice bound
  // (that slice alone holds >= K values above it); (b) a superset threshold of
  // the slice MAXIMA (>= K distinct slices have their maximum above it).
  // (b) keeps the survivor count small even for flat (high-entropy) logits.
  // Their loads go out first and unconditionally (clamped: a repeated bound or maximum changes
  // neither), so wave 0's threshold search runs while the candidate loads are in flight
  const float sm0 = cr.smax(min(tid & 63, nb - 1)), sm1 = cr.smax(min((tid & 63) + 64, nb - 1));
  float lb = cr.bound(min(tid, nb - 1));
  float v[NE2];
  int idx[NE2];
#pragma unroll
  for (int e = 0; e < NE2; ++e) {  // independent loads (no value-dependent second load)
    const int i = min(256 * e + tid, nb * KMAX - 1);
    cr.cand(i, v[e], idx[e]);
  }
  for (int b = tid + 256; b < nb; b += 256) lb = fmaxf(lb, cr.bound(b));
  lb = wave_max_fast(lb);
  if (tid < 64) {
    float mx[2];
    mx[0] = tid < nb ? sm0 : -FLT_MAX;
    mx[1] = tid + 64 < nb ? sm1 : -FLT_MAX;
    int valid = (mx[0] > -FLT_MAX) + (mx[1] > -FLT_MAX);
    valid = (int)wave_sum_fast((float)valid);
    if (valid >= K) lb = fmaxf(lb, wave_superset_threshold<2>(mx, K));
  }
  if ((tid & 63) == 0) redf[tid >> 6] = lb;
  __syncthreads();
  lb = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
  LFK_ST(0);
  // compaction: ONE LDS atomic per wave for all of its survivors (ballot counts), then each
  // survivor's slot from the wave's base and its lane's rank (per-element atomics serialised)
  const int lane0 = tid & 63;
  int cnt = 0;
#pragma unroll
  for (int e = 0; e < NE2; ++e) {
    const bool ok = 256 * e + tid < nb * KMAX && idx[e] >= 0 && v[e] >= lb && v[e] > -FLT_MAX;
    cnt += __popcll(__ballot(ok));
  }
  int base = 0;
  if (lane0 == 0 && cnt) base = atomicAdd(&ncol, cnt);
  base = __shfl(base, 0);
#pragma unroll
  for (int e = 0; e < NE2; ++e) {
    const bool ok = 256 * e + tid < nb * KMAX && idx[e] >= 0 && v[e] >= lb && v[e] > -FLT_MAX;
    const unsigned long long m = __ballot(ok);
    if (ok) {
      const int p = base + lanes_below(m);
      if (p < CAP2) { cval[p] = v[e]; cidx[p] = idx[e]; }
    }
    base += __popcll(m);
  }
  __syncthreads();
  LFK_ST(1);
  if (tid >= 64) return;
  const int lane = tid;
  const int n = min(ncol, CAP2);
  if (lane == 0 && ncol > CAP2) a.state[S_NSTATE - 1] = ncol;  // overflow marker (diagnostics)
  // the usual survivor count (< 256) on 4 registers per lane: the threshold search's every
  // round walks all NW registers of the one working wave, so the CAP2 / 64 = 32-register form
  // cost ~8x the instructions for the same answer (entries past n are -FLT_MAX in both)
  const int mcol = n <= 256 ? top_superset<4>(n, K, cval, cidx, tval, tidx)
                            : top_superset<CAP2 / 64>(n, K, cval, cidx, tval, tidx);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  LFK_ST(2);
  int m = mcol;
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
  if (!P.greedy && m > 2 && P.tfs_z < 1.f) m = tail_free_cut(vv, m, P.tfs_z);
  if (!P.greedy && m > 1 && P.typical_p < 1.f) m = typical_keep(vv, id, m, P.typical_p);
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
    tok = min(max(tok, 0), (a.V_glob > 0 ? a.V_glob : a.V) - 1);  // non-finite logits must not leave an out-of-range id behind
    st[S_TOKEN] = tok;
    const int head = st[S_RING_HEAD];
    a.ring[head & 63] = tok;
    st[S_RING_HEAD] = (head + 1) & 63;
    st[S_RING_LEN] = min(st[S_RING_LEN] + 1, 64);
    if (a.out_tokens) a.out_tokens[st[S_NOUT] % a.out_cap] = tok;
    if (a.batch_out) a.batch_out[brow] = tok;
    if (a.batch_out_host) __hip_atomic_store(a.batch_out_host + brow, tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    LFK_ST(3);
    st[S_NOUT] += 1;
    st[S_STEP] += 1;
    if (a.advance_pos) st[S_POS] += 1;
  }
}

int sampler_blocks(int V) { return (V + SLICE - 1) / SLICE; }
size_t sampler_cand_words(int V) { return cand_words(sampler_blocks(V)); }

void sample_stage1(const SamplerArgs& a, hipStream_t s) {
  const int rows = a.batch > 0 ? a.batch : 1;
  if (a.batch > 0 && (!a.slots || a.logits_ld < (size_t)a.V || a.out_tokens || a.dbg_clk))
    throw std::runtime_error("sample: bad batched arguments");
  if (!a.cand || a.V < 0 || (a.V == 0 && a.V_span <= 0)) throw std::runtime_error("sample: no candidate buffer / empty vocabulary");
  if (a.V_span && a.V_span < a.V) throw std::runtime_error("sample: V_span < V");
  hipLaunchKernelGGL(sample_stage1_kernel, dim3(sampler_blocks(a.V_span ? a.V_span : a.V), rows), dim3(64), 0, s, a);
}

void sample_stage2(const SamplerArgs& a, hipStream_t s) {
  const int nb_l = sampler_blocks(a.V_span ? a.V_span : a.V);
  const int rows = a.batch > 0 ? a.batch : 1;
  if (a.world < 1 || (a.world > 1 && !a.cand_all)) throw std::runtime_error("sample: bad world / gathered blocks");
  const int ncand = nb_l * a.world * KMAX;
  if (a.dbg_clk && ncand <= 256 * 32) hipLaunchKernelGGL((sample_stage2_kernel<32, true>), dim3(1), dim3(256), 0, s, a, nb_l);
  else if (ncand <= 256 * 8) hipLaunchKernelGGL((sample_stage2_kernel<8, false>), dim3(rows), dim3(256), 0, s, a, nb_l);
  else if (ncand <= 256 * 32) hipLaunchKernelGGL((sample_stage2_kernel<32, false>), dim3(rows), dim3(256), 0, s, a, nb_l);
  else throw std::runtime_error("GPU sampler: vocabulary too large (max 8192 candidate slots)");
}

void sample(const SamplerArgs& a, hipStream_t s) {
  if (a.world != 1) throw std::runtime_error("sample: world > 1 needs the gathered two-stage form");
  sample_stage1(a, s);
  sample_stage2(a, s);
}

}  // namespace lfk
