// KV-cache attention: QK^T, masked softmax and PV fused.
//
// Cache layout: per layer [n_kv_head][n_ctx][head_dim] f16 (K and V alike,
// V NOT transposed - both decode and prefill read key/value rows contiguously).
//
// Decode (T=1): split-L "flash decoding". Grid (kv_head, split); each block
// takes 64 keys of one kv head and ALL gqa query heads that share it (GQA
// packing: K/V rows are read once for 4-8 query heads), writes an unnormalised
// partial (o, m, l); a combine kernel merges the splits. The KV length is read
// from device memory, so one graph-captured launch serves every position (blocks
// past the current length exit immediately).
#include <cfloat>

#include "kernels.h"
#include "qdot.h"

namespace lfk {

static constexpr int CH = 64;  // keys per split

// One block = 64 keys of one kv head x all G query heads sharing it.
//   1. every thread issues its K and V loads first (4 lanes per key, HD/4 dims
//      per lane: 2-4 independent 16-B loads each), q goes to LDS meanwhile;
//   2. partial dots -> 2 shuffles -> scores; block softmax over the 64 keys;
//   3. V is staged through LDS and re-read as (head, dim-pair) per thread;
//   4. partial (o, m, l) -> workspace; the LAST arriving block of this kv head
//      (agent-scope release/acquire + counter, reset by that block) merges all
//      splits, so no separate combine launch is needed.
template <int HD>
__global__ __launch_bounds__(256) void attn_decode_kernel(AttnDecodeArgs a) {
  constexpr int DPL = HD / 4;  // dims per lane
  constexpr int NLD = DPL / 8; // 16-B loads per lane per K (or V) row
  const int kvh = blockIdx.x, split = blockIdx.y;
  const int L = *a.pos + 1;
  const int start = split * CH;
  if (start >= L) return;
  const int n = min(CH, L - start);
  const int G = a.n_head / a.n_kv_head;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int key = tid >> 2, sub = tid & 3;
  __shared__ float qs[8][HD];
  __shared__ __attribute__((aligned(16))) __half vs[CH][HD + 8];
  __shared__ float ps[8][CH];
  __shared__ float red[8][4];
  __shared__ float mstat[8][2];
  __shared__ int last;
  (void)mstat;

  // ---- 1. issue K/V row loads (clamped to the last valid key)
  const int kk = min(key, n - 1);
  const size_t row = ((size_t)kvh * a.n_ctx + start + kk) * HD + sub * DPL;
  uint4 kr[NLD], vr[NLD];
#pragma unroll
  for (int i = 0; i < NLD; ++i) kr[i] = *reinterpret_cast<const uint4*>(a.k_cache + row + 8 * i);
#pragma unroll
  for (int i = 0; i < NLD; ++i) vr[i] = *reinterpret_cast<const uint4*>(a.v_cache + row + 8 * i);
  for (int i = tid; i < G * HD; i += 256) qs[i / HD][i % HD] = a.q[(size_t)(kvh * G) * HD + i] * a.scale;
#pragma unroll
  for (int i = 0; i < NLD; ++i) *reinterpret_cast<uint4*>(&vs[key][sub * DPL + 8 * i]) = vr[i];
  __syncthreads();

  // ---- 2. scores
  float kf[DPL];
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const unsigned w[4] = {kr[i].x, kr[i].y, kr[i].z, kr[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      kf[8 * i + 2 * j] = h2f(w[j] & 0xFFFF);
      kf[8 * i + 2 * j + 1] = h2f(w[j] >> 16);
    }
  }
  float sc[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    float p = 0.f;
    if (g < G) {
      const float4* q4 = reinterpret_cast<const float4*>(&qs[g][sub * DPL]);
#pragma unroll
      for (int i = 0; i < DPL / 4; ++i) {
        const float4 q = q4[i];
        p += q.x * kf[4 * i] + q.y * kf[4 * i + 1] + q.z * kf[4 * i + 2] + q.w * kf[4 * i + 3];
      }
    }
    p += __shfl_xor(p, 1);
    p += __shfl_xor(p, 2);
    sc[g] = key < n ? p : -FLT_MAX;
  }
  // block max / sum per head: wave-reduce over its 16 keys, then across the 4 waves
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    if (g < G) {
      float m = sc[g];
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
      if (lane == 0) red[g][wave] = m;
    }
  }
  __syncthreads();
  __shared__ float red2[8][4];
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    if (g < G) {
      const float M = fmaxf(fmaxf(red[g][0], red[g][1]), fmaxf(red[g][2], red[g][3]));
      const float e = key < n ? __expf(sc[g] - M) : 0.f;
      if (sub == 0) ps[g][key] = e;
      float l = sub == 0 ? e : 0.f;
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) l += __shfl_xor(l, o);
      l += __shfl_xor(l, 1);
      l += __shfl_xor(l, 2);
      if (lane == 0) red2[g][wave] = l;
    }
  }
  __syncthreads();
  if (tid < G) {
    mstat[tid][0] = fmaxf(fmaxf(red[tid][0], red[tid][1]), fmaxf(red[tid][2], red[tid][3]));
    mstat[tid][1] = red2[tid][0] + red2[tid][1] + red2[tid][2] + red2[tid][3];
  }

  // ---- 3. PV: thread -> (head g, dim pair)
  const int npairs = G * (HD / 2);
  for (int pi = tid; pi < npairs; pi += 256) {
    const int g = pi / (HD / 2), dp = pi % (HD / 2);
    float o0 = 0.f, o1 = 0.f;
#pragma unroll 8
    for (int k = 0; k < n; ++k) {
      const float p = ps[g][k];
      const __half2 v = *reinterpret_cast<const __half2*>(&vs[k][2 * dp]);
      o0 += p * __low2float(v);
      o1 += p * __high2float(v);
    }
    float* dst = a.part + ((size_t)split * a.n_head + kvh * G + g) * (HD + 2);
    dst[2 * dp] = o0;
    dst[2 * dp + 1] = o1;
  }
  __syncthreads();
  if (tid < G) {
    float* dst = a.part + ((size_t)split * a.n_head + kvh * G + tid) * (HD + 2);
    dst[HD] = mstat[tid][0];
    dst[HD + 1] = mstat[tid][1];
  }

  // ---- 4. last arriver merges the splits of this kv head
  const int ns = (L + CH - 1) / CH;
  if (ns == 1) {
    // single split: normalise in place
    __syncthreads();
    for (int pi = tid; pi < G * HD; pi += 256) {
      const int g = pi / HD, d = pi % HD;
      const float* src = a.part + ((size_t)kvh * G + g) * (HD + 2);
      a.out[(size_t)(kvh * G + g) * HD + d] = src[d] / src[HD + 1];
    }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(a.counters + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (prev == ns - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(a.counters + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (!last) return;
  // merge: M and the denominator per head by a wave reduction over splits, then
  // every output element sums its splits with independent (unrolled) loads
  __shared__ float Ms[8], den_s[8];
  for (int g = wave; g < G; g += 4) {
    const int l = lane;
    const int h = kvh * G + g;
    float m = -FLT_MAX;
    for (int s2 = l; s2 < ns; s2 += 64) m = fmaxf(m, a.part[((size_t)s2 * a.n_head + h) * (HD + 2) + HD]);
    m = wave_max(m);
    float den = 0.f;
    for (int s2 = l; s2 < ns; s2 += 64) {
      const float* p = a.part + ((size_t)s2 * a.n_head + h) * (HD + 2);
      den += __expf(p[HD] - m) * p[HD + 1];
    }
    den = wave_sum(den);
    if (l == 0) { Ms[g] = m; den_s[g] = den; }
  }
  __syncthreads();
  for (int pi = tid; pi < G * HD; pi += 256) {
    const int g = pi / HD, d = pi % HD;
    const int h = kvh * G + g;
    const float M = Ms[g];
    float num = 0.f;
#pragma unroll 4
    for (int s2 = 0; s2 < ns; ++s2) {
      const float* p = a.part + ((size_t)s2 * a.n_head + h) * (HD + 2);
      num += __expf(p[HD] - M) * p[d];
    }
    a.out[(size_t)h * HD + d] = num / den_s[g];
  }
}

size_t attn_decode_workspace_floats(int n_ctx, int n_head, int head_dim) {
  return (size_t)((n_ctx + CH - 1) / CH) * n_head * (head_dim + 2);
}

void attn_decode(const AttnDecodeArgs& a, hipStream_t s) {
  const int G = a.n_head / a.n_kv_head;
  if (G > 8 || a.n_head % a.n_kv_head) throw std::runtime_error("attn_decode: gqa group must be <= 8");
  if (!a.counters) throw std::runtime_error("attn_decode: counters workspace missing");
  dim3 grid(a.n_kv_head, (a.n_ctx + CH - 1) / CH);
  if (a.head_dim == 128) hipLaunchKernelGGL(attn_decode_kernel<128>, grid, dim3(256), 0, s, a);
  else if (a.head_dim == 64) hipLaunchKernelGGL(attn_decode_kernel<64>, grid, dim3(256), 0, s, a);
  else throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
}

// ---------------------------------------------------------------- prefill
// One wave = 4 queries of one head; lanes stride over keys (64 per step) for
// QK^T, then over head dims for PV, with an online softmax per query. Keys are
// bounded by the causal limit of the wave's last query.
template <int HD>
__global__ __launch_bounds__(256) void attn_prefill_kernel(AttnPrefillArgs a) {
  constexpr int QW = 4;
  const int h = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t0 = (blockIdx.y * 4 + wave) * QW;
  const int G = a.n_head / a.n_kv_head;
  const int kvh = h / G;
  __shared__ float qs[4][QW][HD];
  __shared__ float ps[4][QW][64];
  for (int i = lane; i < QW * HD; i += 64) {
    const int qi = i / HD, d = i % HD;
    const int t = t0 + qi;
    qs[wave][qi][d] = t < a.T ? a.q[((size_t)t * a.n_head + h) * HD + d] * a.scale : 0.f;
  }
  __syncthreads();
  if (t0 >= a.T) return;
  const int tlast = min(t0 + QW, a.T) - 1;
  const int nkeys = a.pos0 + tlast + 1;
  constexpr int DPL = HD / 64;  // dims per lane in PV
  float m[QW], l[QW], o[QW][DPL];
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) {
    m[qi] = -FLT_MAX;
    l[qi] = 0.f;
#pragma unroll
    for (int j = 0; j < DPL; ++j) o[qi][j] = 0.f;
  }
  const __half* kb = a.k_cache + (size_t)kvh * a.n_ctx * HD;
  const __half* vb = a.v_cache + (size_t)kvh * a.n_ctx * HD;
  for (int k0 = 0; k0 < nkeys; k0 += 64) {
    const int key = k0 + lane;
    float s[QW];
#pragma unroll
    for (int qi = 0; qi < QW; ++qi) s[qi] = 0.f;
    if (key < nkeys) {
      const uint4* kr = reinterpret_cast<const uint4*>(kb + (size_t)key * HD);
#pragma unroll 4
      for (int c = 0; c < HD / 8; ++c) {
        const uint4 raw = kr[c];
        const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float k0f = h2f(w[i] & 0xFFFF), k1f = h2f(w[i] >> 16);
#pragma unroll
          for (int qi = 0; qi < QW; ++qi)
            s[qi] += qs[wave][qi][8 * c + 2 * i] * k0f + qs[wave][qi][8 * c + 2 * i + 1] * k1f;
        }
      }
    }
#pragma unroll
    for (int qi = 0; qi < QW; ++qi) {
      const int lim = a.pos0 + t0 + qi;  // causal: key <= absolute position of the query
      const float sv = (key <= lim && key < nkeys) ? s[qi] : -FLT_MAX;
      const float cm = wave_max(sv);
      const float mn = fmaxf(m[qi], cm);
      const float p = (key <= lim && key < nkeys) ? __expf(sv - mn) : 0.f;
      const float alpha = __expf(m[qi] - mn);
      l[qi] = l[qi] * alpha + wave_sum(p);
#pragma unroll
      for (int j = 0; j < DPL; ++j) o[qi][j] *= alpha;
      m[qi] = mn;
      ps[wave][qi][lane] = p;
    }
    __builtin_amdgcn_wave_barrier();
    const int kend = min(64, nkeys - k0);
    for (int j = 0; j < kend; ++j) {
      const __half* vr = vb + (size_t)(k0 + j) * HD;
#pragma unroll
      for (int dj = 0; dj < DPL; ++dj) {
        const float v = __half2float(vr[lane + 64 * dj]);
#pragma unroll
        for (int qi = 0; qi < QW; ++qi) o[qi][dj] += ps[wave][qi][j] * v;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) {
    const int t = t0 + qi;
    if (t < a.T) {
#pragma unroll
      for (int dj = 0; dj < DPL; ++dj) a.out[(size_t)t * a.out_stride + h * HD + lane + 64 * dj] = o[qi][dj] / l[qi];
    }
  }
}

void attn_prefill(const AttnPrefillArgs& a, hipStream_t s) {
  if (a.n_head % a.n_kv_head) throw std::runtime_error("attn_prefill: n_head % n_kv_head");
  dim3 grid(a.n_head, (a.T + 15) / 16);
  if (a.head_dim == 128) hipLaunchKernelGGL(attn_prefill_kernel<128>, grid, dim3(256), 0, s, a);
  else if (a.head_dim == 64) hipLaunchKernelGGL(attn_prefill_kernel<64>, grid, dim3(256), 0, s, a);
  else throw std::runtime_error("attn_prefill: head_dim must be 64 or 128");
}

}  // namespace lfk
