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

template <int HD>
__global__ __launch_bounds__(256) void attn_decode_split_kernel(AttnDecodeArgs a) {
  const int kvh = blockIdx.x, split = blockIdx.y;
  const int L = *a.pos + 1;
  const int start = split * CH;
  if (start >= L) return;
  const int n = min(CH, L - start);
  const int G = a.n_head / a.n_kv_head;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float qs[8][HD];
  __shared__ float sc[8][CH];
  __shared__ float ml[8][2];
  constexpr int NDP = HD / 2, NS = 256 / NDP;
  __shared__ float red[NS][8][HD];

  for (int i = tid; i < G * HD; i += 256) qs[i / HD][i % HD] = a.q[(size_t)(kvh * G) * HD + i] * a.scale;
  __syncthreads();

  // ---- scores: HD/8 lanes per key, 8 dims (16 B) per lane
  constexpr int LPK = HD / 8, KPP = 256 / LPK;
  const int sub = tid % LPK, kk = tid / LPK;
  const __half* kb = a.k_cache + ((size_t)kvh * a.n_ctx + start) * HD;
  for (int k0 = 0; k0 < CH; k0 += KPP) {
    const int key = k0 + kk;
    float kv[8];
    if (key < n) {
      const uint4 raw = *reinterpret_cast<const uint4*>(kb + (size_t)key * HD + sub * 8);
      const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        kv[2 * i] = h2f(w[i] & 0xFFFF);
        kv[2 * i + 1] = h2f(w[i] >> 16);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) kv[i] = 0.f;
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g < G) {
        float p = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) p += qs[g][sub * 8 + i] * kv[i];
#pragma unroll
        for (int o = LPK / 2; o > 0; o >>= 1) p += __shfl_xor(p, o);
        if (sub == 0 && key < n) sc[g][key] = p;
      }
    }
  }
  __syncthreads();

  // ---- softmax over the chunk (one wave per query head)
  for (int g = wave; g < G; g += 4) {
    const float s = lane < n ? sc[g][lane] : -FLT_MAX;
    const float m = wave_max(s);
    const float p = lane < n ? __expf(s - m) : 0.f;
    const float l = wave_sum(p);
    sc[g][lane] = p;
    if (lane == 0) { ml[g][0] = m; ml[g][1] = l; }
  }
  __syncthreads();

  // ---- PV: thread = (dim pair, key subset)
  const int dp = tid % NDP, ks = tid / NDP;
  float o[8][2];
#pragma unroll
  for (int g = 0; g < 8; ++g) o[g][0] = o[g][1] = 0.f;
  const __half* vb = a.v_cache + ((size_t)kvh * a.n_ctx + start) * HD;
  for (int key = ks; key < n; key += NS) {
    const unsigned v2 = *reinterpret_cast<const unsigned*>(vb + (size_t)key * HD + 2 * dp);
    const float v0 = h2f(v2 & 0xFFFF), v1 = h2f(v2 >> 16);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g < G) {
        const float p = sc[g][key];
        o[g][0] += p * v0;
        o[g][1] += p * v1;
      }
    }
  }
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    if (g < G) {
      red[ks][g][2 * dp] = o[g][0];
      red[ks][g][2 * dp + 1] = o[g][1];
    }
  }
  __syncthreads();
  for (int i = tid; i < G * HD; i += 256) {
    const int g = i / HD, d = i % HD;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NS; ++k) s += red[k][g][d];
    float* dst = a.part + ((size_t)split * a.n_head + kvh * G + g) * (HD + 2);
    dst[d] = s;
    if (d == 0) { dst[HD] = ml[g][0]; dst[HD + 1] = ml[g][1]; }
  }
}

template <int HD>
__global__ __launch_bounds__(HD) void attn_decode_combine_kernel(AttnDecodeArgs a) {
  const int h = blockIdx.x, d = threadIdx.x;
  const int L = *a.pos + 1;
  const int ns = (L + CH - 1) / CH;
  float M = -FLT_MAX;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, a.part[((size_t)s * a.n_head + h) * (HD + 2) + HD]);
  float num = 0.f, den = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float* p = a.part + ((size_t)s * a.n_head + h) * (HD + 2);
    const float e = __expf(p[HD] - M);
    num += e * p[d];
    den += e * p[HD + 1];
  }
  a.out[(size_t)h * HD + d] = num / den;
}

size_t attn_decode_workspace_floats(int n_ctx, int n_head, int head_dim) {
  return (size_t)((n_ctx + CH - 1) / CH) * n_head * (head_dim + 2);
}

void attn_decode(const AttnDecodeArgs& a, hipStream_t s) {
  const int G = a.n_head / a.n_kv_head;
  if (G > 8 || a.n_head % a.n_kv_head) throw std::runtime_error("attn_decode: gqa group must be <= 8");
  dim3 grid(a.n_kv_head, (a.n_ctx + CH - 1) / CH);
  if (a.head_dim == 128) {
    hipLaunchKernelGGL(attn_decode_split_kernel<128>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(attn_decode_combine_kernel<128>, dim3(a.n_head), dim3(128), 0, s, a);
  } else if (a.head_dim == 64) {
    hipLaunchKernelGGL(attn_decode_split_kernel<64>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(attn_decode_combine_kernel<64>, dim3(a.n_head), dim3(64), 0, s, a);
  } else {
    throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
  }
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
