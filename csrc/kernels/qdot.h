// Device-side block decoding for the planar weight layout (see ../common.h).
//
// Unit of work = one "chunk" = 32 weights of one row = 16 B of 4/6-bit data.
// A row of K weights has K/32 chunks; lane l of a wave takes chunks l, l+64, ...
// The activation vector is pre-quantised to int8 with one f32 scale per 32
// values (q8 activations, as llama.cpp's MMVQ path), so the inner product is
// int8 x int8 on v_dot4c_i32_i8 (4 MACs per VALU op) and the per-sub-block
// scales are applied once per 16-32 weights.
//
// Chunk c -> which x elements it multiplies (per superblock sb = c>>3):
//   Q4_K/Q5_K : j=c&7, g=j>>1, h=j&1 : lo 16 @ sb*256+64g+16h (sub-block 2g),
//                                      hi 16 @ +32               (sub-block 2g+1)
//   Q6_K      : j=c&7, n=j>>2, o=16(j&3): lo 16 @ sb*256+128n+o, hi 16 @ +64
//   Q8_0/F16/F32: 32 contiguous @ 32c
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "../common.h"

namespace lfk {

// two f32 -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (round to nearest even); the scalar
// __float2bfloat16 form costs a conversion per value plus the shift/or to pack
typedef float f32x2_pk_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_pk_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_bf16_pair(float a, float b) {
  const f32x2_pk_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_pk_t));
}

__device__ __forceinline__ float h2f(unsigned short h) {
  return __half2float(__ushort_as_half(h));
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));

// the XCD (XCC) this wave runs on, for timeline stamps (per-XCD clocks; placement tools only)
__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11)); }

// 16-B non-temporal load (weights are streamed once per token: do not pollute L2/MALL)
__device__ __forceinline__ int4 ld_nt16(const void* p) {
  const i32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ int dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// ---- cross-lane reductions without the LDS crossbar (DPP within 16-lane rows,
// v_readlane across rows): a few cycles per step instead of a ds_bpermute trip.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float max8(float v) {   // max over each aligned group of 8 lanes
  v = fmaxf(v, dpp_f<0xB1>(v));                      // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp_f<0x4E>(v));                      // quad_perm [2,3,0,1]
  return fmaxf(v, dpp_f<0x141>(v));                  // row_half_mirror
}
__device__ __forceinline__ float row_sum16(float v) {  // sum over each 16-lane row
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);                        // row_mirror
}
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_max_fast(float v) {  // wave-uniform result
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}
__device__ __forceinline__ float wave_sum_fast(float v) {  // wave-uniform result
  v = row_sum16(v);
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}

// x operand of one chunk, read once from LDS and reused across the NR rows.
struct XChunk {
  int lo[4];
  int hi[4];
  float dlo, dhi;  // x scales
  float slo, shi;  // x scale * sum(q_x) over the 16 lo / hi values (for the min / -32 terms)
};

template <int T>
__device__ __forceinline__ void load_x(XChunk& X, const int8_t* xq, const float* xd, int c) {
  const int sb = c >> 3, j = c & 7;
  int off_lo, off_hi, blo, bhi;
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int g = j >> 1, h = j & 1;
    off_lo = sb * 256 + 64 * g + 16 * h;
    off_hi = off_lo + 32;
    blo = sb * 8 + 2 * g;
    bhi = blo + 1;
  } else if constexpr (T == T_Q6_K) {
    const int n = j >> 2, o = 16 * (j & 3);
    off_lo = sb * 256 + 128 * n + o;
    off_hi = off_lo + 64;
    blo = off_lo >> 5;
    bhi = blo + 2;
  } else {  // Q8_0 / F16 / F32: 32 contiguous values = one x block
    off_lo = 32 * c;
    off_hi = off_lo + 16;
    blo = bhi = c;
  }
  const int4 a = *reinterpret_cast<const int4*>(xq + off_lo);
  const int4 b = *reinterpret_cast<const int4*>(xq + off_hi);
  X.lo[0] = a.x; X.lo[1] = a.y; X.lo[2] = a.z; X.lo[3] = a.w;
  X.hi[0] = b.x; X.hi[1] = b.y; X.hi[2] = b.z; X.hi[3] = b.w;
  X.dlo = xd[blo];
  X.dhi = xd[bhi];
  const int ones = 0x01010101;
  int s0 = dot4(X.lo[0], ones, dot4(X.lo[1], ones, dot4(X.lo[2], ones, dot4(X.lo[3], ones, 0))));
  int s1 = dot4(X.hi[0], ones, dot4(X.hi[1], ones, dot4(X.hi[2], ones, dot4(X.hi[3], ones, 0))));
  X.slo = X.dlo * (float)s0;
  X.shi = X.dhi * (float)s1;
}

// 6-bit (sc, m) pair for sub-blocks 2g and 2g+1 from the 12 packed scale bytes (ggml get_scale_min_k4).
__device__ __forceinline__ void scale_min_pair(int g, unsigned y, unsigned z, unsigned w, float& sc_lo, float& m_lo,
                                               float& sc_hi, float& m_hi) {
  // g < 2: direct 6-bit fields; g >= 2: 4 low bits in w, 2 high bits in the top of y / z.
  const int k = (g & 1) * 16;  // byte offset*8 of sub-block 2g within its dword (g=0,2 -> 0; 1,3 -> 16)
  unsigned a_sc, a_m, b_sc, b_m;
  if (g < 2) {
    a_sc = (y >> k) & 63;
    b_sc = (y >> (k + 8)) & 63;
    a_m = (z >> k) & 63;
    b_m = (z >> (k + 8)) & 63;
  } else {
    a_sc = ((w >> k) & 0xF) | (((y >> (k + 6)) & 3) << 4);
    b_sc = ((w >> (k + 8)) & 0xF) | (((y >> (k + 14)) & 3) << 4);
    a_m = ((w >> (k + 4)) & 0xF) | (((z >> (k + 6)) & 3) << 4);
    b_m = ((w >> (k + 12)) & 0xF) | (((z >> (k + 14)) & 3) << 4);
  }
  sc_lo = (float)a_sc; m_lo = (float)a_m; sc_hi = (float)b_sc; m_hi = (float)b_m;
}

template <int T>
__device__ __forceinline__ float chunk_dot(const uint8_t* __restrict__ base, const Planes& P, size_t row, int c,
                                           const XChunk& X) {
  const int sb = c >> 3, j = c & 7;
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int g = j >> 1;
    const uint8_t* qs_p = base + P.p0 + row * P.s0 + 16 * c;
    int4 q = ld_nt16(qs_p);
    int4 meta, qh;
    if constexpr (T == T_Q4_K) {
      meta = *reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 16);
    } else {
      qh = *reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 32 + 16 * (j & 1));
      meta = *reinterpret_cast<const int4*>(base + P.p2 + row * P.s2 + sb * 16);
    }
    const unsigned dd = (unsigned)meta.x;
    const float d = h2f(dd & 0xFFFF), dmin = h2f(dd >> 16);
    float sc_lo, m_lo, sc_hi, m_hi;
    scale_min_pair(g, (unsigned)meta.y, (unsigned)meta.z, (unsigned)meta.w, sc_lo, m_lo, sc_hi, m_hi);
    const int qv[4] = {q.x, q.y, q.z, q.w};
    int dl = 0, dh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int lo = qv[i] & 0x0F0F0F0F;
      int hi = (qv[i] >> 4) & 0x0F0F0F0F;
      if constexpr (T == T_Q5_K) {
        const int hv = (i == 0 ? qh.x : i == 1 ? qh.y : i == 2 ? qh.z : qh.w);
        lo |= ((hv >> (2 * g)) & 0x01010101) << 4;
        hi |= ((hv >> (2 * g + 1)) & 0x01010101) << 4;
      }
      dl = dot4(lo, X.lo[i], dl);
      dh = dot4(hi, X.hi[i], dh);
    }
    return d * (sc_lo * X.dlo * (float)dl + sc_hi * X.dhi * (float)dh) - dmin * (m_lo * X.slo + m_hi * X.shi);
  } else if constexpr (T == T_Q6_K) {
    const int n = j >> 2, o = 16 * (j & 3);
    int4 ql = ld_nt16(base + P.p0 + row * P.s0 + 16 * c);
    int4 qh = *reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 64 + 32 * n + (o & 31));
    int4 scv = *reinterpret_cast<const int4*>(base + P.p2 + row * P.s2 + sb * 16);
    const float d = h2f(*reinterpret_cast<const unsigned short*>(base + P.p3 + row * P.s3 + sb * 2));
    const int si = 8 * n + (o >> 4);  // lo scale index; hi = si + 4
    const int scw[4] = {scv.x, scv.y, scv.z, scv.w};
    const int sc_lo = (int)(signed char)((scw[si >> 2] >> (8 * (si & 3))) & 0xFF);
    const int sc_hi = (int)(signed char)((scw[(si + 4) >> 2] >> (8 * (si & 3))) & 0xFF);
    const int s = (o >= 32) ? 2 : 0;
    const int lv[4] = {ql.x, ql.y, ql.z, ql.w};
    const int hv[4] = {qh.x, qh.y, qh.z, qh.w};
    int dl = 0, dh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lo = (lv[i] & 0x0F0F0F0F) | (((hv[i] >> s) & 0x03030303) << 4);
      const int hi = ((lv[i] >> 4) & 0x0F0F0F0F) | (((hv[i] >> (s + 4)) & 0x03030303) << 4);
      dl = dot4(lo, X.lo[i], dl);
      dh = dot4(hi, X.hi[i], dh);
    }
    // sum((q-32) x) = dot - 32*sum(x)
    return d * ((float)sc_lo * (X.dlo * (float)dl - 32.f * X.slo) + (float)sc_hi * (X.dhi * (float)dh - 32.f * X.shi));
  } else if constexpr (T == T_Q8_0) {
    const int4* qp = reinterpret_cast<const int4*>(base + P.p0 + row * P.s0 + 32 * c);
    int4 a = ld_nt16(qp);
    int4 b = ld_nt16(qp + 1);
    const float d = h2f(*reinterpret_cast<const unsigned short*>(base + P.p1 + row * P.s1 + 2 * c));
    int acc = dot4(a.x, X.lo[0], 0);
    acc = dot4(a.y, X.lo[1], acc);
    acc = dot4(a.z, X.lo[2], acc);
    acc = dot4(a.w, X.lo[3], acc);
    acc = dot4(b.x, X.hi[0], acc);
    acc = dot4(b.y, X.hi[1], acc);
    acc = dot4(b.z, X.hi[2], acc);
    acc = dot4(b.w, X.hi[3], acc);
    return d * X.dlo * (float)acc;
  } else {  // F32 / F16 weights: dequantised x
    float s = 0.f;
    const int xv[8] = {X.lo[0], X.lo[1], X.lo[2], X.lo[3], X.hi[0], X.hi[1], X.hi[2], X.hi[3]};
    if constexpr (T == T_F32) {
      const float4* wp = reinterpret_cast<const float4*>(base + row * P.s0 + 128 * c);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float4 w = wp[i];
        const int v = xv[i];
        s += w.x * (float)(signed char)(v & 0xFF) + w.y * (float)(signed char)((v >> 8) & 0xFF) +
             w.z * (float)(signed char)((v >> 16) & 0xFF) + w.w * (float)(signed char)((v >> 24) & 0xFF);
      }
    } else {
      const uint2* wp = reinterpret_cast<const uint2*>(base + row * P.s0 + 64 * c);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint2 w = wp[i];
        const int v = xv[i];
        s += h2f(w.x & 0xFFFF) * (float)(signed char)(v & 0xFF) + h2f(w.x >> 16) * (float)(signed char)((v >> 8) & 0xFF) +
             h2f(w.y & 0xFFFF) * (float)(signed char)((v >> 16) & 0xFF) + h2f(w.y >> 16) * (float)(signed char)((v >> 24) & 0xFF);
      }
    }
    return s * X.dlo;
  }
}

// ---------------------------------------------------------------------------
// Split load / compute form of chunk_dot: the GEMV issues the loads of ALL its
// rows x passes first (WRaw), then does the integer math, so every lane keeps
// NR x 2 independent 16-B loads in flight instead of one at a time.
template <int T> struct WRaw;
template <> struct WRaw<T_Q4_K> { int4 q, m; };
template <> struct WRaw<T_Q5_K> { int4 q, h, m; };
template <> struct WRaw<T_Q6_K> { int4 l, h; int slo, shi; unsigned d; };
template <> struct WRaw<T_Q8_0> { int4 a, b; unsigned d; };
template <> struct WRaw<T_F16> { uint4 w[4]; };
template <> struct WRaw<T_F32> { float4 w[8]; };

// per-row plane pointers (wave-uniform -> SGPRs)
struct RowPtr {
  const uint8_t* p0;
  const uint8_t* p1;
  const uint8_t* p2;
  const uint8_t* p3;
};

__device__ __forceinline__ RowPtr row_ptr(const uint8_t* base, const Planes& P, unsigned row) {
  RowPtr r;
  r.p0 = base + P.p0 + (size_t)row * P.s0;
  r.p1 = base + P.p1 + (size_t)row * P.s1;
  r.p2 = base + P.p2 + (size_t)row * P.s2;
  r.p3 = base + P.p3 + (size_t)row * P.s3;
  return r;
}

template <int T>
__device__ __forceinline__ void wload(WRaw<T>& w, const RowPtr& R, int c) {
  const int sb = c >> 3, j = c & 7;
  if constexpr (T == T_Q4_K) {
    w.q = ld_nt16(R.p0 + 16 * c);
    w.m = *reinterpret_cast<const int4*>(R.p1 + 16 * sb);
  } else if constexpr (T == T_Q5_K) {
    w.q = ld_nt16(R.p0 + 16 * c);
    w.h = *reinterpret_cast<const int4*>(R.p1 + 32 * sb + 16 * (j & 1));
    w.m = *reinterpret_cast<const int4*>(R.p2 + 16 * sb);
  } else if constexpr (T == T_Q6_K) {
    const int n = j >> 2, o = 16 * (j & 3);
    w.l = ld_nt16(R.p0 + 16 * c);
    w.h = *reinterpret_cast<const int4*>(R.p1 + 64 * sb + 32 * n + (o & 31));
    const int si = 8 * n + (o >> 4);
    w.slo = *reinterpret_cast<const signed char*>(R.p2 + 16 * sb + si);
    w.shi = *reinterpret_cast<const signed char*>(R.p2 + 16 * sb + si + 4);
    w.d = *reinterpret_cast<const unsigned short*>(R.p3 + 2 * sb);
  } else if constexpr (T == T_Q8_0) {
    w.a = ld_nt16(R.p0 + 32 * c);
    w.b = ld_nt16(R.p0 + 32 * c + 16);
    w.d = *reinterpret_cast<const unsigned short*>(R.p1 + 2 * c);
  } else if constexpr (T == T_F16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) w.w[i] = reinterpret_cast<const uint4*>(R.p0 + 64 * c)[i];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) w.w[i] = reinterpret_cast<const float4*>(R.p0 + 128 * c)[i];
  }
}

template <int T>
__device__ __forceinline__ float wdot(const WRaw<T>& w, const XChunk& X, int c) {
  const int j = c & 7;
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int g = j >> 1;
    const unsigned dd = (unsigned)w.m.x;
    const float d = h2f(dd & 0xFFFF), dmin = h2f(dd >> 16);
    float sc_lo, m_lo, sc_hi, m_hi;
    scale_min_pair(g, (unsigned)w.m.y, (unsigned)w.m.z, (unsigned)w.m.w, sc_lo, m_lo, sc_hi, m_hi);
    const int qv[4] = {w.q.x, w.q.y, w.q.z, w.q.w};
    int dl = 0, dh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int lo = qv[i] & 0x0F0F0F0F;
      int hi = (qv[i] >> 4) & 0x0F0F0F0F;
      if constexpr (T == T_Q5_K) {
        const int hv = (i == 0 ? w.h.x : i == 1 ? w.h.y : i == 2 ? w.h.z : w.h.w);
        lo |= ((hv >> (2 * g)) & 0x01010101) << 4;
        hi |= ((hv >> (2 * g + 1)) & 0x01010101) << 4;
      }
      dl = dot4(lo, X.lo[i], dl);
      dh = dot4(hi, X.hi[i], dh);
    }
    return d * (sc_lo * X.dlo * (float)dl + sc_hi * X.dhi * (float)dh) - dmin * (m_lo * X.slo + m_hi * X.shi);
  } else if constexpr (T == T_Q6_K) {
    const int o = 16 * (j & 3);
    const int sc_lo = w.slo, sc_hi = w.shi;
    const int s = (o >= 32) ? 2 : 0;
    const int lv[4] = {w.l.x, w.l.y, w.l.z, w.l.w};
    const int hv[4] = {w.h.x, w.h.y, w.h.z, w.h.w};
    int dl = 0, dh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lo = (lv[i] & 0x0F0F0F0F) | (((hv[i] >> s) & 0x03030303) << 4);
      const int hi = ((lv[i] >> 4) & 0x0F0F0F0F) | (((hv[i] >> (s + 4)) & 0x03030303) << 4);
      dl = dot4(lo, X.lo[i], dl);
      dh = dot4(hi, X.hi[i], dh);
    }
    const float d = h2f(w.d & 0xFFFF);
    return d * ((float)sc_lo * (X.dlo * (float)dl - 32.f * X.slo) + (float)sc_hi * (X.dhi * (float)dh - 32.f * X.shi));
  } else if constexpr (T == T_Q8_0) {
    int acc = dot4(w.a.x, X.lo[0], 0);
    acc = dot4(w.a.y, X.lo[1], acc);
    acc = dot4(w.a.z, X.lo[2], acc);
    acc = dot4(w.a.w, X.lo[3], acc);
    acc = dot4(w.b.x, X.hi[0], acc);
    acc = dot4(w.b.y, X.hi[1], acc);
    acc = dot4(w.b.z, X.hi[2], acc);
    acc = dot4(w.b.w, X.hi[3], acc);
    return h2f(w.d & 0xFFFF) * X.dlo * (float)acc;
  } else {
    const int xv[8] = {X.lo[0], X.lo[1], X.lo[2], X.lo[3], X.hi[0], X.hi[1], X.hi[2], X.hi[3]};
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = xv[i];
      const float x0 = (float)(signed char)(v & 0xFF), x1 = (float)(signed char)((v >> 8) & 0xFF);
      const float x2 = (float)(signed char)((v >> 16) & 0xFF), x3 = (float)(signed char)((v >> 24) & 0xFF);
      if constexpr (T == T_F32) {
        const float4 ww = w.w[i];
        s += ww.x * x0 + ww.y * x1 + ww.z * x2 + ww.w * x3;
      } else {
        const uint2 ww = (i & 1) ? make_uint2(w.w[i >> 1].z, w.w[i >> 1].w) : make_uint2(w.w[i >> 1].x, w.w[i >> 1].y);
        s += h2f(ww.x & 0xFFFF) * x0 + h2f(ww.x >> 16) * x1 + h2f(ww.y & 0xFFFF) * x2 + h2f(ww.y >> 16) * x3;
      }
    }
    return s * X.dlo;
  }
}

// Dequantise 32 CONTIGUOUS weights [32*q, 32*q+32) of `row` into out[32] (used by
// the embedding gather and the prefill GEMM's LDS staging).
template <int T>
__device__ __forceinline__ void dequant32(const uint8_t* __restrict__ base, const Planes& P, size_t row, int q,
                                          float* out) {
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int sb = q >> 3, s = q & 7, g = s >> 1, hi = s & 1;  // sub-block s of superblock sb
    const uint8_t* qs_p = base + P.p0 + row * P.s0 + sb * 128 + 32 * g;
    int4 meta;
    int4 qh0, qh1;
    if constexpr (T == T_Q4_K) {
      meta = *reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 16);
    } else {
      const int4* qhp = reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 32);
      qh0 = qhp[0];
      qh1 = qhp[1];
      meta = *reinterpret_cast<const int4*>(base + P.p2 + row * P.s2 + sb * 16);
    }
    const float d = h2f((unsigned)meta.x & 0xFFFF), dmin = h2f((unsigned)meta.x >> 16);
    float sc_lo, m_lo, sc_hi, m_hi;
    scale_min_pair(g, (unsigned)meta.y, (unsigned)meta.z, (unsigned)meta.w, sc_lo, m_lo, sc_hi, m_hi);
    const float scl = d * (hi ? sc_hi : sc_lo), mn = dmin * (hi ? m_hi : m_lo);
    const int4 a = reinterpret_cast<const int4*>(qs_p)[0];
    const int4 b = reinterpret_cast<const int4*>(qs_p)[1];
    const int qv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int hv[8] = {qh0.x, qh0.y, qh0.z, qh0.w, qh1.x, qh1.y, qh1.z, qh1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int v = hi ? ((qv[i] >> 4) & 0x0F0F0F0F) : (qv[i] & 0x0F0F0F0F);
      if constexpr (T == T_Q5_K) v |= ((hv[i] >> s) & 0x01010101) << 4;
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) out[4 * i + b8] = scl * (float)((v >> (8 * b8)) & 0xFF) - mn;
    }
  } else if constexpr (T == T_Q6_K) {
    const int sb = q >> 3, r = q & 7;        // 32-run r of the superblock
    const int n = r >> 2, qq = (r >> 1) & 1, half = r & 1;
    const uint8_t* qlp = base + P.p0 + row * P.s0 + sb * 128 + 64 * n + 32 * half;
    const uint8_t* qhp = base + P.p1 + row * P.s1 + sb * 64 + 32 * n;
    const int4 scv = *reinterpret_cast<const int4*>(base + P.p2 + row * P.s2 + sb * 16);
    const float d = h2f(*reinterpret_cast<const unsigned short*>(base + P.p3 + row * P.s3 + sb * 2));
    const int scw[4] = {scv.x, scv.y, scv.z, scv.w};
    const int si = 8 * n + 2 * (2 * qq + half);
    const float s0 = d * (float)(signed char)((scw[si >> 2] >> (8 * (si & 3))) & 0xFF);
    const float s1 = d * (float)(signed char)((scw[(si + 1) >> 2] >> (8 * ((si + 1) & 3))) & 0xFF);
    const int4 la = reinterpret_cast<const int4*>(qlp)[0], lb = reinterpret_cast<const int4*>(qlp)[1];
    const int4 ha = reinterpret_cast<const int4*>(qhp)[0], hb = reinterpret_cast<const int4*>(qhp)[1];
    const int lv[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
    const int hv[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    const int hs = 2 * (2 * qq + half);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = ((lv[i] >> (4 * qq)) & 0x0F0F0F0F) | (((hv[i] >> hs) & 0x03030303) << 4);
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) out[4 * i + b8] = (i < 4 ? s0 : s1) * (float)(((v >> (8 * b8)) & 0xFF) - 32);
    }
  } else if constexpr (T == T_Q8_0) {
    const int4* qp = reinterpret_cast<const int4*>(base + P.p0 + row * P.s0 + 32 * q);
    const int4 a = qp[0], b = qp[1];
    const float d = h2f(*reinterpret_cast<const unsigned short*>(base + P.p1 + row * P.s1 + 2 * q));
    const int qv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) out[4 * i + b8] = d * (float)(signed char)((qv[i] >> (8 * b8)) & 0xFF);
  } else if constexpr (T == T_F32) {
    const float4* wp = reinterpret_cast<const float4*>(base + row * P.s0 + 128 * q);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float4 w = wp[i];
      out[4 * i] = w.x; out[4 * i + 1] = w.y; out[4 * i + 2] = w.z; out[4 * i + 3] = w.w;
    }
  } else {  // F16
    const uint2* wp = reinterpret_cast<const uint2*>(base + row * P.s0 + 64 * q);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint2 w = wp[i];
      out[4 * i] = h2f(w.x & 0xFFFF); out[4 * i + 1] = h2f(w.x >> 16);
      out[4 * i + 2] = h2f(w.y & 0xFFFF); out[4 * i + 3] = h2f(w.y >> 16);
    }
  }
}

// ---------------------------------------------------------------------------
// Split form of dequant32 for software-pipelined GEMM staging: dq_load issues
// the raw loads of one 32-weight run (registers), dq_decode turns them into 32
// floats later, so the loads of K-step k+1 fly while step k's MFMAs run.
template <int T> struct DqRaw;
template <> struct DqRaw<T_Q4_K> { int4 a, b, m; };
template <> struct DqRaw<T_Q5_K> { int4 a, b, m, h0, h1; };
template <> struct DqRaw<T_Q6_K> { int4 la, lb, ha, hb, sc; unsigned d; };
template <> struct DqRaw<T_Q8_0> { int4 a, b; unsigned d; };
template <> struct DqRaw<T_F16> { uint4 w[4]; };
template <> struct DqRaw<T_F32> { float4 w[8]; };

template <int T>
__device__ __forceinline__ void dq_load(DqRaw<T>& r, const uint8_t* __restrict__ base, const Planes& P, size_t row,
                                        int q) {
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int sb = q >> 3, g = (q & 7) >> 1;
    const int4* qs = reinterpret_cast<const int4*>(base + P.p0 + row * P.s0 + sb * 128 + 32 * g);
    r.a = qs[0];
    r.b = qs[1];
    if constexpr (T == T_Q4_K) {
      r.m = *reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 16);
    } else {
      const int4* qh = reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 32);
      r.h0 = qh[0];
      r.h1 = qh[1];
      r.m = *reinterpret_cast<const int4*>(base + P.p2 + row * P.s2 + sb * 16);
    }
  } else if constexpr (T == T_Q6_K) {
    const int sb = q >> 3, rr = q & 7, n = rr >> 2, half = rr & 1;
    const int4* l = reinterpret_cast<const int4*>(base + P.p0 + row * P.s0 + sb * 128 + 64 * n + 32 * half);
    const int4* h = reinterpret_cast<const int4*>(base + P.p1 + row * P.s1 + sb * 64 + 32 * n);
    r.la = l[0]; r.lb = l[1];
    r.ha = h[0]; r.hb = h[1];
    r.sc = *reinterpret_cast<const int4*>(base + P.p2 + row * P.s2 + sb * 16);
    r.d = *reinterpret_cast<const unsigned short*>(base + P.p3 + row * P.s3 + sb * 2);
  } else if constexpr (T == T_Q8_0) {
    const int4* qp = reinterpret_cast<const int4*>(base + P.p0 + row * P.s0 + 32 * q);
    r.a = qp[0];
    r.b = qp[1];
    r.d = *reinterpret_cast<const unsigned short*>(base + P.p1 + row * P.s1 + 2 * q);
  } else if constexpr (T == T_F16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.w[i] = reinterpret_cast<const uint4*>(base + row * P.s0 + 64 * q)[i];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = reinterpret_cast<const float4*>(base + row * P.s0 + 128 * q)[i];
  }
}

template <int T>
__device__ __forceinline__ void dq_decode(const DqRaw<T>& r, int q, float* out) {
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int s = q & 7, hi = s & 1;
    const float d = h2f((unsigned)r.m.x & 0xFFFF), dmin = h2f((unsigned)r.m.x >> 16);
    // this lane's one 6-bit (scale, min) pair, branch-free (s differs per lane; a branch here
    // would also split the GEMM's MFMA/decode scheduling region)
    const unsigned y = r.m.y, z = r.m.z, w = r.m.w;
    const int sh = 8 * (s & 3);
    const unsigned sc_a = (y >> sh) & 63, m_a = (z >> sh) & 63;
    const unsigned sc_b = ((w >> sh) & 0xF) | (((y >> (sh + 6)) & 3) << 4);
    const unsigned m_b = ((w >> (sh + 4)) & 0xF) | (((z >> (sh + 6)) & 3) << 4);
    const float scl = d * (float)(s >= 4 ? sc_b : sc_a), mn = dmin * (float)(s >= 4 ? m_b : m_a);
    const int qv[8] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int v = hi ? ((qv[i] >> 4) & 0x0F0F0F0F) : (qv[i] & 0x0F0F0F0F);
      if constexpr (T == T_Q5_K) {
        const int hv = i < 4 ? (i == 0 ? r.h0.x : i == 1 ? r.h0.y : i == 2 ? r.h0.z : r.h0.w)
                             : (i == 4 ? r.h1.x : i == 5 ? r.h1.y : i == 6 ? r.h1.z : r.h1.w);
        v |= ((hv >> s) & 0x01010101) << 4;
      }
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) out[4 * i + b8] = scl * (float)((v >> (8 * b8)) & 0xFF) - mn;
    }
  } else if constexpr (T == T_Q6_K) {
    const int rr = q & 7, n = rr >> 2, qq = (rr >> 1) & 1, half = rr & 1;
    const float d = h2f(r.d & 0xFFFF);
    const int scw[4] = {r.sc.x, r.sc.y, r.sc.z, r.sc.w};
    const int si = 8 * n + 2 * (2 * qq + half);
    const float s0 = d * (float)(signed char)((scw[si >> 2] >> (8 * (si & 3))) & 0xFF);
    const float s1 = d * (float)(signed char)((scw[(si + 1) >> 2] >> (8 * ((si + 1) & 3))) & 0xFF);
    const int lv[8] = {r.la.x, r.la.y, r.la.z, r.la.w, r.lb.x, r.lb.y, r.lb.z, r.lb.w};
    const int hv[8] = {r.ha.x, r.ha.y, r.ha.z, r.ha.w, r.hb.x, r.hb.y, r.hb.z, r.hb.w};
    const int hs = 2 * (2 * qq + half);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = ((lv[i] >> (4 * qq)) & 0x0F0F0F0F) | (((hv[i] >> hs) & 0x03030303) << 4);
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) out[4 * i + b8] = (i < 4 ? s0 : s1) * (float)(((v >> (8 * b8)) & 0xFF) - 32);
    }
  } else if constexpr (T == T_Q8_0) {
    const float d = h2f(r.d & 0xFFFF);
    const int qv[8] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) out[4 * i + b8] = d * (float)(signed char)((qv[i] >> (8 * b8)) & 0xFF);
  } else if constexpr (T == T_F16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned w[4] = {r.w[i].x, r.w[i].y, r.w[i].z, r.w[i].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        out[8 * i + 2 * j] = h2f(w[j] & 0xFFFF);
        out[8 * i + 2 * j + 1] = h2f(w[j] >> 16);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      out[4 * i] = r.w[i].x; out[4 * i + 1] = r.w[i].y; out[4 * i + 2] = r.w[i].z; out[4 * i + 3] = r.w[i].w;
    }
  }
}

// Dispatch helper: call F.template operator()<T>() for the runtime type (wave-uniform).
#define LFK_DISPATCH_TYPE(t, ...)                          \
  switch (t) {                                             \
    case T_Q4_K: { constexpr int QT = T_Q4_K; __VA_ARGS__; } break; \
    case T_Q5_K: { constexpr int QT = T_Q5_K; __VA_ARGS__; } break; \
    case T_Q6_K: { constexpr int QT = T_Q6_K; __VA_ARGS__; } break; \
    case T_Q8_0: { constexpr int QT = T_Q8_0; __VA_ARGS__; } break; \
    case T_F16: { constexpr int QT = T_F16; __VA_ARGS__; } break;   \
    default: { constexpr int QT = T_F32; __VA_ARGS__; } break;      \
  }

}  // namespace lfk
