// Device building blocks shared by the decode GEMV kernels (gemv.hip, moe.hip,
// bmm.hip): the x prologue (RMSNorm + q8 into LDS), the
// per-wave weight stream, the cross-lane row reduction and item -> row mapping.
#pragma once
#include "kernels.h"
#include "qdot.h"

namespace lfk {

static constexpr int kMaxBlocks = 1024;  // 256 CUs x 4

// Block prologue: x (or x * w_norm) -> per-32 int8 + f32 scale in LDS.
//
// Split in two so its global loads are issued BEFORE the wave's first weight
// loads (vmcnt retires in order: an x load queued behind a weight stream would
// make the prologue wait for the weights):
//   load()   : every thread issues its first NB float4 of x (and w_norm);
//   finish() : per-32 amax on DPP, q8 -> LDS, sum of squares -> one barrier.
// RMSNorm's 1/rms is a scalar, so q8(x * w) equals q8(x * w / rms) up to the
// block scale: the kernel multiplies its final dot products by the returned
// scale instead of making a second pass over x.
typedef unsigned xp_v4u __attribute__((ext_vector_type(4)));
// 16-B load with sc1 (L1 bypassed; agent-coherent with sc1 producer stores of the same launch)
__device__ __forceinline__ float4 ld16f_sc1(const float* base, int i) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7FFFFFFF, 0x00020000);
  const xp_v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, i * (int)sizeof(float), 0, 16);  // aux 16: sc1
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

template <bool NORM, int BLOCK = 256, bool SC1 = false>
struct XPrologue {
  static constexpr int NB = 4;
  static constexpr int SHIFT = (BLOCK == 1024) ? 12 : (BLOCK == 512 ? 11 : 10);  // log2(BLOCK * 4 floats per slot)
  float4 v[NB], w[NB];
  __device__ __forceinline__ void load_batch(const float* __restrict__ x, const float* __restrict__ nw, int K, int j0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = ((j0 + b) << SHIFT) + tid * 4;
      if constexpr (SC1) v[b] = i < K ? ld16f_sc1(x, i) : make_float4(0.f, 0.f, 0.f, 0.f);
      else v[b] = i < K ? *reinterpret_cast<const float4*>(x + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (NORM) w[b] = i < K ? *reinterpret_cast<const float4*>(nw + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ __forceinline__ void load(const float* __restrict__ x, const float* __restrict__ nw, int K) {
    load_batch(x, nw, K, 0);
  }
  // q8-quantise the NB batch slots starting at j0 (already in registers) into LDS
  __device__ __forceinline__ void quant_batch(int j0, int K, int8_t* xq, float* xd, float& ss) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = ((j0 + b) << SHIFT) + tid * 4;
      if (i < K) {
        float4 t = v[b];
        if constexpr (NORM) {
          ss += t.x * t.x + t.y * t.y + t.z * t.z + t.w * t.w;
          t.x *= w[b].x; t.y *= w[b].y; t.z *= w[b].z; t.w *= w[b].w;
        }
        const float amax = max8(fmaxf(fmaxf(fabsf(t.x), fabsf(t.y)), fmaxf(fabsf(t.z), fabsf(t.w))));
        const float d = amax * (1.f / 127.f);
        const float id = d > 0.f ? 1.f / d : 0.f;
        const int q0 = __float2int_rn(t.x * id), q1 = __float2int_rn(t.y * id);
        const int q2 = __float2int_rn(t.z * id), q3 = __float2int_rn(t.w * id);
        *reinterpret_cast<int*>(xq + i) =
            (q0 & 0xFF) | ((q1 & 0xFF) << 8) | ((q2 & 0xFF) << 16) | ((q3 & 0xFF) << 24);
        if ((tid & 7) == 0) xd[i >> 5] = d;
      }
    }
  }
  // returns the RMSNorm scale (1 without NORM). The first NB batch slots (issued
  // by load()) are consumed in straight-line code, so that when weight loads were
  // issued between load() and finish() the compiler's wait covers only the x
  // loads (vmcnt = number of weight loads) instead of draining the weights too.
  __device__ __forceinline__ float finish(const float* __restrict__ x, const float* __restrict__ nw, float eps, int K,
                                          int8_t* xq, float* xd, float* red) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nj = (K + (1 << SHIFT) - 1) >> SHIFT;
    float ss = 0.f;
    quant_batch(0, K, xq, xd, ss);
    for (int j0 = NB; j0 < nj; j0 += NB) {
      load_batch(x, nw, K, j0);
      quant_batch(j0, K, xq, xd, ss);
    }
    if constexpr (NORM) {
      ss = wave_sum_fast(ss);
      if (lane == 0) red[wave] = ss;
    }
    __syncthreads();
    if constexpr (NORM) {
      float tot = 0.f;
#pragma unroll
      for (int i = 0; i < BLOCK / 64; ++i) tot += red[i];
      return rsqrtf(tot / (float)K + eps);
    }
    return 1.f;
  }
};

// one-call form (MoE down, where there is no weight prefetch to order against)
template <bool NORM>
__device__ __forceinline__ float quantize_x(const float* __restrict__ x, const float* __restrict__ nw, float eps, int K,
                                            int8_t* xq, float* xd, float* red) {
  XPrologue<NORM> xp;
  xp.load(x, nw, K);
  return xp.finish(x, nw, eps, K, xq, xd, red);
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// Weight stream of one wave item: NR rows x U passes of 64 chunks, all loads
// issued before any math (NR*U independent 16-B loads per lane in flight).
// Chunks past the row end are clamped (loaded from the last chunk, ignored).
template <int QT, int NR, int U>
struct WStream {
  WRaw<QT> w[U][NR];
  __device__ __forceinline__ void load(const RowPtr (&R)[NR], int c0, int nchunks, int lane) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(c0 + 64 * u + lane, nchunks - 1);
#pragma unroll
      for (int r = 0; r < NR; ++r) wload<QT>(w[u][r], R[r], c);
    }
  }
  __device__ __forceinline__ void dot(int c0, int nchunks, const int8_t* xq, const float* xd, float (&acc)[NR],
                                      int lane) const {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + 64 * u + lane;
      if (c < nchunks) {
        XChunk X;
        load_x<QT>(X, xq, xd, c);
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r] += wdot<QT>(w[u][r], X, c);
      }
    }
  }
  // rest of the row after the first pass group was loaded by the caller
  __device__ __forceinline__ void finish_rows(const RowPtr (&R)[NR], int nchunks, const int8_t* xq, const float* xd,
                                              float (&acc)[NR], int lane) {
    for (int c0 = 0;;) {
      dot(c0, nchunks, xq, xd, acc, lane);
      c0 += 64 * U;
      if (c0 >= nchunks) break;
      load(R, c0, nchunks, lane);
    }
  }
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Reduce NR per-lane partial sums over the wave so that lane l ends up with the
// total of row (l % NR): a butterfly over offsets 32..NR, then a transposing
// exchange for the last log2(NR) offsets (no dynamic register indexing).
template <int NR>
__device__ __forceinline__ float reduce_rows(float (&acc)[NR], int lane) {
#pragma unroll
  for (int o = 32; o >= NR; o >>= 1)
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] += __shfl_xor(acc[r], o);
  if constexpr (NR == 1) {
    return acc[0];
  } else if constexpr (NR == 2) {
    const bool hi = lane & 1;
    float z = hi ? acc[1] : acc[0];
    const float w = hi ? acc[0] : acc[1];
    return z + __shfl_xor(w, 1);
  } else {
    static_assert(NR == 4, "rows per item must be 1, 2 or 4");
    const bool b1 = lane & 2;
    float x0 = b1 ? acc[2] : acc[0], x1 = b1 ? acc[3] : acc[1];
    const float y0 = b1 ? acc[0] : acc[2], y1 = b1 ? acc[1] : acc[3];
    x0 += __shfl_xor(y0, 2);
    x1 += __shfl_xor(y1, 2);
    const bool b0 = lane & 1;
    const float z = b0 ? x1 : x0, w = b0 ? x0 : x1;
    return z + __shfl_xor(w, 1);
  }
}

// ids: the slots' expert indices (a.expert_ids, or the routed GEMV's LDS copy)
template <int EPI, int NR>
__device__ __forceinline__ void item_rows(const GemvArgs& a, int it, int groups, RowPtr (&R)[NR], int& slot, int& f0,
                                          const int* ids) {
  constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
  slot = it / groups;
  f0 = (it - slot * groups) * NF;
  const uint8_t* base = a.w.base;
  if (ids) base += (size_t)ids[slot] * a.w.expert_stride;
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    if constexpr (EPI == EPI_SWIGLU) {
      const int f = f0 + r;
      const unsigned gr = (unsigned)((f >> 5) * 64 + (f & 31));
      R[r] = row_ptr(base, a.w.P, gr);
      R[NF + r] = row_ptr(base, a.w.P, gr + 32);
    } else {
      R[r] = row_ptr(base, a.w.P, (unsigned)min(f0 + r, a.n_out - 1));
    }
  }
}


}  // namespace lfk
