// Decode attention body (split-L flash decoding) shared by attention.hip's attn_decode_kernel
// and bmm.hip's fused attention + Wo launch (attn_wo_kernel). See attention.hip for the design.
#pragma once
#include <cfloat>

#include "kernels.h"
#include "qdot.h"

namespace lfk {

// bmm's k order inside each 4-group: (0, 2, 1, 3) (kernels/bmm.hip)
__device__ __forceinline__ int swz4(int i) { return (i & ~3) | ((i & 1) << 1) | ((i >> 1) & 1); }


static constexpr int CH = 64;  // keys per split

// L2-coherent 4-B store / load (global_store/load ... sc1): the cross-block
// hand-off of split partials needs no agent-scope fence when every byte of it
// goes through these (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same for an 8-byte aligned pair (one dwordx2 access instead of two)
__device__ __forceinline__ void st2_sc1(float* p, float a, float b) {
  const unsigned long long v = ((unsigned long long)__float_as_uint(b) << 32) | __float_as_uint(a);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld2_sc1(const float* p) {
  const unsigned long long v = __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<float*>(p)),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)));
}

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
// c ? a : b per component (a ternary on the uint4 structs, or a conditional overwrite of a load's
// registers, made the compiler keep the K / V load registers in a stack array or wait for every
// outstanding load)
__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b) {
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Cross-lane helpers without the LDS crossbar: DPP within a row of 16 lanes,
// v_readlane across rows (the reduction trees below are 2-4 steps, each a few
// cycles instead of a ds_bpermute round trip).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_sum(float v) {  // sum over the 4 lanes of a quad
  v += dpp<0xB1>(v);                                   // quad_perm [1,0,3,2]
  return v + dpp<0x4E>(v);                             // quad_perm [2,3,0,1]
}
__device__ __forceinline__ float rowq_max(float v) {  // max over lanes i, i+4, i+8, i+12 of a row
  v = fmaxf(v, dpp<0x124>(v));                         // row_ror:4
  return fmaxf(v, dpp<0x128>(v));                      // row_ror:8
}
__device__ __forceinline__ float rowq_sum(float v) {
  v += dpp<0x124>(v);
  return v + dpp<0x128>(v);
}
__device__ __forceinline__ float rows_max(float v) {  // combine the 4 rows (wave-uniform result)
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
__device__ __forceinline__ float rows_sum(float v) {
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// One block = 64 keys of one kv head x all G query heads sharing it; 4 waves of
// 16 keys, lane = (key = lane/4, sub = lane%4) holding HD/4 dims of its key.
//   1. K/V row loads go out first, clamped to the cache (speculative: they do
//      not wait for the device-resident position), q goes to LDS;
//   2. per wave: scores (quad DPP reduce), wave-local softmax (DPP + readlane),
//      P.V over the wave's 16 keys from LDS - no block barrier;
//   3. the 4 wave partials meet in LDS (one barrier) -> block partial;
//   4. single split: normalise and store. Otherwise the partial goes out with
//      sc1 stores and the last-arriving block of the kv head merges all splits
//      (sc1 loads; no cache-maintenance fences).
template <int HD, int G, bool TL>
__device__ __forceinline__ void attn_decode_body(AttnDecodeArgs a) {
  constexpr int DPL = HD / 4;   // dims per lane in QK
  constexpr int NLD = DPL / 8;  // 16-B loads per lane per K (or V) row
  constexpr int KPW = 16;       // keys per wave
  // TL: timeline instrumentation (microbenchmarks; a separate instantiation so
  // the production kernel's code generation is untouched)
  // TL: per-block wall_clock64 stamps (absolute), dbg_clk[16 * linear block + i]: 0 entry, 1 loads
  // issued + position read, 2 V staged, 3 wave partials met, 4 block partial stored, 5 split
  // counter taken, 8 / 9 merge start / end (merging block), 7 exit
  const bool stamp = TL && threadIdx.x == 0;
  long long* const tl = TL ? a.dbg_clk + 16 * ((size_t)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) : nullptr;
#define LFK_STAMP(i) do { if constexpr (TL) { if (stamp) tl[(i) + 1] = wall_clock64(); } } while (0)
  if constexpr (TL) { if (stamp) { tl[0] = wall_clock64(); tl[15] = xcc_id(); } }
  // the prologue's kernarg fields in one scalar batch (as bmm's and gemv's prologues): read where
  // first used they were three dependent round trips before the first K / V load, not two
  asm volatile("" ::"s"(a.q), "s"(a.k_cache), "s"(a.v_cache), "s"(a.pos), "s"(a.n_ctx), "s"(a.n_head), "s"(a.scale),
               "s"(a.part), "s"(a.counters), "s"(a.out), "s"(a.debug_stop), "s"(a.batch), "s"(a.slots),
               "s"(a.slot_stride), "s"(a.q_stride), "s"(a.out_stride), "s"(a.part_stride), "s"(a.out_h),
               "s"(a.out_h_stride), "s"(a.done), "s"(a.qkv_raw), "s"(a.qkv_ld), "s"(a.k_off), "s"(a.v_off), "s"(a.ss),
               "s"(a.inv_k), "s"(a.eps), "s"(a.rope_freq));
  if ((int)blockIdx.z == (a.batch > 0 ? a.batch : 1)) {  // weight-touch plane (see AttnDecodeArgs::pf)
    const int nb = gridDim.x * gridDim.y, b = blockIdx.y * gridDim.x + blockIdx.x;
    uint32_t acc = 0;
    for (int r = 0; r < AttnDecodeArgs::kTouchRanges; ++r) {
      if (!a.pf[r]) continue;
      const size_t lps = (a.pf_bytes[r] + 127) / 128;  // lines per segment
      const size_t nl = lps * a.pf_nseg[r], per = (nl + nb - 1) / nb;
      const size_t beg = (size_t)b * per, end = min(nl, beg + per), last_dw = a.pf_bytes[r] / 4 - 1;
#pragma unroll 4
      for (size_t i = beg + threadIdx.x; i < end; i += 256) {
        const size_t seg = i / lps;
        const uint32_t* p = reinterpret_cast<const uint32_t*>(a.pf[r] + seg * a.pf_seg_stride[r]);
        acc ^= p[min((i - seg * lps) * 32, last_dw)];
      }
    }
    if (acc == 0x9E3779B9u) *a.pf_sink = (int)acc;
    return;
  }
  if (a.batch > 0) {  // batched decode: this row's query, KV slot, position, workspaces and output
    const int b = blockIdx.z;
    const size_t so = (size_t)a.slots[b] * a.slot_stride;
    a.q += (size_t)b * a.q_stride;
    a.k_cache += so;
    a.v_cache += so;
    a.pos += b;
    a.part += (size_t)b * a.part_stride;
    a.counters += 64 * b;
    if (a.out) a.out += (size_t)b * a.out_stride;
    if (a.out_h) a.out_h += (size_t)b * a.out_h_stride;
    if (a.qkv_raw) a.qkv_raw += (size_t)b * a.qkv_ld;
  }
  // split-K Q|K|V (batched): q / k / v are RoPE'd unnormalised sums, this row's RMSNorm scale is
  // applied here (q is read from the raw sums)
  if (a.qkv_raw) a.q = a.qkv_raw;
  const int kvh = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kw = lane >> 2, sub = lane & 3;
  const int start = split * CH;
  const int key = start + wave * KPW + kw;

  __shared__ __attribute__((aligned(16))) h2v qs[G][HD / 2];   // q * scale in f16 pairs
  __shared__ __attribute__((aligned(16))) __half vs[4][KPW][HD + 8];
  __shared__ __attribute__((aligned(16))) float ps[4][G][KPW];
  __shared__ float wm[4][G], wl[4][G];
  __shared__ __attribute__((aligned(16))) float wo[4][G][HD];
  __shared__ int last;
  __shared__ __attribute__((aligned(16))) h2v kvn[2][HD / 2];  // split-K Q|K|V: the new key / value (f16)

  // ---- 1. loads: q (and the split-K new key / value) first, then the K / V rows
  //      (speculative: they do not wait for the device-resident position), so q goes to LDS
  //      while K / V are in flight, the scores wait for K only and P.V for V
  constexpr int QPT = (G * HD / 2 + 255) / 256;  // q pairs per thread
  float2 qv[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int i = min(tid + 256 * j, G * HD / 2 - 1);
    qv[j] = reinterpret_cast<const float2*>(a.q + (size_t)kvh * G * HD)[i];
  }
  // split-K Q|K|V: the row's sum of squares (a VECTOR load beside q - a scalar one at the top was one
  // more dependent round trip before any K / V load went out), the new key / value pairs and, RoPE
  // deferred, the pairs' frequencies - all issued unconditionally (from q when unused) and before
  // K / V, so that waiting for them never waits for the K / V rows
  const bool raw = a.qkv_raw != nullptr, drope = raw && a.rope_freq != nullptr;
  const float ssv = __hip_atomic_load(const_cast<float*>(raw ? a.ss + (a.batch > 0 ? blockIdx.z : 0) : a.q),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int kvsel = tid / (HD / 2), pr = tid % (HD / 2);
  const float2 nv = reinterpret_cast<const float2*>(
      raw && tid < HD ? a.qkv_raw + (kvsel ? a.v_off : a.k_off) + (size_t)kvh * HD : a.q)[raw && tid < HD ? pr : 0];
  float fq[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) fq[j] = (drope ? a.rope_freq : a.q)[drope ? min(tid + 256 * j, G * HD / 2 - 1) % (HD / 2) : 0];
  const size_t row = ((size_t)kvh * a.n_ctx + min(key, a.n_ctx - 1)) * HD + sub * DPL;
  uint4 kr[NLD], vr[NLD];
#pragma unroll
  for (int i = 0; i < NLD; ++i) kr[i] = *reinterpret_cast<const uint4*>(a.k_cache + row + 8 * i);
#pragma unroll
  for (int i = 0; i < NLD; ++i) vr[i] = *reinterpret_cast<const uint4*>(a.v_cache + row + 8 * i);
  const float rs = raw ? rsqrtf(ssv * a.inv_k + a.eps) : 1.f;
  const float qscale = a.scale * rs;
  // deferred RoPE (adjacent pairs): angle = pos * freq in fp32, as llama.cpp computes it
  const float pf = (float)min(max(*a.pos, 0), a.n_ctx - 1);
  auto rot = [&](float2 v, float f) {
    if (!drope) return v;
    float sn, cs;
    sincosf(pf * f, &sn, &cs);
    return make_float2(v.x * cs - v.y * sn, v.x * sn + v.y * cs);
  };
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int i = tid + 256 * j;
    const float2 q2 = rot(qv[j], fq[j]);
    if (i < G * HD / 2) qs[i / (HD / 2)][i % (HD / 2)] = h2v{(_Float16)(q2.x * qscale), (_Float16)(q2.y * qscale)};
  }
  if (raw && tid < HD) {
    const float2 n2 = tid < HD / 2 ? rot(nv, fq[0]) : nv;  // (fq[0]: pair tid % (HD / 2) = tid here)
    kvn[tid / (HD / 2)][tid % (HD / 2)] = h2v{(_Float16)(n2.x * rs), (_Float16)(n2.y * rs)};
  }
  const int L = min(*a.pos + 1, a.n_ctx);
  LFK_STAMP(0);
  if (start >= L || a.debug_stop == 1) return;

  const int ns = (L + CH - 1) / CH;
  __syncthreads();  // qs, kvn
  LFK_STAMP(1);
  // the new position (split-K Q|K|V): its cache rows are written here from the LDS copy (this
  // launch's only reader of them is this lane; write-through stores), and its key / value slices
  // replace the speculatively loaded stale rows where they are used - not by writing into the K / V
  // load registers (a conditional overwrite of those made the wave wait for every load first)
  const bool newkey = a.qkv_raw && key == L - 1;
  // block-uniform: only the block whose 64 keys hold the new position reads the LDS copies
  const bool newblk = a.qkv_raw && start <= L - 1 && L - 1 < start + CH;
  const uint4* kn = reinterpret_cast<const uint4*>(&kvn[0][sub * (DPL / 2)]);
  const uint4* vn = reinterpret_cast<const uint4*>(&kvn[1][sub * (DPL / 2)]);
  if (newkey) {
    const auto rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(a.k_cache), 0, 0x7FFFFFFF, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(a.v_cache), 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int off = (int)((row + 8 * i) * sizeof(__half));
      const uint4 kk = kn[i], vv = vn[i];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, kk), rk, off, 0, 16);  // aux 16: sc1
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, vv), rv, off, 0, 16);
    }
  }
  if (a.debug_stop == 2) {
    if ((float)qs[0][sub][0] == 1234.f) a.out[tid] = 1.f;
    return;
  }

  // ---- 2a. scores
  const bool valid = key < L;
  // K row slice as f16 pairs, dotted with f16 q on v_dot2_f32_f16 (f32 accumulate)
  h2v kh[DPL / 2];
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const uint4 k4 = newblk ? sel4(newkey, kn[i], kr[i]) : kr[i];
    kh[4 * i] = __builtin_bit_cast(h2v, k4.x);
    kh[4 * i + 1] = __builtin_bit_cast(h2v, k4.y);
    kh[4 * i + 2] = __builtin_bit_cast(h2v, k4.z);
    kh[4 * i + 3] = __builtin_bit_cast(h2v, k4.w);
  }
  float sc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint4* q4 = reinterpret_cast<const uint4*>(&qs[g][sub * (DPL / 2)]);
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const uint4 qq = q4[i];
      p0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.x), kh[4 * i], p0, false);
      p1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.y), kh[4 * i + 1], p1, false);
      p0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.z), kh[4 * i + 2], p0, false);
      p1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.w), kh[4 * i + 3], p1, false);
    }
    sc[g] = quad_sum(p0 + p1);
  }
  // ---- 2b. wave-local softmax over the wave's 16 keys
  float mw[G], lw[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float s = valid ? sc[g] : -FLT_MAX;
    mw[g] = rows_max(rowq_max(s));
    const float e = valid ? __expf(s - mw[g]) : 0.f;
    sc[g] = e;
    lw[g] = rows_sum(rowq_sum(e));
  }
  if (sub == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) ps[wave][g][kw] = sc[g];
  }
  // this wave's V rows (the wave's own keys: a wave barrier, no block barrier)
#pragma unroll
  for (int i = 0; i < NLD; ++i) {  // (the new position: its value in place of the stale cache row)
    *reinterpret_cast<uint4*>(&vs[wave][kw][sub * DPL + 8 * i]) = newblk ? sel4(newkey, vn[i], vr[i]) : vr[i];
  }
  LFK_STAMP(2);
  // ---- 2c. P.V over this wave's keys (LDS written by this wave only)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int DV = HD / 64;  // dims per lane in PV (1 or 2)
  float o[G][DV];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < DV; ++j) o[g][j] = 0.f;
  // the weights of 4 keys per head in one 16-byte LDS read (16 instead of 64 reads at G = 4)
#pragma unroll
  for (int k4 = 0; k4 < KPW; k4 += 4) {
    float4 pg[G];
#pragma unroll
    for (int g = 0; g < G; ++g) pg[g] = *reinterpret_cast<const float4*>(&ps[wave][g][k4]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = k4 + kk;
      float v[DV];
      if constexpr (DV == 2) {
        const __half2 h2 = *reinterpret_cast<const __half2*>(&vs[wave][k][2 * lane]);
        v[0] = __low2float(h2);
        v[1] = __high2float(h2);
      } else {
        v[0] = __half2float(vs[wave][k][lane]);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = kk == 0 ? pg[g].x : kk == 1 ? pg[g].y : kk == 2 ? pg[g].z : pg[g].w;
#pragma unroll
        for (int j = 0; j < DV; ++j) o[g][j] += p * v[j];
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int j = 0; j < DV; ++j) wo[wave][g][DV * lane + j] = o[g][j];
    if (lane == 0) {
      wm[wave][g] = mw[g];
      wl[wave][g] = lw[g];
    }
  }
  __syncthreads();
  LFK_STAMP(3);
  if (a.debug_stop == 3) {
    if (tid < G) a.out[tid] = wl[0][tid];
    return;
  }
  // ---- 3. block partial: a pair of adjacent dims (g, d, d + 1) per thread (8-byte sc1 stores;
  //      the (M, l) statistics of a head are one pair too - HD + 2 keeps every pair aligned)
  for (int e2 = tid; e2 < G * HD / 2; e2 += 256) {
    const int g = (2 * e2) / HD, d = (2 * e2) % HD;
    const float M = fmaxf(fmaxf(wm[0][g], wm[1][g]), fmaxf(wm[2][g], wm[3][g]));
    float l = 0.f, acc0 = 0.f, acc1 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = wm[w][g] == -FLT_MAX ? 0.f : __expf(wm[w][g] - M);
      l += f * wl[w][g];
      acc0 += f * wo[w][g][d];
      acc1 += f * wo[w][g][d + 1];
    }
    if (ns == 1) {
      const int o = (kvh * G + g) * HD + d;
      if (a.out && a.done) {
        st2_sc1(a.out + o, acc0 / l, acc1 / l);  // an in-flight consumer reads it (attn_wo1)
      } else if (a.out) {
        a.out[o] = acc0 / l;
        a.out[o + 1] = acc1 / l;
      }
      if (a.out_h) {
        a.out_h[swz4(o)] = __float2half(acc0 / l);
        a.out_h[swz4(o + 1)] = __float2half(acc1 / l);
      }
    } else {
      float* dst = a.part + ((size_t)split * a.n_head + kvh * G + g) * (HD + 2);
      st2_sc1(dst + d, acc0, acc1);
      if (d == 0) st2_sc1(dst + HD, M, l);
    }
  }
  LFK_STAMP(4);
  if (ns == 1 && a.done) {  // (single row) the f32 output went out sc1 above: one add for the block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(a.done + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (ns == 1 || a.debug_stop == 4) return;

  // ---- 4. hand-off: the last arriving block of this kv head merges all splits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(a.counters + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (prev == ns - 1);
    if (last) __hip_atomic_store(a.counters + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  LFK_STAMP(5);
  if constexpr (TL) { if (last && threadIdx.x == 0) tl[8] = wall_clock64(); }
  if (!last) return;
  // every element's split values and the split statistics are loaded in one
  // batch of independent sc1 loads (one memory round trip per 16 splits). A thread
  // takes EPT adjacent dims of ONE head, so the split statistics (m, l) are loaded
  // once per thread, not once per element: 64 instead of 96 VGPRs of loads at G = 4,
  // which keeps the kernel at 4 waves per SIMD (a B = 6 grid of 768 blocks then fits
  // the chip in one dispatch round instead of leaving a third of it for a second one).
  constexpr int EPT = (G * HD + 255) / 256;
  static_assert(HD % EPT == 0, "a thread's elements must share one head");
  constexpr int NSB = 16;
  const int e0 = min(tid * EPT, G * HD - EPT);
  const int h = kvh * G + e0 / HD, d0 = e0 % HD;
  float M = -FLT_MAX, num[EPT], den = 0.f;
#pragma unroll
  for (int j = 0; j < EPT; ++j) num[j] = 0.f;
  for (int s0 = 0; s0 < ns; s0 += NSB) {
    float mv[NSB], lv[NSB], pv[NSB][EPT];
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const int s2 = min(s0 + i, ns - 1);
      const float* p = a.part + ((size_t)s2 * a.n_head + h) * (HD + 2);
      const float2 st = ld2_sc1(p + HD);
      mv[i] = st.x;
      lv[i] = st.y;
      if constexpr (EPT == 1) {
        pv[i][0] = ld_sc1(p + d0);
      } else {
#pragma unroll
        for (int j = 0; j < EPT; j += 2) {
          const float2 v = ld2_sc1(p + d0 + j);
          pv[i][j] = v.x;
          pv[i][j + 1] = v.y;
        }
      }
    }
    float mb = M;
#pragma unroll
    for (int i = 0; i < NSB; ++i) mb = (s0 + i < ns) ? fmaxf(mb, mv[i]) : mb;
    const float r = __expf(M - mb);
    den *= r;
#pragma unroll
    for (int j = 0; j < EPT; ++j) num[j] *= r;
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const float f = (s0 + i < ns) ? __expf(mv[i] - mb) : 0.f;
      den += f * lv[i];
#pragma unroll
      for (int j = 0; j < EPT; ++j) num[j] += f * pv[i][j];
    }
    M = mb;
  }
  // outputs: f32 (if asked for), and the f16 Wo input as one 8-byte store per 4-group (the lanes of
  // a group pass their values to its first lane). (Write-through sc1 stores here and in the SwiGLU
  // epilogue, against dirty lines at the kernel boundary, measured neutral.)
  float r[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) r[j] = num[j] / den;
  const bool live = tid * EPT < G * HD;
  if (a.out && live) {
    if (a.done) {  // an in-flight consumer reads it (attn_wo1): sc1
      if constexpr (EPT % 2 == 0) {
#pragma unroll
        for (int j = 0; j < EPT; j += 2) st2_sc1(a.out + h * HD + d0 + j, r[j], r[j + 1]);
      } else {
#pragma unroll
        for (int j = 0; j < EPT; ++j) st_sc1(a.out + h * HD + d0 + j, r[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) a.out[h * HD + d0 + j] = r[j];
    }
  }
  if (a.out_h) {
    static_assert(EPT == 1 || EPT == 2 || EPT % 4 == 0, "4-groups of the f16 output");
    constexpr int LPG = EPT >= 4 ? 1 : 4 / EPT;  // lanes per 4-group
    float g4[4 * ((EPT + 3) / 4)];
    if constexpr (LPG == 1) {
#pragma unroll
      for (int j = 0; j < EPT; ++j) g4[j] = r[j];
    } else {
#pragma unroll
      for (int q = 0; q < LPG; ++q)
#pragma unroll
        for (int j = 0; j < EPT; ++j) g4[q * EPT + j] = __shfl(r[j], (tid & ~(LPG - 1)) + q, 64);
    }
    if (live && (tid & (LPG - 1)) == 0) {
      const int o0 = h * HD + d0;  // a multiple of 4
#pragma unroll
      for (int k = 0; k < (EPT + 3) / 4; ++k) {
        // swizzled 4-group: (v0, v2, v1, v3)
        const h2v p0 = {(_Float16)g4[4 * k], (_Float16)g4[4 * k + 2]};
        const h2v p1 = {(_Float16)g4[4 * k + 1], (_Float16)g4[4 * k + 3]};
        const unsigned long long w = ((unsigned long long)__builtin_bit_cast(unsigned, p1) << 32) |
                                     __builtin_bit_cast(unsigned, p0);
        *reinterpret_cast<unsigned long long*>(a.out_h + o0 + 4 * k) = w;
      }
    }
  }
  if (a.done) {  // every storing wave drained, then one add for the whole block (Guideline 16, R1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(a.done + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (TL) { if (threadIdx.x == 0) tl[9] = wall_clock64(); }
#undef LFK_STAMP
}

}  // namespace lfk
