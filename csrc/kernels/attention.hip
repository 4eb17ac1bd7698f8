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
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "attn_dev.h"
#include "kernels.h"
#include "qdot.h"

namespace lfk {

template <int HD, int G, bool TL>
__global__ __launch_bounds__(256) void attn_decode_kernel(AttnDecodeArgs a) {
  attn_decode_body<HD, G, TL>(a);
}

size_t attn_decode_workspace_floats(int n_ctx, int n_head, int head_dim) {
  return (size_t)((n_ctx + CH - 1) / CH) * n_head * (head_dim + 2);
}

template <int HD, bool TL>
static void launch_attn_decode_tl(const AttnDecodeArgs& a, int G, dim3 grid, hipStream_t s) {
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<HD, 1, TL>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<HD, 2, TL>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((attn_decode_kernel<HD, 4, TL>), grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL((attn_decode_kernel<HD, 8, TL>), grid, dim3(256), 0, s, a); break;
    default: throw std::runtime_error("attn_decode: gqa group must be 1, 2, 4 or 8");
  }
}
template <int HD>
static void launch_attn_decode(const AttnDecodeArgs& a, int G, dim3 grid, hipStream_t s) {
  if (a.dbg_clk) launch_attn_decode_tl<HD, true>(a, G, grid, s);
  else launch_attn_decode_tl<HD, false>(a, G, grid, s);
}

void attn_decode(const AttnDecodeArgs& a, hipStream_t s) {
  const int G = a.n_head / a.n_kv_head;
  if (a.n_head % a.n_kv_head) throw std::runtime_error("attn_decode: n_head % n_kv_head");
  if (!a.counters) throw std::runtime_error("attn_decode: counters workspace missing");
  bool touch = false;
  for (int r = 0; r < AttnDecodeArgs::kTouchRanges; ++r) {
    if (!a.pf[r]) continue;
    if (!a.pf_sink || a.pf_bytes[r] < 4 || a.pf_nseg[r] < 1) throw std::runtime_error("attn_decode: weight touch needs pf_sink and >= 4 bytes");
    touch = true;
  }
  if (a.batch > 0) {
    if (!a.slots || a.n_kv_head > 64 || a.part_stride < attn_decode_workspace_floats(a.n_ctx, a.n_head, a.head_dim))
      throw std::runtime_error("attn_decode: bad batched arguments");
  }
  if (a.qkv_raw && (a.batch < 1 || !a.ss || a.qkv_ld % 2 || a.k_off % 2 || a.v_off % 2 || touch))
    throw std::runtime_error("attn_decode: split-K Q|K|V arguments");
  if (a.done) throw std::runtime_error("attn_decode: done counters are attn_wo1's (gemv.hip)");
  // z: the rows (batched) or one; the weight-touch plane, if any, is the next z index
  dim3 grid(a.n_kv_head, (a.n_ctx + CH - 1) / CH, (a.batch > 0 ? a.batch : 1) + (touch ? 1 : 0));
  if (a.head_dim == 128) launch_attn_decode<128>(a, G, grid, s);
  else if (a.head_dim == 64) launch_attn_decode<64>(a, G, grid, s);
  else throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
}

// ---------------------------------------------------------------- prefill (scalar)
// Fallback for GQA groups that are not a power of two. One wave = 4 queries of one head; lanes stride over keys (64 per step) for
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

// ---------------------------------------------------------------- prefill on MFMA
// Causal flash attention for a prompt chunk (SURVEY K7-K9 at T > 1; upstream ran KQ and
// KQV as batched cuBLAS GEMMs plus a separate masked softmax).
//
// Block = one kv head x 4 waves; wave = one query head x 32 queries (HB heads of the GQA
// group x 4/HB query tiles per block, so K/V tiles staged in LDS serve 4 waves). Per
// 64-key tile a wave runs
//   S^T[key][query] = K . Q^T   (v_mfma_f32_32x32x16_f16, A = K rows from LDS, B = Q held
//                                in registers for the whole kernel, pre-scaled by log2 e)
//   online softmax per query    (a query is one lane column: 32 in-lane values + one
//                                swap across the two lane halves)
//   O^T[dim][query] += V^T . P^T (A = V^T through ds_read_b64_tr_b16 on a row-major V
//                                tile, B = P^T straight from the S^T accumulators)
// P^T never leaves registers: the MFMA k order over keys is permuted so that a lane's
// S^T registers are exactly its B operand, and the V^T reads use the same permutation.
// Row pitches: K (HD+8 halves) makes the 16-lane ds_read_b128 row reads conflict-free,
// V (HD+32 halves) puts the 4 rows of a transposed read 16 banks apart.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// OUT: 0 f32, 1 bf16, 2 f16 in bmm's 4-group k order (gemm_t16's input)
template <int HD, int OUT>
__global__ __launch_bounds__(256) void attn_prefill_mfma_kernel(AttnPrefillArgs a, int HB) {
  constexpr int KT = 64, KP = HD + 8, VP = HD + 32, NKK = HD / 16, NDT = HD / 32;
  constexpr int CPR = HD / 8, NCH = KT * CPR / 256;  // 16-B chunks per row / per thread
  __shared__ __attribute__((aligned(16))) _Float16 Ks[KT * KP];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[KT * VP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, hh = lane >> 5;
  const int G = a.n_head / a.n_kv_head, QTB = 4 / HB;
  const int kvh = blockIdx.x;
  const int qblk = gridDim.y - 1 - blockIdx.y;  // latest (longest) query tiles dispatch first
  // packed pieces: z = piece x head group; the piece's rows, positions and KV slot
  int T = a.T, pos0 = a.pos0, hz = blockIdx.z;
  size_t row0 = 0, cache0 = 0;
  if (a.n_pieces > 0) {
    const int HZ = G / HB, pc = blockIdx.z / HZ;
    hz = blockIdx.z - pc * HZ;
    T = a.pc_n[pc];
    pos0 = a.pc_pos[pc];
    row0 = (size_t)a.pc_row[pc];
    cache0 = (size_t)a.pc_slot[pc] * a.slot_stride;
    if (qblk * QTB * 32 >= T) return;  // a shorter piece's missing tiles: whole block, no barrier yet
  }
  const int head = kvh * G + hz * HB + wave % HB;
  const int tq = (qblk * QTB + wave / HB) * 32;
  const int nkeys = pos0 + min(T, (qblk + 1) * QTB * 32);  // keys the block needs
  const int wkeys = pos0 + min(T, tq + 32);                 // keys this wave needs
  const int t = tq + lr;
  const int qpos = pos0 + min(t, T - 1);  // padded query columns attend like the last real one

  f16x8_t qf[NKK];
  {
    const float* qr = a.q + ((row0 + min(t, T - 1)) * a.n_head + head) * HD + 8 * hh;
    const float qs = a.scale * 1.44269504088896341f;
    f32x4_t qv[2 * NKK];  // all loads issued before the first use (one round trip)
#pragma unroll
    for (int i = 0; i < 2 * NKK; ++i) qv[i] = *reinterpret_cast<const f32x4_t*>(qr + 8 * (i >> 1) * 2 + 4 * (i & 1));
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const f32x4_t v0 = qv[2 * kk], v1 = qv[2 * kk + 1];
      const f32x8_t v = {v0.x * qs, v0.y * qs, v0.z * qs, v0.w * qs, v1.x * qs, v1.y * qs, v1.z * qs, v1.w * qs};
      qf[kk] = __builtin_convertvector(v, f16x8_t);
    }
  }
  const _Float16* kb = reinterpret_cast<const _Float16*>(a.k_cache) + cache0 + (size_t)kvh * a.n_ctx * HD;
  const _Float16* vb = reinterpret_cast<const _Float16*>(a.v_cache) + cache0 + (size_t)kvh * a.n_ctx * HD;
  // rows clamped to the last needed key: the rows past it hold real (finite) data that the
  // mask gives weight 0, so no NaN can leak into P.V; every load is unconditional
  int goff[NCH], soff[NCH], skey[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = tid + 256 * i;
    skey[i] = c / CPR;
    goff[i] = 8 * (c % CPR);
    soff[i] = skey[i] * KP + goff[i];
  }
  u32x4_t kr[NCH], vr[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const size_t row = (size_t)min(skey[i], nkeys - 1) * HD + goff[i];
    kr[i] = *reinterpret_cast<const u32x4_t*>(kb + row);
    vr[i] = *reinterpret_cast<const u32x4_t*>(vb + row);
  }
  f32x16_t o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m = -1e30f, l = 0.f;
  // transposed-read addresses (T10): lane 4q+p of a 16-lane group reads row q, columns 4p..4p+3
  const int trow = ((lane & 15) >> 2) + 4 * hh, tcol = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  for (int k0 = 0; k0 < nkeys; k0 += KT) {
    __syncthreads();  // every wave is done with the previous tile
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      *reinterpret_cast<u32x4_t*>(Ks + soff[i]) = kr[i];
      *reinterpret_cast<u32x4_t*>(Vs + soff[i] + skey[i] * (VP - KP)) = vr[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NCH; ++i) {  // next tile in flight during this one's math (clamped on the last)
      const size_t row = (size_t)min(k0 + KT + skey[i], nkeys - 1) * HD + goff[i];
      kr[i] = *reinterpret_cast<const u32x4_t*>(kb + row);
      vr[i] = *reinterpret_cast<const u32x4_t*>(vb + row);
    }
    if (k0 < wkeys) {  // wave-uniform: EXEC stays full for the transposed reads
      f32x16_t sc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[j][r] = 0.f;
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          const f16x8_t kv = *reinterpret_cast<const f16x8_t*>(Ks + (32 * j + lr) * KP + 16 * kk + 8 * hh);
          sc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kv, qf[kk], sc[j], 0, 0, 0);
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sc[j][r] = key <= qpos ? sc[j][r] : -INFINITY;
          mx = fmaxf(mx, sc[j][r]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mn = fmaxf(m, mx), alpha = exp2f(m - mn);
      m = mn;
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sc[j][r] = exp2f(sc[j][r] - mn);
          ls += sc[j][r];
        }
      l = l * alpha + ls;  // this half's keys; the halves are summed once at the end
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          const f32x8_t pv = {sc[j][8 * hs], sc[j][8 * hs + 1], sc[j][8 * hs + 2], sc[j][8 * hs + 3],
                              sc[j][8 * hs + 4], sc[j][8 * hs + 5], sc[j][8 * hs + 6], sc[j][8 * hs + 7]};
          const f16x8_t pb = __builtin_convertvector(pv, f16x8_t);
          // B element i <-> key 32j + 16hs + 8(i>>2) + 4hh + (i&3): rows r0 and r0 + 8 of V
          const _Float16* vrow = Vs + (32 * j + 16 * hs + trow) * VP + tcol;
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vrow + 32 * dt));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vrow + 8 * VP + 32 * dt));
            const f16x8_t va = __builtin_bit_cast(f16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(va, pb, o[dt], 0, 0, 0);
          }
        }
    }
  }
  l += __shfl_xor(l, 32);
  const float inv = 1.f / l;
  if (t < T) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int d = 32 * dt + 8 * rg + 4 * hh;  // o[dt][4rg + 0..3] = dims d .. d+3
        const size_t off = (row0 + t) * a.out_stride + (size_t)head * HD + d;
        const float v0 = o[dt][4 * rg] * inv, v1 = o[dt][4 * rg + 1] * inv;
        const float v2 = o[dt][4 * rg + 2] * inv, v3 = o[dt][4 * rg + 3] * inv;
        if constexpr (OUT == 1) {
          const uint2 pk = make_uint2(pk_bf16_pair(v0, v1), pk_bf16_pair(v2, v3));
          *reinterpret_cast<uint2*>(a.out_bf16 + off) = pk;
        } else if constexpr (OUT == 2) {  // positions (0, 2, 1, 3) of the 4-group
          const __half2 p0 = __floats2half2_rn(v0, v2), p1 = __floats2half2_rn(v1, v3);
          *reinterpret_cast<uint2*>(a.out_h + off) =
              make_uint2(__builtin_bit_cast(unsigned, p0), __builtin_bit_cast(unsigned, p1));
        } else {
          *reinterpret_cast<float4*>(a.out + off) = make_float4(v0, v1, v2, v3);
        }
      }
  }
}

template <int HD>
static void launch_attn_prefill_mfma(const AttnPrefillArgs& a, int G, hipStream_t s) {
  const int HB = std::min(G, 4), QTB = 4 / HB;
  int tmax = a.T;
  if (a.n_pieces > 0) {
    tmax = 0;
    for (int i = 0; i < a.n_pieces; ++i) tmax = std::max(tmax, a.pc_n[i]);
  }
  dim3 grid(a.n_kv_head, (tmax + 32 * QTB - 1) / (32 * QTB), (G / HB) * std::max(1, a.n_pieces));
  if (a.out_h) hipLaunchKernelGGL((attn_prefill_mfma_kernel<HD, 2>), grid, dim3(256), 0, s, a, HB);
  else if (a.out_bf16) hipLaunchKernelGGL((attn_prefill_mfma_kernel<HD, 1>), grid, dim3(256), 0, s, a, HB);
  else hipLaunchKernelGGL((attn_prefill_mfma_kernel<HD, 0>), grid, dim3(256), 0, s, a, HB);
}

void attn_prefill(const AttnPrefillArgs& a, hipStream_t s) {
  if (a.n_pieces < 0 || a.n_pieces > AttnPrefillArgs::kMaxPieces) throw std::runtime_error("attn_prefill: 0-16 pieces");
  if (a.n_pieces > 0) {
    for (int i = 0; i < a.n_pieces; ++i)
      if (a.pc_n[i] <= 0 || a.pc_pos[i] < 0 || a.pc_pos[i] + a.pc_n[i] > a.n_ctx || a.pc_row[i] < 0 || a.pc_slot[i] < 0)
        throw std::runtime_error("attn_prefill: bad piece");
  } else if (a.T <= 0) {
    return;
  }
  if (a.n_head % a.n_kv_head) throw std::runtime_error("attn_prefill: n_head % n_kv_head");
  if (a.head_dim != 128 && a.head_dim != 64) throw std::runtime_error("attn_prefill: head_dim must be 64 or 128");
  if (a.n_pieces == 0 && a.pos0 + a.T > a.n_ctx) throw std::runtime_error("attn_prefill: pos0 + T > n_ctx");
  const int G = a.n_head / a.n_kv_head;
  if (a.n_pieces > 0 && !((G & (G - 1)) == 0 && G <= 16)) throw std::runtime_error("attn_prefill: pieces need the MFMA path");
  if ((G & (G - 1)) == 0 && G <= 16) {  // GQA group a power of two (every Llama/Mixtral)
    if (a.head_dim == 128) launch_attn_prefill_mfma<128>(a, G, s);
    else launch_attn_prefill_mfma<64>(a, G, s);
    return;
  }
  if (!a.out) throw std::runtime_error("attn_prefill: the scalar path writes f32 only (no bf16 / f16 output)");
  dim3 grid(a.n_head, (a.T + 15) / 16);
  if (a.head_dim == 128) hipLaunchKernelGGL(attn_prefill_kernel<128>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(attn_prefill_kernel<64>, grid, dim3(256), 0, s, a);
}

}  // namespace lfk
