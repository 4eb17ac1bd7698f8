// Batched decode projection on MFMA (continuous batching, 1-16 activation rows):
//   out[b][row] += sum_k W[row][k] * x[b][k]
// W block-quantised (Q4_K / Q5_K / Q6_K / Q8_0) read from a tile-ordered copy (tile16, below);
// x f16 rows in a 4-group swizzled k order, staged per block in LDS - from xh (written by
// bprep or by the attention kernel) or, for Q|K|V and gate/up, straight from the fp32
// residual with the RMSNorm folded in.
//
// Why MFMA: with 2-16 rows the integer-dot GEMV (bgemv.hip) does B dot products per decoded
// weight on the VALU and ran VALU/epilogue-bound (6.2 ms per 8B step at B = 8,
// profiles/README.md). Here a wave owns a 16-row weight tile and feeds it to
// v_mfma_f32_16x16x32_f16 as the A operand, the activation rows as B: the matrix core does
// all 16 columns in the same 16 cycles, so the per-weight work is the dequantisation only
// (independent of B) and the weights stay ONE HBM stream. The kernel is bound by instruction
// issue (profiles/README.md, r2g/r2i), so the dequantisation is counted per instruction.
//
// Dequantisation straight into MFMA fragments: lane l holds A[row l&15][k = 8(l>>4) + j];
// lane group kq = l>>4 takes chunk 8s + 4h + kq (32 weights: a low and a high 16-run) of its
// row at step s. Quant bytes are masked to one value per byte (low / high nibbles, plus the
// Q5_K / Q6_K high bits), one v_perm_b32 per pair puts two bytes under the f16 exponent of
// 1024 (1024 + q exactly), one v_pk_add removes the 1024 (exact) and one v_pk_fma applies
// (d*sc, -dmin*m) - pre-decoded per sub-block in the Q4_K tile16 copy. A pair holds bytes
// (0, 2) or (1, 3) of a dword, so the k order inside each 4-group is (0, 2, 1, 3); x is
// written in that order. MFMA m of a chunk takes 8 weights of ONE run (low run 0-7 / 8-15,
// then high run 0-7 / 8-15): its B operand is one 16-byte LDS read as it stands.
//
// Work items are (16-row tile, K part); partial tiles are added to `out` atomically (split-K
// keeps >= 2 waves per SIMD busy on every projection shape, including the 256-tile Wo /
// down); one-part launches own their outputs (epilogues: RoPE + KV append, SwiGLU).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "gemv_dev.h"

namespace lfk {

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ h2_t as_h2(unsigned v) { return __builtin_bit_cast(h2_t, v); }
__device__ __forceinline__ unsigned as_u(h2_t v) { return __builtin_bit_cast(unsigned, v); }

// bytes 0 and 2 (or 1 and 3) of x under the f16 exponent of 1024: one v_perm_b32 builds the
// pair (1024 + b0, 1024 + b2) - the and / shift / or it replaces were 2-3 VALU ops per pair
// (the compiler did not form v_and_or_b32: CDNA VOP3 takes no literal constant)
__device__ __forceinline__ unsigned bytes02(unsigned x) { return __builtin_amdgcn_perm(0x64646464u, x, 0x04020400u); }
__device__ __forceinline__ unsigned bytes13(unsigned x) { return __builtin_amdgcn_perm(0x64646464u, x, 0x04030401u); }

// a (1024 + v0, 1024 + v1) f16 pair -> (v * a + m): exact subtraction of `bias`, one fma
__device__ __forceinline__ unsigned deq_pair(unsigned magic_pair, h2_t bias, h2_t a, h2_t m) {
  const h2_t v = as_h2(magic_pair) - bias;
  return as_u(v * a + m);
}

struct HFrag {
  unsigned w[16];  // MFMA i takes w[4i .. 4i+3]
};

// bmm's raw weights of one chunk: the WRaw layouts, except Q4_K, whose tile16 copy carries
// the sub-block scales pre-decoded - per row and sub-block one f16 pair (d * sc, -dmin * m) -
// instead of the packed 12-byte scales: the 6-bit unpacking was ~40 VALU ops per chunk, about
// a third of the dequantisation (the kernel ran with its SIMDs ~75 % busy issuing)
struct Q4Raw {
  int4 q;
  uint2 m;  // (d*sc, -dmin*m) as f16 pairs of sub-blocks 2g (low nibbles) and 2g + 1 (high)
};
// Q6_K likewise: the chunk's two scales arrive as one f16 pair (d * sc_lo, d * sc_hi), and its
// 2-bit high fields as two dwords already in place for the bit assembly (tile16 layout below):
// 6.5 VALU per quant dword instead of 9, no per-chunk scale conversion, one scale load not three
struct Q6Raw {
  int4 l;
  uint2 x;     // high fields of quant dwords (0, 1) and (2, 3)
  unsigned s;  // (d * sc_lo, d * sc_hi) f16 pair
};
template <int T> struct BRaw { using type = WRaw<T>; };
template <> struct BRaw<T_Q4_K> { using type = Q4Raw; };
template <> struct BRaw<T_Q6_K> { using type = Q6Raw; };
// Q5_K: as Q4_K plus the chunk's high bits
struct Q5Raw {
  int4 q, h;
  uint2 m;
};
template <> struct BRaw<T_Q5_K> { using type = Q5Raw; };
template <int T> using BRawT = typename BRaw<T>::type;

// chunk c of one row (raw loads in WRaw) -> the four A fragments
template <int T>
__device__ __forceinline__ void dequant_frags(const BRawT<T>& w, int c, HFrag& F) {
  const int j = c & 7;
  if constexpr (T == T_Q4_K) {
    const h2_t pa = as_h2(w.m.x), pb = as_h2(w.m.y);
    const h2_t alo = {pa[0], pa[0]}, mlo = {pa[1], pa[1]};
    const h2_t ahi = {pb[0], pb[0]}, mhi = {pb[1], pb[1]};
    const h2_t bias = {(_Float16)1024.f, (_Float16)1024.f};
    const int qv[4] = {w.q.x, w.q.y, w.q.z, w.q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (unsigned)qv[i] & 0x0F0F0F0Fu, hi = ((unsigned)qv[i] >> 4) & 0x0F0F0F0Fu;
      F.w[4 * i + 0] = deq_pair(bytes02(lo), bias, alo, mlo);
      F.w[4 * i + 1] = deq_pair(bytes13(lo), bias, alo, mlo);
      F.w[4 * i + 2] = deq_pair(bytes02(hi), bias, ahi, mhi);
      F.w[4 * i + 3] = deq_pair(bytes13(hi), bias, ahi, mhi);
    }
    (void)j;
  } else if constexpr (T == T_Q5_K) {
    const int g = j >> 1;
    const h2_t pa = as_h2(w.m.x), pb = as_h2(w.m.y);  // pre-decoded, as for Q4_K
    const h2_t alo = {pa[0], pa[0]}, mlo = {pa[1], pa[1]};
    const h2_t ahi = {pb[0], pb[0]}, mhi = {pb[1], pb[1]};
    const h2_t bias = {(_Float16)1024.f, (_Float16)1024.f};
    const int qv[4] = {w.q.x, w.q.y, w.q.z, w.q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned lo, hi;  // the dword's 4 low-nibble and 4 high-nibble values as bytes
      if constexpr (T == T_Q4_K) {
        lo = (unsigned)qv[i] & 0x0F0F0F0Fu;
        hi = ((unsigned)qv[i] >> 4) & 0x0F0F0F0Fu;
      } else {
        const unsigned hv = (unsigned)(i == 0 ? w.h.x : i == 1 ? w.h.y : i == 2 ? w.h.z : w.h.w);
        lo = ((unsigned)qv[i] & 0x0F0F0F0Fu) | (((hv >> (2 * g)) & 0x01010101u) << 4);
        hi = (((unsigned)qv[i] >> 4) & 0x0F0F0F0Fu) | (((hv >> (2 * g + 1)) & 0x01010101u) << 4);
      }
      F.w[4 * i + 0] = deq_pair(bytes02(lo), bias, alo, mlo);
      F.w[4 * i + 1] = deq_pair(bytes13(lo), bias, alo, mlo);
      F.w[4 * i + 2] = deq_pair(bytes02(hi), bias, ahi, mhi);
      F.w[4 * i + 3] = deq_pair(bytes13(hi), bias, ahi, mhi);
    }
  } else if constexpr (T == T_Q6_K) {
    const h2_t p = as_h2(w.s);
    const h2_t alo = {p[0], p[0]}, ahi = {p[1], p[1]};
    const h2_t zero = {(_Float16)0.f, (_Float16)0.f};
    const h2_t bias = {(_Float16)1056.f, (_Float16)1056.f};  // 1024 + 32: (q - 32) exactly
    const unsigned lv[4] = {(unsigned)w.l.x, (unsigned)w.l.y, (unsigned)w.l.z, (unsigned)w.l.w};
    // per byte of x dword e: bits 5:4 / 7:6 = the low / high 16-run fields of quant dword 2e,
    // bits 1:0 / 3:2 = those of dword 2e + 1; each lands on bits 5:4 with one shift and a mask
    const unsigned xv[2] = {w.x.x, w.x.y};
    unsigned fl[4], fh[4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      fl[2 * e] = xv[e] & 0x30303030u;
      fh[2 * e] = (xv[e] >> 2) & 0x30303030u;
      fl[2 * e + 1] = (xv[e] << 4) & 0x30303030u;
      fh[2 * e + 1] = (xv[e] << 2) & 0x30303030u;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (lv[i] & 0x0F0F0F0Fu) | fl[i];
      const unsigned hi = ((lv[i] >> 4) & 0x0F0F0F0Fu) | fh[i];
      F.w[4 * i + 0] = deq_pair(bytes02(lo), bias, alo, zero);
      F.w[4 * i + 1] = deq_pair(bytes13(lo), bias, alo, zero);
      F.w[4 * i + 2] = deq_pair(bytes02(hi), bias, ahi, zero);
      F.w[4 * i + 3] = deq_pair(bytes13(hi), bias, ahi, zero);
    }
    (void)j;
  } else {  // Q8_0: signed bytes, flipped to unsigned for the magic, one scale
    const float d = h2f(w.d & 0xFFFF);
    const h2_t a = {(_Float16)d, (_Float16)d};
    const h2_t zero = {(_Float16)0.f, (_Float16)0.f};
    const h2_t bias = {(_Float16)1152.f, (_Float16)1152.f};  // 1024 + 128
    const int lo4[4] = {w.a.x, w.a.y, w.a.z, w.a.w};
    const int hi4[4] = {w.b.x, w.b.y, w.b.z, w.b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (unsigned)lo4[i] ^ 0x80808080u, hi = (unsigned)hi4[i] ^ 0x80808080u;
      F.w[4 * i + 0] = deq_pair(bytes02(lo), bias, a, zero);
      F.w[4 * i + 1] = deq_pair(bytes13(lo), bias, a, zero);
      F.w[4 * i + 2] = deq_pair(bytes02(hi), bias, a, zero);
      F.w[4 * i + 3] = deq_pair(bytes13(hi), bias, a, zero);
    }
  }
}

// element offsets (into an x row) of chunk c's low and high 16-runs
template <int T>
__device__ __forceinline__ void chunk_runs(int c, int& off_lo, int& off_hi) {
  const int sb = c >> 3, j = c & 7;
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    off_lo = sb * 256 + 64 * (j >> 1) + 16 * (j & 1);
    off_hi = off_lo + 32;
  } else if constexpr (T == T_Q6_K) {
    off_lo = sb * 256 + 128 * (j >> 2) + 16 * (j & 3);
    off_hi = off_lo + 64;
  } else {
    off_lo = 32 * c;
    off_hi = off_lo + 16;
  }
}


// ---------------------------------------------------------------- tile16 weight layout
// A second, batched-path copy of every projection matrix (288 GB of HBM holds it): per
// 16-row tile and per 256-k step ONE contiguous block, ordered so that each of the kernel's
// load instructions reads 1 KB contiguous (planar rows would give every instruction 16
// scattered 64-B pieces - measured 1-2 TB/s). Lane l = 16 kq + r16 takes chunks 8s + kq
// (h = 0) and 8s + 4 + kq (h = 1) of row 16t + r16:
//   Q4_K: qs[h][l][16] | sb[r16][8][(d*sc, -dmin*m) f16]                         2560 B
//   Q5_K: qs[h][l][16] | qh[r16][32] | sb[r16][8][(d*sc, -dmin*m) f16]             3072 B
//   Q6_K: ql[h][l][16] | qx[h][l][8] | sc[r16][h][kq][(d*sc_lo, d*sc_hi) f16]   3584 B
//         (qx: the chunk's 2-bit high fields regrouped per lane - see dequant_frags)
//   Q8_0: qs[h][a|b][l][16] | d[h][l][2]                                        4352 B
// Rows past the matrix are zero.
__host__ __device__ constexpr int t16_step_bytes(int t) {
  return t == T_Q4_K ? 2560 : t == T_Q5_K ? 3072 : t == T_Q6_K ? 3584 : t == T_Q8_0 ? 4352 : 0;
}

size_t t16_bytes(int type, int rows, int K) {
  return (size_t)((rows + 15) / 16) * (size_t)(K / 256) * (size_t)t16_step_bytes(type);
}

__device__ __forceinline__ void copy16(uint8_t* d, const uint8_t* s, bool ok) {
  *reinterpret_cast<uint4*>(d) = ok ? *reinterpret_cast<const uint4*>(s) : make_uint4(0, 0, 0, 0);
}

template <int T>
__global__ __launch_bounds__(64) void t16_repack_kernel(QMat w, uint8_t* dst, int swiglu) {
  const int s = blockIdx.x, t = blockIdx.y, steps = gridDim.x;
  const int l = threadIdx.x, r16 = l & 15, kq = l >> 4;
  int row = t * 16 + r16;
  bool ok = row < w.rows;
  if (swiglu) {  // tile t: gate rows of features 8t .. 8t+7, then their up rows (32-row groups in `w`)
    const int f = 8 * t + (r16 & 7);
    row = 64 * (f >> 5) + (r16 >= 8 ? 32 : 0) + (f & 31);
    ok = f < w.rows / 2;
  }
  const size_t r = ok ? (size_t)row : 0;
  uint8_t* blk = dst + ((size_t)t * steps + s) * t16_step_bytes(T);
  const Planes& P = w.P;
  const uint8_t* base = w.base;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 8 * s + 4 * h + kq;
    if constexpr (T == T_Q8_0) {
      copy16(blk + h * 2048 + l * 16, base + P.p0 + r * P.s0 + 32 * c, ok);
      copy16(blk + h * 2048 + 1024 + l * 16, base + P.p0 + r * P.s0 + 32 * c + 16, ok);
      *reinterpret_cast<unsigned short*>(blk + 4096 + h * 128 + l * 2) =
          ok ? *reinterpret_cast<const unsigned short*>(base + P.p1 + r * P.s1 + 2 * c) : 0;
    } else {
      copy16(blk + h * 1024 + l * 16, base + P.p0 + r * P.s0 + 16 * c, ok);
    }
  }
  if (T != T_Q6_K && kq != 0) return;  // Q6_K: every lane writes its own chunks' fields
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    // decode the 8 sub-block scale / min pairs once, here (as the old in-kernel decode did:
    // f32 products, one rounding to f16); Q5_K's metadata plane is p2, Q4_K's p1
    const uint8_t* m = T == T_Q4_K ? base + P.p1 + r * P.s1 + 16 * s : base + P.p2 + r * P.s2 + 16 * s;
    const float d = ok ? h2f(*reinterpret_cast<const unsigned short*>(m)) : 0.f;
    const float dmin = ok ? h2f(*reinterpret_cast<const unsigned short*>(m + 2)) : 0.f;
    const uint8_t* q = m + 4;
    unsigned outw[8];
#pragma unroll
    for (int sb = 0; sb < 8; ++sb) {
      unsigned sc, mn;
      if (sb < 4) {
        sc = q[sb] & 63;
        mn = q[sb + 4] & 63;
      } else {
        sc = (q[sb + 4] & 0xF) | ((q[sb - 4] >> 6) << 4);
        mn = (q[sb + 4] >> 4) | ((q[sb] >> 6) << 4);
      }
      const h2_t p = {(_Float16)(d * (float)sc), (_Float16)(-dmin * (float)mn)};
      outw[sb] = ok ? as_u(p) : 0u;
    }
    uint4* dst16 = reinterpret_cast<uint4*>(blk + (T == T_Q4_K ? 2048 : 2560) + r16 * 32);
    dst16[0] = make_uint4(outw[0], outw[1], outw[2], outw[3]);
    dst16[1] = make_uint4(outw[4], outw[5], outw[6], outw[7]);
  }
  if constexpr (T == T_Q5_K) {
    copy16(blk + 2048 + r16 * 32, base + P.p1 + r * P.s1 + 32 * s, ok);
    copy16(blk + 2048 + r16 * 32 + 16, base + P.p1 + r * P.s1 + 32 * s + 16, ok);
  }
  if constexpr (T == T_Q6_K) {
    // every lane: its chunks 4h + kq. Chunk j of a 256-block reads ql bytes 16 (j & 3) of half
    // j >> 2, whose high fields sit in qh[32 (j >> 2) + 16 (kq & 1) + byte] at bit 2 (kq >> 1)
    // (low 16-run) and 4 + 2 (kq >> 1) (high 16-run); x dword e packs the fields of quant
    // dwords 2e (bits 5:4 low run, 7:6 high run) and 2e + 1 (bits 1:0, 3:2) of each byte
    const int sh = 2 * (kq >> 1);
    const uint8_t* scp = base + P.p2 + r * P.s2 + 16 * s;
    const float d = ok ? h2f(*reinterpret_cast<const unsigned short*>(base + P.p3 + r * P.s3 + 2 * s)) : 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint8_t* qh = base + P.p1 + r * P.s1 + 64 * s + 32 * h + 16 * (kq & 1);
      unsigned xw[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const unsigned q0 = ok ? qh[8 * e + b] : 0u, q1 = ok ? qh[8 * e + 4 + b] : 0u;
          const unsigned byte = (((q0 >> sh) & 3u) << 4) | (((q0 >> (sh + 4)) & 3u) << 6) |
                                ((q1 >> sh) & 3u) | (((q1 >> (sh + 4)) & 3u) << 2);
          xw[e] |= byte << (8 * b);
        }
      *reinterpret_cast<uint2*>(blk + 2048 + h * 512 + l * 8) = make_uint2(xw[0], xw[1]);
      // scales as in the old in-kernel decode: f32 product, one rounding to f16
      const int si = 8 * h + kq;  // the chunk's low 16-run; the high run uses si + 4
      const float slo = ok ? d * (float)(signed char)scp[si] : 0.f;
      const float shi = ok ? d * (float)(signed char)scp[si + 4] : 0.f;
      const h2_t pr = {(_Float16)slo, (_Float16)shi};
      *reinterpret_cast<unsigned*>(blk + 3072 + r16 * 32 + (4 * h + kq) * 4) = as_u(pr);
    }
  }
}

void t16_repack(const QMat& w, uint8_t* dst, hipStream_t st, bool swiglu) {
  if (!bmm_supported(w.type, w.K)) throw std::runtime_error("t16_repack: unsupported type / K");
  if (swiglu && w.rows % 64) throw std::runtime_error("t16_repack: SwiGLU copy needs 32-row gate / up groups");
  const dim3 grid(w.K / 256, (w.rows + 15) / 16);
  const int sw = swiglu ? 1 : 0;
  switch (w.type) {
    case T_Q4_K: hipLaunchKernelGGL(t16_repack_kernel<T_Q4_K>, grid, dim3(64), 0, st, w, dst, sw); break;
    case T_Q5_K: hipLaunchKernelGGL(t16_repack_kernel<T_Q5_K>, grid, dim3(64), 0, st, w, dst, sw); break;
    case T_Q6_K: hipLaunchKernelGGL(t16_repack_kernel<T_Q6_K>, grid, dim3(64), 0, st, w, dst, sw); break;
    default: hipLaunchKernelGGL(t16_repack_kernel<T_Q8_0>, grid, dim3(64), 0, st, w, dst, sw); break;
  }
}

// raw loads of lane l's chunk h (8s + 4h + kq) from a tile16 step block (NT: the quant
// bytes non-temporal - decode reads every weight once; the prefill GEMM's token blocks
// re-read them, so it loads them plainly)
template <int T, bool NT = true>
__device__ __forceinline__ int4 ld_q16(const uint8_t* p) {
  if constexpr (NT) return ld_nt16(p);
  else return *reinterpret_cast<const int4*>(p);
}
template <int T, bool NT = true>
__device__ __forceinline__ void tload(BRawT<T>& w, const uint8_t* blk, int h, int l, int r16, int kq) {
  if constexpr (T == T_Q4_K) {
    w.q = ld_q16<T, NT>(blk + h * 1024 + l * 16);
    // chunk 4h + kq covers sub-blocks 2g, 2g + 1 with g = 2h + kq / 2
    w.m = *reinterpret_cast<const uint2*>(blk + 2048 + r16 * 32 + 8 * (2 * h + (kq >> 1)));
  } else if constexpr (T == T_Q5_K) {
    w.q = ld_q16<T, NT>(blk + h * 1024 + l * 16);
    w.h = *reinterpret_cast<const int4*>(blk + 2048 + r16 * 32 + 16 * (kq & 1));
    w.m = *reinterpret_cast<const uint2*>(blk + 2560 + r16 * 32 + 8 * (2 * h + (kq >> 1)));
  } else if constexpr (T == T_Q6_K) {
    w.l = ld_q16<T, NT>(blk + h * 1024 + l * 16);
    w.x = *reinterpret_cast<const uint2*>(blk + 2048 + h * 512 + l * 8);
    w.s = *reinterpret_cast<const unsigned*>(blk + 3072 + r16 * 32 + (4 * h + kq) * 4);
  } else {
    w.a = ld_q16<T, NT>(blk + h * 2048 + l * 16);
    w.b = ld_q16<T, NT>(blk + h * 2048 + 1024 + l * 16);
    w.d = *reinterpret_cast<const unsigned short*>(blk + 4096 + h * 128 + l * 2);
  }
}

// tload through a buffer resource over the matrix (IL kernels): the step's byte offset is a
// uniform scalar (soffset), the lane's part a constant voffset and the plane offsets immediates -
// no per-step 64-bit address arithmetic, whose temporaries the register allocator placed in the
// registers of loads still in flight (a vmcnt wait on them drained the ring at every round)
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));
template <int T, bool NTQ = true>
__device__ __forceinline__ void tload_rs(BRawT<T>& w, __amdgpu_buffer_rsrc_t rs, int so, int h, int l, int r16, int kq) {
  auto b128 = [&](int vo, int imm) {  // quant planes: non-temporal (aux 2: each weight is read once per step)
    const v4i_t t = __builtin_bit_cast(v4i_t, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so + imm, NTQ ? 2 : 0));
    return make_int4(t.x, t.y, t.z, t.w);
  };
  auto b128c = [&](int vo, int imm) {
    const v4i_t t = __builtin_bit_cast(v4i_t, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so + imm, 0));
    return make_int4(t.x, t.y, t.z, t.w);
  };
  auto b64 = [&](int vo, int imm) {
    const v2i_t t = __builtin_bit_cast(v2i_t, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so + imm, 0));
    return make_uint2((unsigned)t.x, (unsigned)t.y);
  };
  if constexpr (T == T_Q4_K) {
    w.q = b128(l * 16, h * 1024);
    w.m = b64(r16 * 32 + 8 * (kq >> 1), 2048 + 16 * h);
  } else if constexpr (T == T_Q5_K) {
    w.q = b128(l * 16, h * 1024);
    w.h = b128c(r16 * 32 + 16 * (kq & 1), 2048);
    w.m = b64(r16 * 32 + 8 * (kq >> 1), 2560 + 16 * h);
  } else if constexpr (T == T_Q6_K) {
    w.l = b128(l * 16, h * 1024);
    w.x = b64(l * 8, 2048 + h * 512);
    w.s = __builtin_amdgcn_raw_buffer_load_b32(rs, r16 * 32 + kq * 4, so + 3072 + 16 * h, 0);
  } else {
    w.a = b128(l * 16, h * 2048);
    w.b = b128(l * 16, h * 2048 + 1024);
    w.d = __builtin_amdgcn_raw_buffer_load_b16(rs, l * 2, so + 4096 + h * 128, 0);
  }
}

template <int T>
__device__ __forceinline__ int raw_word(const BRawT<T>& w) {
  if constexpr (T == T_Q4_K || T == T_Q5_K) return w.q.x;
  else if constexpr (T == T_Q6_K) return w.l.x;
  else return w.a.x;
}

// One 256-k step of a 16-row tile: lane l's chunks 8s + 4h + kq (h = 0, 1) dequantised into
// MFMA A fragments, B = the staged x row of column r16 (xrow indexed by global k), one
// accumulator per chunk h (two dependent chains of 4 MFMAs instead of one of 8: the MFMA
// read-after-write stalls were 24 % of the gate/up kernel's wave cycles).
// IL: all 8 B-operand LDS reads first (the dequantisation then covers their latency; read per
// chunk, each group of 4 was waited for right behind its issue), both chunks dequantised, and the
// two accumulators' MFMAs alternating (one chain after the other stalled on every MFMA)
template <int QT, bool RAW = false, bool IL = false>
__device__ __forceinline__ void bmm_step(const BRawT<QT>* wc, int s, int kq, const __half* xrow, f4_t& acc, f4_t& acc2) {
  // MFMA m takes 8 weights of ONE run: the low run's 0-7 / 8-15 (m = 0 / 1), then the high run's
  // (m = 2 / 3) - pairs of quant dwords 2(m % 2), 2(m % 2) + 1 - so its B operand is the 16-byte
  // LDS read as it stands (taking 4 halves from each run cost 3 v_mov per MFMA)
  auto frag = [](const HFrag& F, int m) {
    const int dw = 2 * (m & 1), sh = (m >> 1) * 2;
    return make_uint4(F.w[4 * dw + sh], F.w[4 * dw + sh + 1], F.w[4 * dw + 4 + sh], F.w[4 * dw + 5 + sh]);
  };
  auto deq = [&](int h, int c, HFrag& F) {
    if constexpr (RAW) {  // microbenchmark (wt_body DBG 7): the MFMAs on the raw quant words
      const int rw = raw_word<QT>(wc[h]);
#pragma unroll
      for (int i = 0; i < 16; ++i) F.w[i] = (unsigned)rw + i;
    } else {
      dequant_frags<QT>(wc[h], c, F);
    }
  };
  if constexpr (IL) {
    uint4 xr[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int off_lo, off_hi;
      chunk_runs<QT>(8 * s + 4 * h + kq, off_lo, off_hi);
      const uint4* xl = reinterpret_cast<const uint4*>(xrow + off_lo);
      const uint4* xh = reinterpret_cast<const uint4*>(xrow + off_hi);
      xr[h][0] = xl[0]; xr[h][1] = xl[1]; xr[h][2] = xh[0]; xr[h][3] = xh[1];
    }
    HFrag F0, F1;
    deq(0, 8 * s + kq, F0);
    deq(1, 8 * s + 4 + kq, F1);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, frag(F0, m)),
                                                   __builtin_bit_cast(h8_t, xr[0][m]), acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, frag(F1, m)),
                                                    __builtin_bit_cast(h8_t, xr[1][m]), acc2, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 8 * s + 4 * h + kq;
      int off_lo, off_hi;
      chunk_runs<QT>(c, off_lo, off_hi);
      const uint4* xl = reinterpret_cast<const uint4*>(xrow + off_lo);
      const uint4* xh = reinterpret_cast<const uint4*>(xrow + off_hi);
      const uint4 xr[4] = {xl[0], xl[1], xh[0], xh[1]};
      HFrag F;
      deq(h, c, F);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        f4_t& ac = h == 0 ? acc : acc2;
        ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, frag(F, m)),
                                                    __builtin_bit_cast(h8_t, xr[m]), ac, 0, 0, 0);
      }
    }
  }
}

// f16 rows xh[b][k0, k0 + kn) into LDS: every thread's loads go out before any LDS store - one
// memory round trip for the slice (a load-store loop waited for each load in turn: 3-6 round trips,
// 1.5-3.6 us per launch)
template <int NW>
__device__ __forceinline__ void bmm_stage_x_plain(const BmmArgs& a, __half* xs, int ldx, int k0, int kn, int tid,
                                                  int i_begin = 0) {
  constexpr int kBlock = NW * 64, U = 8;
  const int nv = kn >> 3, n = a.B * nv;
  for (int i0 = i_begin; i0 < n; i0 += U * kBlock) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * kBlock + tid, n - 1);
      const int b = i / nv, c = i - b * nv;
      v[u] = *reinterpret_cast<const uint4*>(a.xh + (size_t)b * a.ldh + k0 + 8 * c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kBlock + tid;
      if (i < n) {
        const int b = i / nv, c = i - b * nv;
        *reinterpret_cast<uint4*>(xs + b * ldx + 8 * c) = v[u];
      }
    }
  }
}

// Stage x[b][k0, k0 + kn) of the B rows in LDS (f16, row stride ldx halves): from xh, or -
// with the RMSNorm folded in (a.xf, K = 4096, B <= 8, kBlock >= 512: each thread holds 2
// float4 of every row) - from the fp32 residual rows: every load is issued first (one memory
// round trip, like the f16 staging), then f16(x * w) goes to LDS in bprep's 4-group order and
// each wave leaves its per-row partial sum of squares in rowss[b * NW + wave] (rows past B load
// row B - 1 and are dropped: straight-line code, no predicated loads)
template <int NW>
__device__ __forceinline__ void bmm_stage_x(const BmmArgs& a, __half* xs, float* rowss, int ldx, int k0, int kn,
                                            int tid, int lane, int wave, int i_begin = 0) {
  constexpr int kBlock = NW * 64;
  if (NW >= 8 && a.xf) {
    constexpr int J = NW >= 8 ? 1024 / kBlock : 1;  // float4 of a 4096-wide row per thread
    float4 xv[8 * J], w[J];
#pragma unroll
    for (int j = 0; j < J; ++j) w[j] = *reinterpret_cast<const float4*>(a.norm_w + 4 * (tid + j * kBlock));
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const float* xr = a.xf + (size_t)min(b, a.B - 1) * a.ldxf;
#pragma unroll
      for (int j = 0; j < J; ++j) xv[J * b + j] = *reinterpret_cast<const float4*>(xr + 4 * (tid + j * kBlock));
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const float4 x = xv[J * b + j], ww = w[j];
        ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
        const h2_t p0 = {(_Float16)(x.x * ww.x), (_Float16)(x.z * ww.z)};
        const h2_t p1 = {(_Float16)(x.y * ww.y), (_Float16)(x.w * ww.w)};
        if (b < a.B) *reinterpret_cast<uint2*>(xs + b * ldx + 4 * (tid + j * kBlock)) = make_uint2(as_u(p0), as_u(p1));
      }
      ss = wave_sum_fast(ss);
      if (lane == 0) rowss[b * NW + wave] = ss;
    }
  } else {
    bmm_stage_x_plain<NW>(a, xs, ldx, k0, kn, tid, i_begin);
  }
}

// Q|K|V epilogue of one reduced 16-row tile (lane: rows 4kq .. 4kq+3, column r16): RoPE on the
// adjacent pairs (0,1), (2,3) this lane holds for Q and K, Q rows to q_out, K / V rows as f16
// into the row's KV slot at its position (the batched rope_kv_prefill folded in)
__device__ __forceinline__ void qkv_epilogue(const BmmArgs& a, int sg, int tile, int n_out, const f4_t& acc, int r16,
                                             int kq) {
  const auto& q = a.qkv;
  const int kind = sg == 0 ? q.kind[0] : sg == 1 ? q.kind[1] : q.kind[2], b = r16, hd = q.head_dim;
  const int pos = min(max(q.pos[b], 0), q.n_ctx - 1);
  const size_t so = (size_t)q.slots[b] * q.slot_stride;
#pragma unroll
  for (int i = 0; i < 4; i += 2) {
    const int row = tile * 16 + 4 * kq + i;
    if (row < n_out) {  // rows come in (even, odd) pairs: n_out is even
      float y0 = acc[i], y1 = acc[i + 1];
      const int dd = row % hd;
      if (kind < 2) {
        const float2 cs = q.rope[(size_t)pos * (hd >> 1) + (dd >> 1)];
        y0 = acc[i] * cs.x - acc[i + 1] * cs.y;
        y1 = acc[i] * cs.y + acc[i + 1] * cs.x;
      }
      if (kind == 0) {
        q.q_out[(size_t)b * q.q_ld + row] = y0;
        q.q_out[(size_t)b * q.q_ld + row + 1] = y1;
      } else {
        __half* c = (kind == 1 ? q.k_cache : q.v_cache) + so + ((size_t)(row / hd) * q.n_ctx + pos) * hd + dd;
        c[0] = __float2half(y0);
        c[1] = __float2half(y1);
      }
    }
  }
}

// Block barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads. __syncthreads() is a workgroup release/acquire, which makes every wave drain
// its outstanding global loads (s_waitcnt vmcnt(0)) - at every tile boundary that emptied
// the weight ring the loop keeps in flight across tiles.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Items are (16-row tile, K part). A block serves ONE K part (block b: part b % kparts):
// it stages that part of the B activation rows in LDS once (f16, row stride padded 16 B), then
// its 4 waves share every tile - wave w takes the part's steps w, w + 4, ... - and add their
// partial tiles through LDS, so a tile leaves the block as one store (or one atomic add per
// K part when the part count is > 1: few-way, not the 28-way contention of wave-level split-K).
//
// NW waves per block: 4 for the split-K shapes (4 blocks per CU), 8 for the one-part shapes
// (Q|K|V and SwiGLU epilogues: the whole-K x slice limits a CU to 2 blocks, so 8 waves keep
// 16 waves per CU streaming).
//
// Weights are double-buffered in registers with FIXED roles (ping-pong, the step loop
// unrolled by two): step i computes from one buffer while step i + 1 loads into the other.
// A rotating copy (wc = wn at the end of each step) made the compiler wait for the in-flight
// loads before the copy - s_waitcnt vmcnt(0) every step, so no load ever overlapped the
// next step's compute and the kernel ran on HBM latency. The buffers also run across tiles:
// the last step of a tile loads the next tile's first one (the roles swap after a tile with
// an odd number of steps per wave).
// (second launch bound = minimum waves per SIMD: 4, except the 8-wave Q6_K kernel, which
// would spill at 128 VGPRs)
template <int QT, int NW, int PD>
__device__ __attribute__((always_inline)) inline void bmm_body(const BmmArgs* __restrict__ ap, const int bid, const int nbk) {
  const BmmArgs& a = *ap;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);                       // [NW-1][64][4]
  float* rowss = reinterpret_cast<float*>(smem + (NW - 1) * 64 * 16);  // [8 rows][NW waves] folded norm
  __half* xs = reinterpret_cast<__half*>(smem + (NW - 1) * 64 * 16 + 512);
  const int lane = threadIdx.x & 63, wave = wave_id(), tid = threadIdx.x;
  const int r16 = lane & 15, kq = lane >> 4;
  const int K = a.w.K, steps = K >> 8;
  // microbenchmark timeline: [0] entry [1] weights issued [2] x staged [3] first tile computed
  // [4] exit [5] tiles done by the block
  long long* clk = a.dbg_clk ? a.dbg_clk + (size_t)bid * 8 : nullptr;
  if (clk && tid == 0) {
    clk[0] = wall_clock64();
    clk[6] = xcc_id();
  }
  // segments (Q|K|V in one launch): tile index -> (matrix, local tile)
  const int t1 = (a.n_out + 15) >> 4;
  const int t2 = t1 + (a.nseg > 1 ? (a.seg_rows[1] + 15) >> 4 : 0);
  const int t3 = t2 + (a.nseg > 2 ? (a.seg_rows[2] + 15) >> 4 : 0);
  const int tiles = a.nseg == 1 ? t1 : a.nseg == 2 ? t2 : t3;
  auto seg_of = [&](int g) { return g >= t1 ? (g >= t2 ? 2 : 1) : 0; };
  auto seg_first = [&](int sg) { return sg == 0 ? 0 : sg == 1 ? t1 : t2; };
  const int kparts = a.kparts, spp = a.spp;
  const int kp = bid % kparts;
  const int s0 = kp * spp, s1 = min(steps, s0 + spp);
  if (s0 >= s1) return;  // whole block, before any barrier
  if (a.ew && a.steps_per_expert > 0) {  // MoE down: the part of an unrouted expert adds nothing
    const int e = s0 / a.steps_per_expert;  // (the launcher keeps every part inside one expert)
    bool any = false;
    for (int b = 0; b < a.B; ++b) any = any || a.ew[(size_t)b * a.ew_ld + e] != 0.f;
    if (!any) return;  // whole block (uniform), before any barrier
  }
  const int k0 = s0 * 256, kn = (s1 - s0) * 256, ldx = kn + 8;
  const int gstride = nbk / kparts;
  // tile order: SwiGLU blocks take a contiguous range of tiles, balanced per CU: blocks b and
  // b + G (G = a.tile_groups, the CU count; placement only moves speed, never results) split
  // the quota T / G (+1) of group b % G between them - at 2 blocks per CU and T = 7 G every CU
  // gets exactly 7 tiles (an even split of whole units left a quarter of the CUs half-loaded)
  const bool sw = a.swiglu_epi;
  int gt = bid / kparts, tiles_end = tiles;
  // MoE gate/up: only the experts some row is routed to are computed - the split below runs
  // over their tiles alone ("active" index space: expert rank * tpe + local tile), so the
  // blocks share the routed experts' work evenly (E <= 64: one bit per expert, block-uniform)
  const bool moe_sw = sw && a.ew;
  const int tpe = moe_sw ? a.tiles_per_expert : 1;
  unsigned long long act = ~0ull;
  if (moe_sw) {
    bool any = false;
    if (lane < tiles / tpe)
      for (int b = 0; b < a.B; ++b) any = any || a.ew[(size_t)b * a.ew_ld + lane] != 0.f;
    act = __ballot(any);
  }
  auto glob = [&](int ai) {  // active index -> global tile
    if (!moe_sw) return ai;
    unsigned long long m = act;
    for (int r = ai / tpe; r > 0; --r) m &= m - 1;  // drop the lowest set bits: the rank-th expert
    return m ? (int)__builtin_ctzll(m) * tpe + ai % tpe : tiles;
  };
  if (sw) {
    const int ta = moe_sw ? __popcll(act) * tpe : tiles;  // tiles to compute
    const int G = a.tile_groups, g = bid % G, rnd = bid / G, nr = (nbk + G - 1) / G;
    const int q = ta / G + (g < ta % G ? 1 : 0), p0 = g * (ta / G) + min(g, ta % G);
    const int a0 = p0 + rnd * q / nr, a1 = p0 + (rnd + 1) * q / nr;
    gt = a0 < a1 ? glob(a0) : tiles;
    tiles_end = a1 >= ta ? tiles : glob(a1);
  }
  auto next_tile = [&](int g) {
    if (!sw) return g + gstride;
    ++g;
    if (moe_sw && g % tpe == 0 && g < tiles) {  // past an expert: the next routed one
      const unsigned long long m = act >> (g / tpe);
      g = m ? g + (int)__builtin_ctzll(m) * tpe : tiles;
    }
    return g;
  };
  if (gt >= tiles_end) return;  // whole block, before any barrier
  const int SB = t16_step_bytes(QT);
  auto tile_base = [&](int g) {  // first byte of global tile g's tile16 data
    const int sg = seg_of(g);
    const uint8_t* base = sg == 0 ? a.w.base : sg == 1 ? a.seg_base[1] : a.seg_base[2];
    return base + (size_t)(g - seg_first(sg)) * steps * SB;
  };
  const int ws0 = s0 + wave;                     // this wave's steps: ws0, ws0 + NW, ...
  const bool has = ws0 < s1;                      // (a part shorter than NW steps idles some waves)
  const int n_ws = has ? (s1 - 1 - ws0) / NW + 1 : 1;  // this wave's steps per tile
  // the first tile's first weights load before the x staging round trip
  const uint8_t* tb = tile_base(gt);
  // tiles after the first (past the end: an earlier valid tile - loaded, never used)
  const int g1 = next_tile(gt);
  const uint8_t* tbn = g1 < tiles_end ? tile_base(g1) : tb;
  const uint8_t* tbn2 = g1 < tiles_end && next_tile(g1) < tiles_end ? tile_base(next_tile(g1)) : tbn;
  auto addr = [&](int j) {  // weights of the wave's step j counted from this tile's first
    return j < n_ws ? tb + (size_t)(ws0 + j * NW) * SB
         : j < 2 * n_ws ? tbn + (size_t)(ws0 + (j - n_ws) * NW) * SB : tbn2 + (size_t)ws0 * SB;
  };
  BRawT<QT> wa[2], wb[2], wc[2];
  if (has) {
    const uint8_t* p0 = addr(0);
    tload<QT>(wa[0], p0, 0, lane, r16, kq);
    tload<QT>(wa[1], p0, 1, lane, r16, kq);
    if constexpr (PD == 2) {
      const uint8_t* p1 = addr(1);
      tload<QT>(wb[0], p1, 0, lane, r16, kq);
      tload<QT>(wb[1], p1, 1, lane, r16, kq);
    }
  }
  if (clk && tid == 0) clk[1] = wall_clock64();
  // stage x[b][k0, k0 + kn) for the B rows
  bmm_stage_x<NW>(a, xs, rowss, ldx, k0, kn, tid, lane, wave);
  __syncthreads();
  if (clk && tid == 0) clk[2] = wall_clock64();
  const bool col_ok = r16 < a.B;
  // folded norm: this lane's column scale (applied to the reduced tile before any epilogue)
  float cs = 1.f;
  if (NW >= 8 && a.xf) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += rowss[(col_ok ? r16 : 0) * NW + w];
    cs = rsqrtf(t / (float)kn + a.eps);
  }
  const __half* xrow = xs + (col_ok ? r16 : 0) * ldx - k0;  // indexed by global k
  // the wave's steps as one flattened sequence over its tiles, the buffers alternating
  // (wa, wb, wa, ...) along it: no register copies, and a tile's end is just a point in it
  // two accumulators (chunk h = 0 / 1): the 8 MFMAs of a step form two dependent chains of 4
  // instead of one of 8 (SQ_WAIT_INST_ANY, the MFMA read-after-write stalls, was 24 % of the
  // gate/up kernel's wave cycles)
  f4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  int i = 0;  // step of the current tile
  auto compute = [&](const BRawT<QT>* wc, int i) {
    // one step per scheduling region: interleaving two steps' dequantisation raised the
    // register count from ~110 to 150-180 (2-3 waves per SIMD)
    __builtin_amdgcn_sched_barrier(0);
    const int s = ws0 + i * NW;
    if (a.debug == 1) {  // microbenchmark: weight stream only
      acc[0] += (float)raw_word<QT>(wc[0]) + (float)raw_word<QT>(wc[1]);
      return;
    }
    bmm_step<QT>(wc, s, kq, xrow, acc, acc2);
  };
  // reduction + epilogue of tile gt (every wave of the block, once per tile)
  int ntiles_done = 0;
  auto finish_tile = [&]() {
    if (clk && tid == 0 && ntiles_done == 0) clk[3] = wall_clock64();
    ++ntiles_done;
    acc += acc2;
    const int sg = seg_of(gt);   // wave-uniform
    const int tile = gt - seg_first(sg);
    const int n_out = sg == 0 ? a.n_out : sg == 1 ? a.seg_rows[1] : a.seg_rows[2];
    float* out = sg == 0 ? a.out : sg == 1 ? a.seg_out[1] : a.seg_out[2];
    // the 4 waves' partial tiles meet in LDS; wave 0 writes C[row 4kq + i][col r16]
    if (wave > 0) *reinterpret_cast<f4_t*>(red + ((wave - 1) * 64 + lane) * 4) = acc;
    lds_barrier();
    if (wave == 0) {
#pragma unroll
      for (int w = 0; w < NW - 1; ++w) acc += *reinterpret_cast<const f4_t*>(red + (w * 64 + lane) * 4);
      if (NW >= 8 && a.xf) acc *= cs;
      if (sw) {
        // rows 0-7 of the tile (lanes 0-31): gate of features 8 gt + 4 kq + i; rows 8-15 (lanes
        // 32-63): the up rows of the same features
        f4_t up;
#pragma unroll
        for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(acc[i], 32);
        if (col_ok && lane < 32) {
          const int f0 = gt * 8 + 4 * kq;  // 4 consecutive features
          // MoE: the row's routing weight of this tile's expert (0: the row is not routed here)
          const float rw = a.ew ? a.ew[(size_t)r16 * a.ew_ld + gt / a.tiles_per_expert] : 1.f;
          const h2_t p0 = {(_Float16)(silu(acc[0]) * up[0] * rw), (_Float16)(silu(acc[2]) * up[2] * rw)};
          const h2_t p1 = {(_Float16)(silu(acc[1]) * up[1] * rw), (_Float16)(silu(acc[3]) * up[3] * rw)};
          *reinterpret_cast<uint2*>(a.h_out + (size_t)r16 * a.ldh_out + f0) = make_uint2(as_u(p0), as_u(p1));
        }
      } else if (col_ok && a.qkv_epi) {
        qkv_epilogue(a, sg, tile, n_out, acc, r16, kq);
      } else if (col_ok) {
        float* o = out + (size_t)r16 * a.ldo;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = tile * 16 + 4 * kq + i;
          if (row < n_out) {
            if (kparts > 1) atomicAdd(o + row, acc[i]);
            else if (a.store_out) o[row] = acc[i];
            else o[row] += acc[i];   // one owner per (row, column)
          }
        }
      }
    }
    lds_barrier();  // red is reused by the next tile
    acc = f4_t{0.f, 0.f, 0.f, 0.f};
    acc2 = acc;
  };
  // after step i: the tile's end finishes it and moves to the next tile (false: block done)
  auto advance = [&]() {
    if (++i < n_ws) return true;
    finish_tile();
    i = 0;
    gt = next_tile(gt);
    if (gt >= tiles_end) return false;
    tb = tbn;
    tbn = tbn2;
    const int gn2 = next_tile(gt) < tiles_end ? next_tile(next_tile(gt)) : tiles_end;
    tbn2 = gn2 < tiles_end ? tile_base(gn2) : tbn;
    return true;
  };
  // one step: load step i + PD into `ld`, compute step i from `cur`
  auto step = [&](BRawT<QT>* ld, const BRawT<QT>* cur) {
    const uint8_t* p = addr(i + PD);
    tload<QT>(ld[0], p, 0, lane, r16, kq);
    tload<QT>(ld[1], p, 1, lane, r16, kq);
    compute(cur, i);
    return advance();
  };
  if (has) {
    if constexpr (PD == 1) {
      for (;;) {
        if (!step(wb, wa)) break;
        if (!step(wa, wb)) break;
      }
    } else {
      for (;;) {
        if (!step(wc, wa)) break;
        if (!step(wa, wb)) break;
        if (!step(wb, wc)) break;
      }
    }
  } else {
    for (; gt < tiles_end; gt = next_tile(gt)) finish_tile();  // idle waves still join every tile's barriers
  }
  if (clk && tid == 0) {
    clk[4] = wall_clock64();
    clk[5] = ntiles_done;
  }
}

// Q|K|V of the bumped layers in ONE launch: blocks [0, a.nb1) run the Q|K run (type QT, args a),
// the rest the V run (type QT2, args a2; Q4_K_M bumps V to Q6_K on half the layers). As its own
// launch the 64-tile V projection cost 10.4 us on a 3.6 MB matrix (B = 6, r3c profile); a
// side-stream graph branch for it measured no gain (r2 profiles).
template <int QT, int NW, int PD, int QT2 = 0>
__global__ __launch_bounds__(NW * 64, ((QT == T_Q6_K || QT2 == T_Q6_K) && NW == 8) || PD == 2 ? 3 : 4)
void bmm_kernel(BmmArgs a, BmmArgs a2) {
  // the body reads its arguments through the kernarg segment pointer: a reference to the
  // by-value parameter made the compiler copy the whole block to scratch (544 B per lane)
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  if constexpr (QT2 != 0) {
    if ((int)blockIdx.x >= ka[0].nb1) {
      bmm_body<QT2, NW, PD>(ka + 1, blockIdx.x - ka[0].nb1, gridDim.x - ka[0].nb1);
      return;
    }
    bmm_body<QT, NW, PD>(ka, blockIdx.x, ka[0].nb1);
  } else {
    bmm_body<QT, NW, PD>(ka, blockIdx.x, gridDim.x);
  }
  (void)a;
  (void)a2;
}

// ---------------------------------------------------------------- wave-owned tiles
// One-part projections with many tiles (dense SwiGLU gate/up: 1792 tiles = 7 per CU for the 8B
// shape; the head) and the split-K ones (Wo, down, Q|K|V): every WAVE streams whole tiles of its
// block's K part with PD steps of weights in flight in registers, so there is no cross-wave
// reduction and no barrier after the x staging. bmm_kernel splits a tile's steps over the block's
// 8 waves (2 steps per wave at K = 4096): every tile ended in an LDS reduction behind two block
// barriers, each wave had one step in flight, and 46 % of the wave cycles sat in s_waitcnt /
// barriers (r2g PMC).
// Blocks are (K part kp, tile group): part > 1 adds its partial tiles atomically. Gate/up, Wo and
// down run one block per CU (the launcher asks for more than half the LDS, so two never share a
// CU): the x slice is staged once per CU, and block b takes the contiguous tile range
// [t0, t0 + tn) of an even split - wave w its tiles t0 + w + i * NW. Split-K Q|K|V groups are
// a.tpg tiles of one weight type (run A: segments [0, seg_split), run B: the rest, type QT2).
// Weights rotate through PD + 1 register buffers with fixed roles (the step loop unrolled by
// PD + 1): no register copies, so no wait on in-flight loads before they are needed.

// x staging of one K part with the RMSNorm folded in (split-K Q|K|V): rows xf[b][k0, k0 + kn) as
// f16(x * norm_w) in bmm's 4-group order, each row's sum of squares over the part added to
// rowss[b] (LDS, zeroed by the caller). All loads of a batch go out before any use (one memory
// round trip); kn % 256 == 0, so the 64 float4 of a wave lie in one row.
template <int NW>
__device__ __forceinline__ void stage_x_part_norm(const BmmArgs& a, __half* xs, float* rowss, int ldx, int k0, int kn,
                                                  int tid, int lane, int i_begin = 0) {
  constexpr int kBlock = NW * 64, U = 4;
  const int nv = kn >> 2, n = a.B * nv;
  for (int i0 = i_begin; i0 < n; i0 += U * kBlock) {
    float4 v[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * kBlock + tid, n - 1);
      const int b = i / nv, c = i - b * nv;
      v[u] = *reinterpret_cast<const float4*>(a.xf + (size_t)b * a.ldxf + k0 + 4 * c);
      w[u] = *reinterpret_cast<const float4*>(a.norm_w + k0 + 4 * c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int iw = i0 + u * kBlock + (tid & ~63);  // the wave's first index (wave-uniform)
      if (iw >= n) break;
      const int i = iw + lane;
      const int b = i / nv, c = i - b * nv;
      const float4 x = v[u], ww = w[u];
      const h2_t p0 = {(_Float16)(x.x * ww.x), (_Float16)(x.z * ww.z)};
      const h2_t p1 = {(_Float16)(x.y * ww.y), (_Float16)(x.w * ww.w)};
      *reinterpret_cast<uint2*>(xs + b * ldx + 4 * c) = make_uint2(as_u(p0), as_u(p1));
      const float ss = wave_sum_fast(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
      if (lane == 0) atomicAdd(rowss + b, ss);
    }
  }
}

// x-first staging (XF): the x loads of a block's first staging pass go out BEFORE its first weight
// steps, and are written to LDS after those are issued. A CU returns its loads in order: x issued
// behind the weights waited for those weight bytes (~40 KB per CU at the CU's ~24 GB/s share of
// HBM - the 2.2-4.2 us x-staged stamps of profiles/r5a_batch_step_b6_block_timeline_layer5.json),
// while issued first it returns from L2 and the weights stream behind it. (Round 2's x-first form
// waited for x before it issued any weight: the whole stream started a round trip late.)
// mode 1: fp32 rows with the RMSNorm folded (K = 4096, B <= 8); 2: one split-K Q|K|V part with
// its norm; 0: f16 rows (xh)
// Each form keeps its x registers in ONE ext_vector value local to its function, and runs `issue`
// - the first weight steps - between its loads and its LDS stores. (Arrays of float4 / uint4 held
// across the inlined `issue` went to scratch - 144-560 B per lane, stored right behind the loads
// with a vmcnt wait each - where a single vector value stays in VGPRs.)
template <int N>
using f32v = float __attribute__((ext_vector_type(N)));
template <int N>
using u32v = unsigned __attribute__((ext_vector_type(N)));
// global-address-space loads: pointer arithmetic on the staging rows made the compiler emit flat
// loads, which its waitcnt accounting only ever retires with a full vmcnt(0) + lgkmcnt(0)
// (through native vector types: HIP's float4 / uint4 copy through a generic reference, which turned
// the load back into a flat one)
__device__ __forceinline__ float4 ldg4(const float* p) {
  typedef float v4 __attribute__((ext_vector_type(4)));
  const v4 t = *(const __attribute__((address_space(1))) v4*)(p);
  return make_float4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ uint4 ldg4(const __half* p) {
  typedef unsigned v4 __attribute__((ext_vector_type(4)));
  const v4 t = *(const __attribute__((address_space(1))) v4*)(p);
  return make_uint4(t.x, t.y, t.z, t.w);
}
template <int N>
__device__ __forceinline__ void vput(f32v<N>& v, int i, float4 t) {
  v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
}
template <int N>
__device__ __forceinline__ float4 vget(const f32v<N>& v, int i) {
  return make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}
// (SC1: the rows with sc1 loads - written in this launch by atomics from other CUs, a plain load
// could hit a stale L2 line)
template <int NW, bool SC1 = false, class Issue>
__device__ __forceinline__ void xfirst_norm(const BmmArgs& a, __half* xs, float* rowss, int ldx, int tid, int lane,
                                            int wave, Issue&& issue) {
  constexpr int kBlock = NW * 64, J = NW >= 8 ? 1024 / kBlock : 1;  // float4 of a 4096-wide row per thread
  f32v<32 * J> xv;
  f32v<4 * J> w;
#pragma unroll
  for (int j = 0; j < J; ++j) vput(w, j, ldg4(a.norm_w + 4 * (tid + j * kBlock)));
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.xf), 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const float* xr = a.xf + (size_t)min(b, a.B - 1) * a.ldxf;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if constexpr (SC1) {
        const int off = (int)(((size_t)min(b, a.B - 1) * a.ldxf + 4 * (tid + j * kBlock)) * sizeof(float));
        const f32v<4> t = __builtin_bit_cast(f32v<4>, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 16));  // sc1
        vput(xv, J * b + j, make_float4(t[0], t[1], t[2], t[3]));
      } else {
        vput(xv, J * b + j, ldg4(xr + 4 * (tid + j * kBlock)));
      }
    }
  }
  issue();
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const float4 x = vget(xv, J * b + j), ww = vget(w, j);
      ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
      const h2_t p0 = {(_Float16)(x.x * ww.x), (_Float16)(x.z * ww.z)};
      const h2_t p1 = {(_Float16)(x.y * ww.y), (_Float16)(x.w * ww.w)};
      if (b < a.B) *reinterpret_cast<uint2*>(xs + b * ldx + 4 * (tid + j * kBlock)) = make_uint2(as_u(p0), as_u(p1));
    }
    ss = wave_sum_fast(ss);
    if (lane == 0) rowss[b * NW + wave] = ss;
  }
}

// split-K Q|K|V part with its norm (rowss zeroed by the caller before `issue` returns: the first
// pass's LDS side waits for the caller's barrier inside `issue`)
template <int NW, class Issue>
__device__ __forceinline__ void xfirst_part_norm(const BmmArgs& a, __half* xs, float* rowss, int ldx, int k0, int kn,
                                                 int tid, int lane, Issue&& issue) {
  constexpr int kBlock = NW * 64, U = 4;
  const int nv = kn >> 2, n = a.B * nv;
  f32v<4 * U> v, w;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = min(u * kBlock + tid, n - 1);
    const int b = i / nv, c = i - b * nv;
    vput(v, u, ldg4(a.xf + (size_t)b * a.ldxf + k0 + 4 * c));
    vput(w, u, ldg4(a.norm_w + k0 + 4 * c));
  }
  issue();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int iw = u * kBlock + (tid & ~63);  // the wave's first index (wave-uniform)
    if (iw < n) {
      const int i = iw + lane;
      const int b = i / nv, c = i - b * nv;
      const float4 x = vget(v, u), ww = vget(w, u);
      const h2_t p0 = {(_Float16)(x.x * ww.x), (_Float16)(x.z * ww.z)};
      const h2_t p1 = {(_Float16)(x.y * ww.y), (_Float16)(x.w * ww.w)};
      *reinterpret_cast<uint2*>(xs + b * ldx + 4 * c) = make_uint2(as_u(p0), as_u(p1));
      const float ss = wave_sum_fast(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
      if (lane == 0) atomicAdd(rowss + b, ss);
    }
  }
  if (n > U * kBlock) stage_x_part_norm<NW>(a, xs, rowss, ldx, k0, kn, tid, lane, U * kBlock);
}

// f16 rows (xh)
template <int NW, class Issue>
__device__ __forceinline__ void xfirst_plain(const BmmArgs& a, __half* xs, float* rowss, int ldx, int k0, int kn,
                                             int tid, int lane, int wave, Issue&& issue) {
  constexpr int kBlock = NW * 64, U = 8;
  const int nv = kn >> 3, n = a.B * nv;
  u32v<4 * U> v;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = min(u * kBlock + tid, n - 1);
    const int b = i / nv, c = i - b * nv;
    const uint4 t = ldg4(a.xh + (size_t)b * a.ldh + k0 + 8 * c);
    v[4 * u] = t.x; v[4 * u + 1] = t.y; v[4 * u + 2] = t.z; v[4 * u + 3] = t.w;
  }
  issue();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = u * kBlock + tid;
    if (i < n) {
      const int b = i / nv, c = i - b * nv;
      *reinterpret_cast<uint4*>(xs + b * ldx + 8 * c) = make_uint4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
    }
  }
  if (n > U * kBlock) bmm_stage_x_plain<NW>(a, xs, ldx, k0, kn, tid, U * kBlock);
}

// In-launch chain (BmmArgs::chain_*), consumer side: thread 0 waits (bounded, sc1 polls) until the
// block's K part has all of its producer tiles, then the block stages its x with sc1 loads (the
// producer wrote it write-through from other CUs; a plain load could hit a stale L2 line of the
// previous layer's use of the same buffer).
// wave 0 waits (bounded, sc1 polls) until the 8 XCD shards of counter `part` sum to `need`
__device__ __forceinline__ void count_wait(const BmmArgs& a, int part, int need, int tid) {
  if (tid < 64) {
    const int* c = a.chain_cnt + (part * kChainXcds + (tid & (kChainXcds - 1))) * kChainStride;
    const long long t0 = wall_clock64();
    for (;;) {
      int v = tid < kChainXcds ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      if (__shfl(v, 0) >= need) break;
      if (wall_clock64() - t0 > 200000000LL) {  // 2 s (100 MHz): report, never hang the stream
        if (a.chain_err && tid == 0) __hip_atomic_store(a.chain_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      for (int i = 0; i < a.chain_poll; ++i) __builtin_amdgcn_s_sleep(1);
    }
  }
  lds_barrier();
}

__device__ __forceinline__ void chain_wait(const BmmArgs& a, int kp, int tid) {
  if (tid < 64) {
    // wave 0: lanes 0-7 poll the part's 8 XCD shards, lanes 8-15 those of the producers' x-staged
    // count (every producer must have read its x before this block's epilogue adds into the
    // residual rows that x is read from); the sums are broadcast from lanes 0 and 8
    const int need = min(a.chain_tpp, a.chain_tiles - kp * a.chain_tpp);
    const int part = tid < kChainXcds ? kp : kChainStagedPart;
    const int* c = a.chain_cnt + (part * kChainXcds + (tid & (kChainXcds - 1))) * kChainStride;
    const long long t0 = wall_clock64();
    for (;;) {
      int v = tid < 2 * kChainXcds ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      if (__shfl(v, 0) >= need && __shfl(v, 8) >= a.chain_staged) break;
      if (wall_clock64() - t0 > 200000000LL) {  // 2 s (100 MHz): report, never hang the stream
        if (a.chain_err && tid == 0) __hip_atomic_store(a.chain_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      for (int i = 0; i < a.chain_poll; ++i) __builtin_amdgcn_s_sleep(1);
    }
  }
  lds_barrier();
}

template <int NW>
__device__ __forceinline__ void xstage_sc1(const BmmArgs& a, __half* xs, int ldx, int k0, int kn, int tid) {
  constexpr int kBlock = NW * 64, U = 8;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(a.xh), 0, 0x7FFFFFFF, 0x00020000);
  const int nv = kn >> 3, n = a.B * nv;
  for (int i0 = 0; i0 < n; i0 += U * kBlock) {
    u32v<4 * U> v;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * kBlock + tid, n - 1);
      const int b = i / nv, c = i - b * nv;
      const u32v<4> t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((size_t)b * a.ldh + k0 + 8 * c) * sizeof(__half)), 0,
                                                          16);  // aux 16: sc1
      v[4 * u] = t.x; v[4 * u + 1] = t.y; v[4 * u + 2] = t.z; v[4 * u + 3] = t.w;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kBlock + tid;
      if (i < n) {
        const int b = i / nv, c = i - b * nv;
        *reinterpret_cast<uint4*>(xs + b * ldx + 8 * c) = make_uint4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
      }
    }
  }
}

// The staged x rows' stride past the part (f16 elements): rows 24 halves = 12 banks apart make the
// ds_read_b128 B-operand reads of the K-quant chunk order conflict-free at B <= 6 (1.5-way at 7-8;
// 8 halves: 2-way from B = 4). Lane groups of ds_read_b128 per MI355X_MICROARCH's LDS table.
constexpr int kWtXPad = 24;
// interleaved step (bmm_step's IL) in the dense wave-owned kernels; LFK_BMM_IL=0 for the A/B
static bool bmm_il() {
  static const bool v = [] {
    const char* e = std::getenv("LFK_BMM_IL");
    return !(e && e[0] == '0');
  }();
  return v;
}


// SK: the split-K Q|K|V launch (segments, RoPE'd atomic partials, per-part norm staging) - a
// compile-time switch: the generic code paths cost the gate/up / Wo / down instantiations ~0.7 us
// per launch (registers and branches) when they were runtime ones
// (bid, nblk): the block's index and count in the launch's wave-owned grid (the fused attention +
// Wo launch runs this body in planes of its grid past the attention's)
// DBG (microbenchmarks, tools/boundary_bench.py; BmmArgs::debug 4-7): 4 = the weight stream alone
// (no x staging, no MFMA), 5 = x staging + weight stream (no MFMA), 6 = weight stream + MFMA (no x
// staging), 7 = as 6 with the MFMAs on the raw quant words (no dequantisation)
// CR: the in-launch chain role of the x staging, compile-time (0 x-first, kChainConsume: wait for the
// K part's gate/up tiles, kChainWaitWo: wait for every Wo block) - as a runtime branch the staging
// paths with the weights issued before x merged into the step loop, and the waitcnt pass then
// drained the weight ring at every round of every wave-owned kernel
template <int QT, int PD, bool SK, int NW = 8, bool MOE = false, bool XF = false, int DBG = 0, bool IL = false,
          int EPI = 0, int CR = 0>
__device__ __forceinline__ void wt_body(const BmmArgs& a, const int run, const int bid, const int nblk) {
  constexpr int R = PD + 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* rowss = reinterpret_cast<float*>(smem);            // [8 rows][NW waves] folded norm
  __half* xs = reinterpret_cast<__half*>(smem + 256);
  // the prologue's kernarg fields in ONE batch of scalar loads: read where first used, each behind
  // its own s_waitcnt, they were ~10 dependent round trips (~1.2 us) before the first weight load
  {
    const int f0 = a.w.K, f1 = a.kparts, f2 = a.spp, f3 = a.n_out, f4 = a.B, f5 = a.nseg, f6 = a.debug, f7 = a.chain_role;
    const int f8 = a.ldh, f9 = a.ldxf, f10 = a.zero_n, f11 = a.ldo, f12 = a.nb1, f13 = a.tpg, f14 = a.seg_split;
    const void *p0 = a.w.base, *p1 = a.xh, *p2 = a.xf, *p3 = a.norm_w, *p4 = a.zero, *p5 = a.dbg_clk, *p6 = a.out,
               *p7 = a.chain_cnt, *p8 = a.ss_out;
    asm volatile("" ::"s"(f0), "s"(f1), "s"(f2), "s"(f3), "s"(f4), "s"(f5), "s"(f6), "s"(f7), "s"(f8), "s"(f9), "s"(f10),
                 "s"(f11), "s"(f12), "s"(f13), "s"(f14), "s"(p0), "s"(p1), "s"(p2), "s"(p3), "s"(p4), "s"(p5), "s"(p6),
                 "s"(p7), "s"(p8), "s"(nblk));
  }
  const int lane = threadIdx.x & 63, wave = wave_id(), tid = threadIdx.x;
  const int r16 = lane & 15, kq = lane >> 4;
  const int K = a.w.K, steps = K >> 8;
  // block = (K part kp, tile group grp): parts > 1 add their partial tiles atomically (Wo /
  // down: 8 parts x 32 groups of 8 tiles = one block per CU for the 256-tile shapes)
  const int kparts = a.kparts, kp = bid % kparts, grp = bid / kparts, G = nblk / kparts;
  const int s0 = kp * a.spp, ns = min(steps, s0 + a.spp) - s0;  // this part's steps [s0, s0 + ns)
  const int k0 = s0 * 256, kn = ns * 256, ldx = kn + kWtXPad;
  if (MOE && !SK && a.ew && a.steps_per_expert > 0) {
    // MoE down: the part of an unrouted expert adds nothing (and its SwiGLU rows were never
    // written - its gate/up tiles were skipped): the whole block leaves, before any barrier
    const int e = s0 / a.steps_per_expert;
    bool any = false;
    for (int b = 0; b < a.B; ++b) any = any || a.ew[(size_t)b * a.ew_ld + e] != 0.f;
    if (!any) {
      if (a.zero) {  // (its share of the zero side job still gets done)
        float4* z = reinterpret_cast<float4*>(a.zero);
        for (int i = bid * (NW * 64) + threadIdx.x; i < (a.zero_n >> 2); i += nblk * (NW * 64))
          z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      return;
    }
  }
  // segments (split-K Q|K|V): global tile g -> (segment, local tile)
  const int t1 = (a.n_out + 15) >> 4;
  const int t2 = SK ? t1 + (a.nseg > 1 ? (a.seg_rows[1] + 15) >> 4 : 0) : t1;
  const int t3 = SK ? t2 + (a.nseg > 2 ? (a.seg_rows[2] + 15) >> 4 : 0) : t1;
  const int tiles = !SK || a.nseg == 1 ? t1 : a.nseg == 2 ? t2 : t3;
  auto seg_of = [&](int g) { return SK ? (g >= t1 ? (g >= t2 ? 2 : 1) : 0) : 0; };
  auto seg_first = [&](int sg) { return sg == 0 ? 0 : sg == 1 ? t1 : t2; };
  int t0, tn;
  if constexpr (SK) {  // groups of a.tpg tiles inside one run (run B: from segment seg_split on)
    const int ta = a.seg_split >= a.nseg ? tiles : a.seg_split == 1 ? t1 : t2;
    const int gl = run == 0 ? grp : grp - a.nb1;
    t0 = (run == 0 ? 0 : ta) + gl * a.tpg;
    tn = max(0, min(a.tpg, (run == 0 ? ta : tiles) - t0));
  }
  // MoE gate/up (the experts stacked as one SwiGLU matrix, routing weights a.ew [B][E]): only the
  // experts some row is routed to are computed - the even split runs over their tiles alone
  // ("active" index space: expert rank * tpe + local tile; E <= 64, one bit per expert)
  const bool moe_sw = MOE && !SK && a.swiglu_epi && a.ew;  // (a separate instantiation)
  const int tpe = moe_sw ? a.tiles_per_expert : 1;
  unsigned long long act = ~0ull;
  if (moe_sw) {
    bool any = false;
    if (lane < tiles / tpe)
      for (int b = 0; b < a.B; ++b) any = any || a.ew[(size_t)b * a.ew_ld + lane] != 0.f;
    act = __ballot(any);
  }
  if constexpr (!SK) {
    const int ta = moe_sw ? (int)__popcll(act) * tpe : tiles;
    t0 = grp * (ta / G) + min(grp, ta % G);
    tn = ta / G + (grp < ta % G ? 1 : 0);
  }
  const int nt = wave < tn ? (tn - 1 - wave) / NW + 1 : 0;  // this wave's tiles (wave-uniform)
  const int N = nt * ns;                                    // ... as one sequence of steps
  const int SB = t16_step_bytes(QT);
  auto tile_of = [&](int i) {
    const int ai = t0 + wave + i * NW;
    if (!moe_sw) return ai;
    unsigned long long m = act;  // the (ai / tpe)-th routed expert: drop the lower set bits
    for (int r = ai / tpe; r > 0; --r) m &= m - 1;
    return (int)__builtin_ctzll(m) * tpe + ai % tpe;
  };
  auto tbase = [&](int i) {
    const int g = tile_of(i), sg = seg_of(g);
    const uint8_t* base = !SK || sg == 0 ? a.w.base : sg == 1 ? a.seg_base[1] : a.seg_base[2];
    return base + ((size_t)(g - seg_first(sg)) * steps + s0) * SB;
  };
  BRawT<QT> buf[R][2];
  int li = 0, ls = 0;  // load cursor: the wave's tile, step
  const uint8_t* lp = nt > 0 ? tbase(0) : a.w.base;
  auto load_next = [&](BRawT<QT>* dst) {
    tload<QT>(dst[0], lp + (size_t)ls * SB, 0, lane, r16, kq);
    tload<QT>(dst[1], lp + (size_t)ls * SB, 1, lane, r16, kq);
    if (++ls == ns) {
      ls = 0;
      if (++li < nt) lp = tbase(li);
    }
  };
  // the first steps: issued whether or not the wave has them (past its last step: the matrix's
  // first block, never used), so the loads are branch-free - a conditional load makes the
  // compiler's vmcnt accounting assume the path without it and wait for every later load at the
  // x staging (XF)
  // IL: a buffer resource over the wave's current tile (its steps at soffset ls * SB); the
  // matrix's first block for the steps past the wave's last
  auto rsrc = [](const uint8_t* p) { return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, 0x7FFFFFFF, 0x00020000); };
  const auto rs0 = rsrc(a.w.base);
  auto rs_cur = rsrc(lp);
  auto load_first = [&](BRawT<QT>* dst, bool real) {
    if constexpr (IL) {
      const auto rs = real ? rs_cur : rs0;
      const int so = real ? ls * SB : 0;
      tload_rs<QT>(dst[0], rs, so, 0, lane, r16, kq);
      tload_rs<QT>(dst[1], rs, so, 1, lane, r16, kq);
    } else {
      const uint8_t* p = real ? lp + (size_t)ls * SB : a.w.base;
      tload<QT>(dst[0], p, 0, lane, r16, kq);
      tload<QT>(dst[1], p, 1, lane, r16, kq);
    }
    if (real && ++ls == ns) {
      ls = 0;
      if (++li < nt) {
        lp = tbase(li);
        if constexpr (IL) rs_cur = rsrc(lp);
      }
    }
  };
  // microbenchmark timeline (wave 0, as bmm_kernel's): [0] entry [1] weights issued [2] x staged
  // [3] first tile computed [4] exit [5] tiles of wave 0
  long long* clk = a.dbg_clk ? a.dbg_clk + (size_t)bid * 8 : nullptr;
  if (clk && tid == 0) {
    clk[0] = wall_clock64();
    clk[6] = xcc_id();
  }
  if (a.debug == 2) {  // microbenchmark: the launch alone (kernel boundary of this launch shape)
    if (clk && tid == 0) clk[4] = wall_clock64();
    return;
  }
  const bool col_ok = r16 < a.B;
  // split-K Q|K|V: the row's position and the RoPE factors of the wave's first tile, loaded
  // beside the weights (the epilogue of each tile prefetches the next tile's)
  int pos = 0;
  float2 rc[2] = {make_float2(1.f, 0.f), make_float2(1.f, 0.f)};
  auto rope_load = [&](int i) {
    const int g = tile_of(i), sg = seg_of(g);
    const int row = (g - seg_first(sg)) * 16 + 4 * kq, hd = a.qkv.head_dim;
#pragma unroll
    for (int j = 0; j < 2; ++j) rc[j] = a.qkv.rope[(size_t)pos * (hd >> 1) + ((row + 2 * j) % hd >> 1)];
  };
  if (SK && tid < 8) rowss[tid] = 0.f;  // the part's row sums of squares (stage_x_part_norm)
  // staging form: 2 = split-K Q|K|V part with its norm, 1 = whole rows with the norm folded, 0 = f16 rows
  const int xmode = (SK && a.ss_out) ? 2 : (NW >= 8 && a.xf) ? 1 : 0;
  // the first PD steps of weights go out ahead of the x staging round trip - or, XF, right behind
  // the x loads, which then no longer queue behind them; the row's position (split-K Q|K|V: its RoPE
  // factors load after the staging, beside the first tile's weights) and the zero side job follow
  // (the side job's stores and the stamp go before the weights: ops of uncertain count behind the x
  // loads would make the compiler's vmcnt accounting wait for the weights at the x staging)
  auto issue = [&]() __attribute__((always_inline)) {
    if (clk && tid == 0) clk[1] = wall_clock64();
    if (a.zero) {  // side job: zero the next consumer's accumulation rows
      float4* z = reinterpret_cast<float4*>(a.zero);
      for (int i = bid * (NW * 64) + tid; i < (a.zero_n >> 2); i += nblk * (NW * 64)) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int p = 0; p < PD; ++p) load_first(buf[p], p < N);
    if constexpr (SK && !IL) pos = a.qkv.pos[col_ok ? r16 : 0];
    if (!XF && xmode == 2) lds_barrier();  // rowss zeroed
  };
  // (XF: that barrier goes first - an asm memory clobber between the x loads and their LDS stores
  // made the compiler keep the x registers in scratch)
  if (XF && xmode == 2) lds_barrier();
  // kChainWoDone: the block's waves count their exits here; the last one publishes the block
  __shared__ int wo_exits;
  if (tid == 0) wo_exits = 0;  // (ordered before any exit by the staging barrier below)
  auto wo_arrive = [&]() {
    if (!SK && (a.chain_role & kChainWoDone)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's residual atomics are done
      if (lane == 0 && atomicAdd(&wo_exits, 1) == NW - 1)
        __hip_atomic_fetch_add(a.chain_cnt + (kChainWoPart * kChainXcds + (xcc_id() & (kChainXcds - 1))) * kChainStride, 1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  if constexpr (DBG == 4 || DBG == 6) issue();
  else if constexpr (XF) {
    if constexpr (!SK && CR == kChainConsume) {  // chain consumer: the weights do not depend on the producer
      issue();
      chain_wait(a, kp, tid);
      xstage_sc1<NW>(a, xs, ldx, k0, kn, tid);
    } else if constexpr (!SK && CR == kChainWaitWo) {  // x = the rows Wo adds into (xmode 1)
      issue();
      count_wait(a, kChainWoPart, a.chain_wo, tid);
      xfirst_norm<NW, true>(a, xs, rowss, ldx, tid, lane, wave, [] {});
    } else if (xmode == 2) xfirst_part_norm<NW>(a, xs, rowss, ldx, k0, kn, tid, lane, issue);
    else if (xmode == 1) xfirst_norm<NW>(a, xs, rowss, ldx, tid, lane, wave, issue);
    else xfirst_plain<NW>(a, xs, rowss, ldx, k0, kn, tid, lane, wave, issue);
  } else {
    issue();
    if (xmode == 2) stage_x_part_norm<NW>(a, xs, rowss, ldx, k0, kn, tid, lane);
    else bmm_stage_x<NW>(a, xs, rowss, ldx, k0, kn, tid, lane, wave);
  }
  // XF: an LDS-only barrier - __syncthreads() would drain the weight steps just issued (vmcnt(0))
  if constexpr (XF) lds_barrier();
  else __syncthreads();
  if (clk && tid == 0) clk[2] = wall_clock64();
  // chain producer: its x is read (the loads landed before their LDS stores, the barrier above)
  if (!SK && (a.chain_role & kChainProduce) && tid == 0)
    __hip_atomic_fetch_add(a.chain_cnt + (kChainStagedPart * kChainXcds + (xcc_id() & (kChainXcds - 1))) * kChainStride, 1,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (SK && a.ss_out && run == 0 && grp == 0 && tid < a.B) atomicAdd(a.ss_out + tid, rowss[tid]);
  if (N == 0) {
    wo_arrive();
    return;
  }
  if constexpr (SK && !IL) {  // (IL: the RoPE is the attention's - bmm_qkv_sk_defers_rope)
    pos = min(max(pos, 0), a.qkv.n_ctx - 1);
    rope_load(0);
  }
  float cs = 1.f;  // folded norm (one K part): this lane's column scale
  if (a.xf && !SK) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += rowss[(col_ok ? r16 : 0) * NW + w];
    cs = rsqrtf(t / (float)K + a.eps);
  }
  const __half* xrow = xs + (col_ok ? r16 : 0) * ldx - k0;  // indexed by global k
  f4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  int ci = 0, cstep = 0;  // compute cursor (step s0 + cstep of tile ci)
  auto finish = [&]() {   // tile ci is complete in acc + acc2: C[row 4kq + i][col r16]
    acc += acc2;
    if (a.debug == 3) {  // microbenchmark: no epilogue writes (an empty asm keeps the tile live)
      asm volatile("" ::"v"(acc[0]), "v"(acc[1]), "v"(acc[2]), "v"(acc[3]));
      acc = f4_t{0.f, 0.f, 0.f, 0.f};
      acc2 = acc;
      return;
    }
    if (a.xf && !SK) acc *= cs;
    const int gt = tile_of(ci);
    if constexpr (SK) {
      const int sg = seg_of(gt), kind = sg == 0 ? a.qkv.kind[0] : sg == 1 ? a.qkv.kind[1] : a.qkv.kind[2];
      const int n_out = sg == 0 ? a.n_out : sg == 1 ? a.seg_rows[1] : a.seg_rows[2];
      float* o = (sg == 0 ? a.out : sg == 1 ? a.seg_out[1] : a.seg_out[2]) + (size_t)r16 * a.ldo;
      const int row0 = (gt - seg_first(sg)) * 16 + 4 * kq;
      f4_t y = acc;
      if (!IL && kind < 2) {  // RoPE on the adjacent pairs (0, 1), (2, 3) of this lane's rows
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          y[2 * j] = acc[2 * j] * rc[j].x - acc[2 * j + 1] * rc[j].y;
          y[2 * j + 1] = acc[2 * j] * rc[j].y + acc[2 * j + 1] * rc[j].x;
        }
      }
      if constexpr (!IL) {
        if (ci + 1 < nt) rope_load(ci + 1);
      }
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row0 + i < n_out) atomicAdd(o + row0 + i, y[i]);
      }
    } else if (EPI == 1 || (EPI == 0 && a.swiglu_epi)) {
      // rows 0-7 (lanes 0-31): gate of features 8 gt + 4 kq + i; rows 8-15 (lanes 32-63): up
      f4_t up;
#pragma unroll
      for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(acc[i], 32);
      if (col_ok && lane < 32) {
        const int f0 = gt * 8 + 4 * kq;
        // MoE: the row's routing weight of this tile's expert (0: not routed there)
        const float rw = moe_sw ? a.ew[(size_t)r16 * a.ew_ld + gt / tpe] : 1.f;
        const h2_t p0 = {(_Float16)(silu(acc[0]) * up[0] * rw), (_Float16)(silu(acc[2]) * up[2] * rw)};
        const h2_t p1 = {(_Float16)(silu(acc[1]) * up[1] * rw), (_Float16)(silu(acc[3]) * up[3] * rw)};
        __half* h = a.h_out + (size_t)r16 * a.ldh_out + f0;
        if (!MOE && (a.chain_role & kChainProduce))  // chain producer: write-through (a consumer CU reads it next)
          __hip_atomic_store(reinterpret_cast<unsigned long long*>(h),
                             ((unsigned long long)as_u(p1) << 32) | as_u(p0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          *reinterpret_cast<uint2*>(h) = make_uint2(as_u(p0), as_u(p1));
      }
      if (EPI == 0 && !MOE && (a.chain_role & kChainProduce)) {  // the tile's rows have landed: count it for its consumer part
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(a.chain_cnt + (gt / a.chain_tpp * kChainXcds + (xcc_id() & (kChainXcds - 1))) * kChainStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (EPI == 3) {  // one part, plain stores (the batched head's logits): no loads in the loop
      if (col_ok) {
        float* o = a.out + (size_t)r16 * a.ldo;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = gt * 16 + 4 * kq + i;
          if (row < a.n_out) o[row] = acc[i];
        }
      }
    } else if (EPI == 2) {  // split-K only: fp32 atomics, no read-modify-write path
      if (col_ok) {
        float* o = a.out + (size_t)r16 * a.ldo;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = gt * 16 + 4 * kq + i;
          if (row < a.n_out) atomicAdd(o + row, acc[i]);
        }
      }
    } else if (col_ok) {
      float* o = a.out + (size_t)r16 * a.ldo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = gt * 16 + 4 * kq + i;
        if (row < a.n_out) {
          if (kparts > 1) atomicAdd(o + row, acc[i]);
          else if (a.store_out) o[row] = acc[i];
          else o[row] += acc[i];  // one owner per (row, column)
        }
      }
    }
    acc = f4_t{0.f, 0.f, 0.f, 0.f};
    acc2 = acc;
  };
  auto step = [&](int r, int j0) __attribute__((always_inline)) {
    // branch-free (past the wave's last step: the matrix's first block, never used): under an
    // `if` the waitcnt pass merged the paths with and without these loads and waited for every
    // load in flight - vmcnt(0) every 1-2 steps, the PD-deep ring drained
    if constexpr (IL) load_first(buf[(r + PD) % R], j0 + r + PD < N);
    else if (j0 + r + PD < N) load_next(buf[(r + PD) % R]);
    __builtin_amdgcn_sched_barrier(0);  // one step per scheduling region (register count)
    if constexpr (DBG == 4 || DBG == 5)
      asm volatile("" ::"v"(raw_word<QT>(buf[r][0])), "v"(raw_word<QT>(buf[r][1])));
    else
      bmm_step<QT, DBG == 7, IL>(buf[r], s0 + cstep, kq, xrow, acc, acc2);
    if (++cstep == ns) {
      finish();
      cstep = 0;
      ++ci;
      if (clk && tid == 0 && ci == 1) clk[3] = wall_clock64();
    }
  };
  int j0 = 0;
  if constexpr (IL) {
    // whole rounds of R steps without an exit inside (the loop back-edge then has ONE predecessor
    // state: the waitcnt pass's merge of the early-exit paths waited for more loads than needed),
    // then the remaining N % R steps
    for (; j0 + R <= N; j0 += R) {
#pragma unroll
      for (int r = 0; r < R; ++r) step(r, j0);
    }
  }
  for (; j0 < N; j0 += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (j0 + r >= N) break;  // wave-uniform
      step(r, j0);
    }
  }
  // EPI 1 (the SwiGLU epilogue alone): the chain producer counts its tiles once all are stored - a
  // vmcnt(0) at every tile end made the waitcnt pass drain the weight ring in the step loop
  if constexpr (EPI == 1 && !MOE) {
    if ((a.chain_role & kChainProduce) && nt > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        for (int i = 0; i < nt; ++i)
          __hip_atomic_fetch_add(a.chain_cnt + (tile_of(i) / a.chain_tpp * kChainXcds + (xcc_id() & (kChainXcds - 1))) * kChainStride,
                                 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  wo_arrive();
  if (clk) {  // exit: the block's LAST wave (waves of one block can end microseconds apart)
    if (lane == 0) atomicMax(reinterpret_cast<unsigned long long*>(clk + 4), (unsigned long long)wall_clock64());
    if (tid == 0) clk[5] = nt;
  }
}

// (the body reads its arguments through the kernarg segment pointer: a reference to the by-value
// parameter made the compiler copy the whole block to scratch, as in bmm_kernel)
// (PD > 2: one block per CU - the launchers' LDS request - so a register budget of 256, not 128)
// EPI: the epilogue as a compile-time kind (0 any, 1 SwiGLU, 2 split-K atomics, 3 one-part plain stores)
template <int QT, int PD, bool MOE = false, bool XF = false, bool IL = false, int EPI = 0>
__global__ __launch_bounds__(512, PD > 2 ? 1 : 2) void bmm_wt_kernel(BmmArgs a) {
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  wt_body<QT, PD, false, 8, MOE, XF, 0, IL, EPI>(*ka, 0, blockIdx.x, gridDim.x);
  (void)a;
}

template <int QT, int DBG>
__global__ __launch_bounds__(512, 2) void bmm_wt_dbg_kernel(BmmArgs a) {
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  wt_body<QT, 2, false, 8, false, true, DBG>(*ka, 0, blockIdx.x, gridDim.x);
  (void)a;
}

// split-K Q|K|V of one weight type
template <int QT, int PD, bool XF = false, bool IL = false>
__global__ __launch_bounds__(512, 2) void bmm_sk_kernel(BmmArgs a) {
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  wt_body<QT, PD, true, 8, false, XF, 0, IL>(*ka, 0, blockIdx.x, gridDim.x);
  (void)a;
}

// split-K Q|K|V over two weight types (Q|K Q4_K + V Q6_K / Q5_K on the bumped layers of the
// K-quant mixes, Q Q4_K + K|V Q8_0 in Mixtral's): groups from a.nb1 on are run B, type QT2 (a
// uniform branch per block; each run's body keeps its own registers)
template <int QT, int QT2, int PD, bool XF = false, bool IL = false>
__global__ __launch_bounds__(512, 2) void bmm_wt2_kernel(BmmArgs a) {
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  if ((int)blockIdx.x / ka->kparts >= ka->nb1) wt_body<QT2, PD, true, 8, false, XF, 0, IL>(*ka, 1, blockIdx.x, gridDim.x);
  else wt_body<QT, PD, true, 8, false, XF, 0, IL>(*ka, 0, blockIdx.x, gridDim.x);
  (void)a;
}

// The SwiGLU gate/up (QT1, producer) and the down projection (QT2, consumer) in ONE launch:
// blocks [0, a.nb1) run the gate/up, the rest the down (their own BmmArgs: the second kernarg).
template <int QT1, int QT2, bool IL = false, int PD = 2>
__global__ __launch_bounds__(512, PD > 2 ? 1 : 2) void bmm_chain_kernel(BmmArgs a, BmmArgs b) {
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const int n1 = ka[0].nb1;
  if ((int)blockIdx.x < n1) wt_body<QT1, PD, false, 8, false, true, 0, IL, IL ? 1 : 0>(ka[0], 0, blockIdx.x, n1);
  else wt_body<QT2, PD, false, 8, false, true, 0, IL, IL ? 2 : 0, kChainConsume>(ka[1], 0, blockIdx.x - n1, gridDim.x - n1);
  (void)a;
  (void)b;
}

// Wo (QT0, split-K into the residual) -> gate/up (QT1) -> down (QT2) in ONE launch (bmm_wo_ffn_chain)
template <int QT0, int QT1, int QT2>
__global__ __launch_bounds__(512, 2) void bmm_chain3_kernel(BmmArgs a, BmmArgs b, BmmArgs c) {
  const BmmArgs* ka = (const BmmArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const int n0 = ka[0].nb1, n1 = ka[1].nb1;
  const int bid = blockIdx.x;
  if (bid < n0) wt_body<QT0, 2, false, 8, false, true, 0, true, 2>(ka[0], 0, bid, n0);
  else if (bid < n0 + n1) wt_body<QT1, 2, false, 8, false, true, 0, true, 1, kChainWaitWo>(ka[1], 0, bid - n0, n1);
  else wt_body<QT2, 2, false, 8, false, true, 0, true, 2, kChainConsume>(ka[2], 0, bid - n0 - n1, gridDim.x - n0 - n1);
  (void)a;
  (void)b;
  (void)c;
}

// ---------------------------------------------------------------- activation prep
// One block per activation row: optional SwiGLU (gate/up pre-activations in 32-feature
// interleaved groups), optional RMSNorm (* w), f16, k order (0,2,1,3) inside every 4-group.
// Side job: zero [zero, zero + zero_n) (the split-K output of the projection this feeds) -
// done by extra blocks past the B row blocks (up to 4 MB for the lm_head logits: 8 row blocks
// alone took tens of microseconds for it).
static constexpr int kPrepBlock = 1024;
static constexpr int kPrepMaxVec = 8;  // float4 per thread: K <= 32768

__global__ __launch_bounds__(kPrepBlock) void bprep_kernel(BPrepArgs a) {
  __shared__ float red[kPrepBlock / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b >= a.B) {
    float4* z = reinterpret_cast<float4*>(a.zero);
    const int nzb = gridDim.x - a.B;
    for (int i = (b - a.B) * kPrepBlock + tid; i < (a.zero_n >> 2); i += nzb * kPrepBlock)
      z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float* xr = a.x + (size_t)b * a.ldx;
  float4 v[kPrepMaxVec];
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < kPrepMaxVec; ++u) {
    const int i = 4 * (tid + u * kPrepBlock);
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < a.K) {
      if (a.swiglu) {
        const int G = a.swiglu_group;  // 32 or 8 (a power of two, i % 4 == 0 stays in one group)
        const int gi = (i / G) * 2 * G + (i % G);
        const float4 g = *reinterpret_cast<const float4*>(xr + gi);
        const float4 up = *reinterpret_cast<const float4*>(xr + gi + G);
        v[u] = make_float4(silu(g.x) * up.x, silu(g.y) * up.y, silu(g.z) * up.z, silu(g.w) * up.w);
      } else {
        v[u] = *reinterpret_cast<const float4*>(xr + i);
      }
      ss += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
    }
  }
  float rs = 1.f;
  if (a.norm_w) {
    ss = wave_sum_fast(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kPrepBlock / 64; ++w) t += red[w];
    rs = rsqrtf(t / (float)a.K + a.eps);
  }
  __half* out = a.xh + (size_t)b * a.ldh;
#pragma unroll
  for (int u = 0; u < kPrepMaxVec; ++u) {
    const int i = 4 * (tid + u * kPrepBlock);
    if (i < a.K) {
      float4 t = v[u];
      if (a.norm_w) {
        const float4 nw = *reinterpret_cast<const float4*>(a.norm_w + i);
        t = make_float4(t.x * rs * nw.x, t.y * rs * nw.y, t.z * rs * nw.z, t.w * rs * nw.w);
      }
      const h2_t p0 = {(_Float16)t.x, (_Float16)t.z}, p1 = {(_Float16)t.y, (_Float16)t.w};
      *reinterpret_cast<uint2*>(out + i) = make_uint2(as_u(p0), as_u(p1));
    }
  }
}

void bprep(const BPrepArgs& a, hipStream_t s) {
  if (a.B < 1 || a.K % 128 || a.K > 4 * kPrepBlock * kPrepMaxVec) throw std::runtime_error("bprep: bad shape");
  if (a.zero_n % 4) throw std::runtime_error("bprep: zero_n must be a multiple of 4");
  if (a.swiglu && a.swiglu_group != 32 && a.swiglu_group != 8) throw std::runtime_error("bprep: swiglu group 8 or 32");
  // zero blocks: >= 4 float4 stores per thread, at most 512 blocks
  const int nz = a.zero && a.zero_n ? std::min(512, std::max(1, (a.zero_n / 4 + 4 * kPrepBlock - 1) / (4 * kPrepBlock))) : 0;
  hipLaunchKernelGGL(bprep_kernel, dim3(a.B + nz), dim3(kPrepBlock), 0, s, a);
}

// ---------------------------------------------------------------- launch
static size_t bmm_lds(int B, int spp, int nw) { return (size_t)(nw - 1) * 64 * 16 + 512 + (size_t)B * (spp * 256 + 8) * 2; }

// one-part shapes run 8-wave blocks; two of them must fit a CU's 160 KB of LDS
bool bmm_qkv_fits(int K, int B) { return K % 256 == 0 && B >= 1 && bmm_lds(B, K / 256, 8) <= 80 * 1024; }
// folded norm: the 512-thread staging holds 2 float4 of each of <= 8 rows per thread
bool bmm_norm_fits(int K, int B) { return bmm_qkv_fits(K, B) && K == 4096 && B <= 8; }

bool bmm_supported(int type, int K) {
  if (type != T_Q4_K && type != T_Q5_K && type != T_Q6_K && type != T_Q8_0) return false;
  return K % 256 == 0;  // 256 k per step
}

static int bmm_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      throw std::runtime_error("bmm: cannot query the device's CU count");
    return std::max(1, n);
  }();
  return cus;
}

// The wave-owned launch shape (K parts, steps per part, one block per CU): sets a.spp / a.kparts,
// returns the block count and the dynamic LDS (wt_k: split-K shapes; else the one-part SwiGLU)
static int wt_config(BmmArgs& a, bool wt_k, size_t& lds) {
  int tiles = (a.n_out + 15) / 16;
  for (int i = 1; i < a.nseg; ++i) tiles += (a.seg_rows[i] + 15) / 16;
  const int steps = a.w.K / 256;
  const int cus = bmm_cus();
  int kparts = 1;
  if (wt_k) {  // one 8-wave block per CU: parts = CUs x 8 waves / tiles, >= 2 steps per part
    // (8 parts for the 256-tile shapes; 4 / 16 measured 7 / 13 % slower steps, r3 sweep)
    kparts = std::max(1, std::min(steps / 2, (cus * 8 + tiles / 2) / std::max(1, tiles)));
    if (a.ew) {
      // MoE down (K = the experts' F concatenated): every part inside one expert, the parts of
      // an unrouted expert skipped whole; parts per expert: the count nearest the dense rule
      // whose staged slice fits the LDS and divides the expert's steps
      const int spe = a.steps_per_expert, E = steps / spe;
      int ppe = std::max(1, (kparts + E / 2) / E);
      while (ppe < spe && (spe % ppe || (size_t)a.B * (spe / ppe * 256 + kWtXPad) * 2 > 150 * 1024)) ++ppe;
      kparts = E * ppe;
    }
    if (a.store_out) kparts = 1;  // plain stores: one owner per output
    // the staged slice (B rows x part) stays within the LDS
    while (!a.ew && kparts < steps && (size_t)a.B * ((steps + kparts - 1) / kparts * 256 + kWtXPad) * 2 > 150 * 1024) ++kparts;
  }
  a.spp = (steps + kparts - 1) / kparts;
  a.kparts = kparts = (steps + a.spp - 1) / a.spp;
  // tile groups: one block per CU over all parts, at most 8 tiles (one per wave) per split-K
  // group (two blocks per CU - twice the weight bytes in flight - measured the same, r3 sweep)
  const int G = std::max(1, std::min(std::max(1, cus / kparts), wt_k ? (tiles + 7) / 8 : tiles));
  // more than half the CU's LDS: one block per CU, so the even tile split is an even CU split
  lds = std::max<size_t>(256 + (size_t)a.B * (a.spp * 256 + kWtXPad) * 2, 81 * 1024);
  return G * kparts;
}

// (2 weight steps in flight per wave: 3 / 4 measured 1-4 % slower steps with the IL loop too,
// profiles/README.md round 5)
template <int QT, int EPI>
static void launch_wt_il(int nblk, size_t lds, const BmmArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((bmm_wt_kernel<QT, 2, false, true, true, EPI>), dim3(nblk), dim3(512), lds, s, a);
}

template <int QT>
static void launch_bmm(BmmArgs a, hipStream_t s) {
  int tiles = (a.n_out + 15) / 16;
  for (int i = 1; i < a.nseg; ++i) tiles += (a.seg_rows[i] + 15) / 16;
  const int steps = a.w.K / 256;
  // dense SwiGLU gate/up: wave-owned tiles, 2 steps of weights in flight per wave (3: same
  // time, r3 sweep); plain split-K projections (Wo, down): the same kernel over (K part,
  // 8-tile group) blocks
  const bool wt_sw = a.swiglu_epi && !a.qkv_epi && a.nseg == 1 && (!a.xf || a.w.K == 4096) &&
                     a.B <= 8;
  const bool wt_k = !a.swiglu_epi && (!a.ew || a.steps_per_expert > 0) && !a.qkv_epi && !a.xf && !a.one_part &&
                    a.nseg == 1 && a.B <= 8;
  if (wt_sw || wt_k) {
    size_t lds = 0;
    const int nblk = wt_config(a, wt_k, lds);
    if (a.store_out && a.kparts > 1) throw std::runtime_error("bmm: store_out needs one K part");
    if (a.debug >= 4 && !a.ew) {  // microbenchmarks (wt_body's DBG)
      if (a.debug == 4) hipLaunchKernelGGL((bmm_wt_dbg_kernel<QT, 4>), dim3(nblk), dim3(512), lds, s, a);
      else if (a.debug == 5) hipLaunchKernelGGL((bmm_wt_dbg_kernel<QT, 5>), dim3(nblk), dim3(512), lds, s, a);
      else if (a.debug == 6) hipLaunchKernelGGL((bmm_wt_dbg_kernel<QT, 6>), dim3(nblk), dim3(512), lds, s, a);
      else hipLaunchKernelGGL((bmm_wt_dbg_kernel<QT, 7>), dim3(nblk), dim3(512), lds, s, a);
      return;
    }
    // (x-first staging everywhere: weights-first measured 2.295 vs 2.246 ms per B = 6 step, r5b)
    if (a.ew && bmm_il()) {  // MoE: the experts' SwiGLU gate/up (EPI 1) and grouped down (split-K, EPI 2)
      if (wt_sw) hipLaunchKernelGGL((bmm_wt_kernel<QT, 2, true, true, true, 1>), dim3(nblk), dim3(512), lds, s, a);
      else if (a.kparts > 1) hipLaunchKernelGGL((bmm_wt_kernel<QT, 2, true, true, true, 2>), dim3(nblk), dim3(512), lds, s, a);
      else hipLaunchKernelGGL((bmm_wt_kernel<QT, 2, true, true, true, 0>), dim3(nblk), dim3(512), lds, s, a);
    } else if (a.ew) hipLaunchKernelGGL((bmm_wt_kernel<QT, 2, true, true>), dim3(nblk), dim3(512), lds, s, a);
    else if (bmm_il()) {
      const int epi = wt_sw ? 1 : a.kparts > 1 ? 2 : a.store_out ? 3 : 0;
      if (epi == 1) launch_wt_il<QT, 1>(nblk, lds, a, s);
      else if (epi == 2) launch_wt_il<QT, 2>(nblk, lds, a, s);
      else if (epi == 3) launch_wt_il<QT, 3>(nblk, lds, a, s);
      else launch_wt_il<QT, 0>(nblk, lds, a, s);
    } else {
      hipLaunchKernelGGL((bmm_wt_kernel<QT, 2, false, true>), dim3(nblk), dim3(512), lds, s, a);
    }
    return;
  }
  if (a.zero) throw std::runtime_error("bmm: the zero side job runs on the wave-owned kernels only");
  if (a.store_out && !a.xf && !a.qkv_epi && !a.swiglu_epi && !a.one_part)
    throw std::runtime_error("bmm: store_out needs one K part");
  if (a.qkv_epi || a.swiglu_epi || a.xf || a.one_part) {
    // one K part (the epilogue needs whole rows); 8-wave blocks (the folded norm needs 8), 2 per
    // CU by LDS (16-wave blocks staging x once per CU: 5 % slower steps, r2)
    constexpr int nw1 = 8;
    a.spp = steps;
    a.kparts = 1;
    const size_t lds = bmm_lds(a.B, steps, nw1);
    // blocks per CU: LDS and the 16 waves a CU holds at this kernel's register count
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>((160 * 1024) / lds, 16 / nw1));
    int nb = std::max(1, std::min(tiles, per_cu * bmm_cus()));
    // one tile per Q|K|V block although every block stages the whole x slice: 2-4 tiles per
    // block (fewer stagings, less weight parallelism) measured 1-8 % slower steps (r3 sweep)
    if (a.swiglu_epi) {  // every CU group gets the same number of blocks (the range split assumes it)
      const int G = std::max(1, std::min(bmm_cus(), tiles));
      nb = G * std::max(1, std::min(per_cu, tiles / G));
      a.tile_groups = G;
    }
    hipLaunchKernelGGL((bmm_kernel<QT, nw1, 1>), dim3(nb), dim3(nw1 * 64), lds, s, a, a);
    return;
  }
  // K part: the staged x slice stays <= 32 KB (B rows x part x 2 B); parts are split further
  // (more blocks, more-way atomics) only while there are fewer than ~4 blocks per CU
  const int bp = a.B <= 4 ? 4 : a.B <= 8 ? 8 : 16;
  constexpr int xkb = 32;  // staged-x budget (KB)
  int spp = std::max(1, std::min(steps, 2 * xkb / bp));
  const int want = 4 * bmm_cus();
  while (spp > 4 && (size_t)tiles * ((steps + spp - 1) / spp) < (size_t)want) spp = (spp + 1) / 2;
  // MoE down: every K part inside ONE expert - an unrouted expert's SwiGLU rows were never
  // written (its gate/up tiles are skipped), so its parts must be skipped whole, not mixed in
  if (a.ew && a.steps_per_expert > 0)
    while (a.steps_per_expert % spp) --spp;
  const int kparts = (steps + spp - 1) / spp;
  a.spp = spp;
  a.kparts = kparts;
  // blocks per part: ~4 blocks per CU overall (each block loops over tiles, so its staged x
  // slice - as many bytes as a tile's weights at B = 8 - is amortised over several tiles)
  constexpr int per_cu = 4;
  // blocks past per_cu * CUs would start only when a first-round block retires (a whole
  // block lifetime of tail): the grid stays within one resident round
  const int bpk = std::max(1, std::min(tiles, (per_cu * bmm_cus()) / kparts));
  const size_t lds = bmm_lds(a.B, spp, 4);
  hipLaunchKernelGGL((bmm_kernel<QT, 4, 1>), dim3(bpk * kparts), dim3(256), lds, s, a, a);
}

// split-K Q|K|V: (K part, group of a.tpg tiles of one run) blocks, every wave one tile of the part
template <int QT, int QT2>
static void launch_qkv_sk(BmmArgs a, hipStream_t s) {
  int ta = 0, tb = 0;
  for (int i = 0; i < a.nseg; ++i) {
    const int t = ((i == 0 ? a.n_out : a.seg_rows[i]) + 15) / 16;
    if (i < a.seg_split) ta += t;
    else tb += t;
  }
  const int steps = a.w.K / 256;
  // 4 parts x 8-tile groups measured best at B = 6 (8 x 8: +3 %, 4 x 6 / 2 x 3: +1-4 %, 16 x 6: +15 %)
  const int kparts = std::max(1, std::min(steps, 4));
  a.spp = (steps + kparts - 1) / kparts;
  a.kparts = (steps + a.spp - 1) / a.spp;
  a.tpg = 8;
  const int ga = (ta + a.tpg - 1) / a.tpg, gb = (tb + a.tpg - 1) / a.tpg;
  a.nb1 = ga;
  const dim3 grid((ga + gb) * a.kparts);
  const size_t lds = 256 + (size_t)a.B * (a.spp * 256 + kWtXPad) * 2;
  if constexpr (QT2 == 0) {
    if (bmm_il()) hipLaunchKernelGGL((bmm_sk_kernel<QT, 2, true, true>), grid, dim3(512), lds, s, a);  // (un-RoPE'd sums)
    else hipLaunchKernelGGL((bmm_sk_kernel<QT, 2, true>), grid, dim3(512), lds, s, a);
  } else {
    if (bmm_il()) hipLaunchKernelGGL((bmm_wt2_kernel<QT, QT2, 2, true, true>), grid, dim3(512), lds, s, a);
    else hipLaunchKernelGGL((bmm_wt2_kernel<QT, QT2, 2, true>), grid, dim3(512), lds, s, a);
  }
}

bool bmm_qkv_sk_defers_rope() { return bmm_il(); }

bool bmm_qkv_sk_supported(int tq, int tk, int tv, int K, int B) {
  if (B < 1 || B > 8 || K % 256 || !bmm_supported(tq, K) || !bmm_supported(tk, K) || !bmm_supported(tv, K)) return false;
  const int t2 = tk != tq ? tk : tv;
  if (tk != tq && tv != tk) return false;  // at most two runs: Q [| K] of one type, the rest of another
  if (t2 == tq) return true;
  return tq == T_Q4_K && (t2 == T_Q6_K || t2 == T_Q5_K || t2 == T_Q8_0);
}

static void bmm_check(const BmmArgs& a) {
  if (!bmm_supported(a.w.type, a.w.K)) throw std::runtime_error("bmm: unsupported type / K");
  if (a.B < 1 || a.B > kBmmMaxRows) throw std::runtime_error("bmm: 1 <= B <= 16");
  if (a.nseg < 1 || a.nseg > 3) throw std::runtime_error("bmm: 1 to 3 segments");
  if (a.qkv_epi && (!bmm_qkv_fits(a.w.K, a.B) || a.qkv.head_dim % 2)) throw std::runtime_error("bmm: qkv epilogue");
  if (a.swiglu_epi && (a.qkv_epi || a.nseg != 1 || !bmm_qkv_fits(a.w.K, a.B) || a.n_out % 16 || !a.h_out ||
                       a.ldh_out < a.n_out / 2 || a.ldh_out % 4))
    throw std::runtime_error("bmm: swiglu epilogue");
  if (a.xf && !a.qkv_sk && (!a.norm_w || !bmm_norm_fits(a.w.K, a.B) || a.ldxf < a.w.K || a.ldxf % 4))
    throw std::runtime_error("bmm: folded norm");
  if (a.one_part && !bmm_qkv_fits(a.w.K, a.B)) throw std::runtime_error("bmm: one_part x slice exceeds LDS");
  if (a.ew && (a.ew_ld < 1 || (a.swiglu_epi ? a.tiles_per_expert < 1 || ((a.n_out + 15) / 16) % a.tiles_per_expert
                                            : a.steps_per_expert < 1 || (a.w.K / 256) % a.steps_per_expert)))
    throw std::runtime_error("bmm: expert routing weights need whole experts of tiles / K steps");
  if (a.ew && a.swiglu_epi && (a.n_out + 15) / 16 / a.tiles_per_expert > 64) throw std::runtime_error("bmm: <= 64 experts");
  if (a.ew && !a.swiglu_epi && (a.xf || a.qkv_epi || a.one_part))
    throw std::runtime_error("bmm: the MoE down projection runs split-K (whole-expert parts)");
  if (a.qkv_sk) {
    if (a.B > 8 || a.qkv_epi || a.swiglu_epi || a.ew || a.one_part || a.store_out || !a.qkv.pos || !a.qkv.rope ||
        a.qkv.head_dim % 2 || a.qkv.n_ctx < 1 || a.seg_split < 1 || a.seg_split > a.nseg ||
        (a.seg_split < a.nseg && !bmm_qkv_sk_supported(a.w.type, a.type2, a.type2, a.w.K, a.B)))
      throw std::runtime_error("bmm: split-K Q|K|V arguments");
    if (a.xf && (!a.norm_w || !a.ss_out || a.ldxf < a.w.K || a.ldxf % 4)) throw std::runtime_error("bmm: split-K Q|K|V norm");
  }
  if (a.ss_out && !(a.qkv_sk && a.xf)) throw std::runtime_error("bmm: ss_out needs the split-K Q|K|V norm");
  if (a.zero && (a.zero_n % 4 || reinterpret_cast<uintptr_t>(a.zero) % 16)) throw std::runtime_error("bmm: zero side job alignment");
}

void bmm(const BmmArgs& a0, hipStream_t s) {
  BmmArgs a = a0;
  bmm_check(a);
  if (a.n_out <= 0) return;
  if (a.qkv_sk) {
    const bool two = a.seg_split < a.nseg;
    const int t2 = two ? a.type2 : 0;
    if (a.w.type == T_Q4_K && t2 == T_Q6_K) launch_qkv_sk<T_Q4_K, T_Q6_K>(a, s);
    else if (a.w.type == T_Q4_K && t2 == T_Q5_K) launch_qkv_sk<T_Q4_K, T_Q5_K>(a, s);
    else if (a.w.type == T_Q4_K && t2 == T_Q8_0) launch_qkv_sk<T_Q4_K, T_Q8_0>(a, s);
    else if (t2 != 0) throw std::runtime_error("bmm: split-K Q|K|V type pair");
    else if (a.w.type == T_Q4_K) launch_qkv_sk<T_Q4_K, 0>(a, s);
    else if (a.w.type == T_Q5_K) launch_qkv_sk<T_Q5_K, 0>(a, s);
    else if (a.w.type == T_Q6_K) launch_qkv_sk<T_Q6_K, 0>(a, s);
    else launch_qkv_sk<T_Q8_0, 0>(a, s);
    return;
  }
  switch (a.w.type) {
    case T_Q4_K: launch_bmm<T_Q4_K>(a, s); break;
    case T_Q5_K: launch_bmm<T_Q5_K>(a, s); break;
    case T_Q6_K: launch_bmm<T_Q6_K>(a, s); break;
    case T_Q8_0: launch_bmm<T_Q8_0>(a, s); break;
    default: throw std::runtime_error("bmm: unsupported weight type");
  }
}

bool bmm_ffn_chain_supported(const BmmArgs& gu, const BmmArgs& dn) {
  return gu.swiglu_epi && !gu.ew && !gu.qkv_epi && gu.nseg == 1 && gu.B <= 8 && (!gu.xf || gu.w.K == 4096) &&
         !dn.swiglu_epi && !dn.ew && !dn.qkv_epi && !dn.xf && !dn.one_part && !dn.store_out && dn.nseg == 1 &&
         dn.B == gu.B && gu.w.type == T_Q4_K && (dn.w.type == T_Q4_K || dn.w.type == T_Q6_K) &&
         dn.xh == gu.h_out && dn.ldh == gu.ldh_out && dn.w.K == gu.n_out / 2;
}

void bmm_ffn_chain(const BmmArgs& gu0, const BmmArgs& dn0, int* cnt, int* err, hipStream_t s) {
  if (!bmm_ffn_chain_supported(gu0, dn0) || !cnt) throw std::runtime_error("bmm_ffn_chain: unsupported shapes");
  BmmArgs gu = gu0, dn = dn0;
  bmm_check(gu);
  bmm_check(dn);
  size_t lds1 = 0, lds2 = 0;
  const int n1 = wt_config(gu, false, lds1), n2 = wt_config(dn, true, lds2);
  // a consumer block takes K part kp = bid % kparts: its 256 * spp features are 32 * spp gate/up tiles
  gu.chain_role = kChainProduce; gu.chain_cnt = cnt; gu.chain_tpp = 32 * dn.spp;
  dn.chain_role = kChainConsume; dn.chain_cnt = cnt; dn.chain_tpp = 32 * dn.spp; dn.chain_tiles = (gu.n_out + 15) / 16;
  dn.chain_err = err;
  if (dn.kparts > kChainStagedPart) throw std::runtime_error("bmm_ffn_chain: too many K parts for the counters");
  dn.chain_staged = n1;  // every gate/up block has read its x rows before any down block adds into them
  dn.chain_poll = 8;  // (1-40 s_sleep units between polls measured the same, r5d)
  gu.nb1 = n1;
  const dim3 grid(n1 + n2);
  const size_t lds = std::max(lds1, lds2);
  if (bmm_il()) {
    if (dn.w.type == T_Q6_K) hipLaunchKernelGGL((bmm_chain_kernel<T_Q4_K, T_Q6_K, true>), grid, dim3(512), lds, s, gu, dn);
    else hipLaunchKernelGGL((bmm_chain_kernel<T_Q4_K, T_Q4_K, true>), grid, dim3(512), lds, s, gu, dn);
  } else {
    if (dn.w.type == T_Q6_K) hipLaunchKernelGGL((bmm_chain_kernel<T_Q4_K, T_Q6_K>), grid, dim3(512), lds, s, gu, dn);
    else hipLaunchKernelGGL((bmm_chain_kernel<T_Q4_K, T_Q4_K>), grid, dim3(512), lds, s, gu, dn);
  }
}

bool bmm_wo_ffn_chain_supported(const BmmArgs& wo, const BmmArgs& gu, const BmmArgs& dn) {
  return bmm_il() && bmm_ffn_chain_supported(gu, dn) && gu.xf && wo.w.type == T_Q4_K && !wo.ew && !wo.xf &&
         !wo.swiglu_epi && !wo.qkv_epi && !wo.one_part && !wo.store_out && !wo.zero && wo.nseg == 1 && wo.B == gu.B &&
         wo.out == gu.xf && wo.ldo == gu.ldxf && wo.n_out == gu.w.K;
}

void bmm_wo_ffn_chain(const BmmArgs& wo0, const BmmArgs& gu0, const BmmArgs& dn0, int* cnt, int* err, hipStream_t s) {
  if (!bmm_wo_ffn_chain_supported(wo0, gu0, dn0) || !cnt) throw std::runtime_error("bmm_wo_ffn_chain: unsupported shapes");
  BmmArgs wo = wo0, gu = gu0, dn = dn0;
  bmm_check(wo);
  bmm_check(gu);
  bmm_check(dn);
  size_t lds0 = 0, lds1 = 0, lds2 = 0;
  const int n0 = wt_config(wo, true, lds0), n1 = wt_config(gu, false, lds1), n2 = wt_config(dn, true, lds2);
  if (wo.kparts < 2 || dn.kparts < 2) throw std::runtime_error("bmm_wo_ffn_chain: one-part Wo / down");
  if (dn.kparts > kChainWoPart) throw std::runtime_error("bmm_wo_ffn_chain: too many K parts for the counters");
  wo.chain_role = kChainWoDone; wo.chain_cnt = cnt; wo.nb1 = n0;
  gu.chain_role = kChainProduce | kChainWaitWo; gu.chain_cnt = cnt; gu.chain_tpp = 32 * dn.spp; gu.chain_wo = n0;
  gu.chain_err = err; gu.chain_poll = 8; gu.nb1 = n1;
  dn.chain_role = kChainConsume; dn.chain_cnt = cnt; dn.chain_tpp = 32 * dn.spp; dn.chain_tiles = (gu.n_out + 15) / 16;
  dn.chain_err = err; dn.chain_staged = n1; dn.chain_poll = 8;
  const dim3 grid(n0 + n1 + n2);
  const size_t lds = std::max(lds0, std::max(lds1, lds2));
  if (dn.w.type == T_Q6_K) hipLaunchKernelGGL((bmm_chain3_kernel<T_Q4_K, T_Q4_K, T_Q6_K>), grid, dim3(512), lds, s, wo, gu, dn);
  else hipLaunchKernelGGL((bmm_chain3_kernel<T_Q4_K, T_Q4_K, T_Q4_K>), grid, dim3(512), lds, s, wo, gu, dn);
}

bool bmm_qkv2(const BmmArgs& a0, const BmmArgs& b0, hipStream_t s) {
  if (!a0.qkv_epi || !b0.qkv_epi || a0.B != b0.B || a0.w.K != b0.w.K || a0.n_out <= 0 || b0.n_out <= 0)
    return false;
  if ((a0.xf == nullptr) != (b0.xf == nullptr)) return false;
  BmmArgs a = a0, b = b0;
  bmm_check(a);
  bmm_check(b);
  auto tiles_of = [](const BmmArgs& x) {
    int t = (x.n_out + 15) / 16;
    for (int i = 1; i < x.nseg; ++i) t += (x.seg_rows[i] + 15) / 16;
    return t;
  };
  const int steps = a.w.K / 256;
  a.spp = b.spp = steps;
  a.kparts = b.kparts = 1;
  const size_t lds = bmm_lds(a.B, steps, 8);
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>((160 * 1024) / lds, 2));
  const int ta = tiles_of(a), tb = tiles_of(b);
  const int cap = std::max(2, std::min(per_cu * bmm_cus(), ta + tb));
  // blocks in proportion to the runs' tiles, each run at least one block, within one resident round
  int na = std::min(ta, std::max(1, (int)((long long)cap * ta / (ta + tb))));
  int nbb = std::min(tb, std::max(1, cap - na));
  a.nb1 = na;
  const dim3 grid(na + nbb), blk(512);
  const int ta_ = a.w.type, tb_ = b.w.type;
  if (ta_ == T_Q4_K && tb_ == T_Q6_K) hipLaunchKernelGGL((bmm_kernel<T_Q4_K, 8, 1, T_Q6_K>), grid, blk, lds, s, a, b);
  else if (ta_ == T_Q4_K && tb_ == T_Q5_K) hipLaunchKernelGGL((bmm_kernel<T_Q4_K, 8, 1, T_Q5_K>), grid, blk, lds, s, a, b);
  else return false;
  return true;
}

// ---------------------------------------------------------------- prefill GEMM on the tile16 copy
// Y[T][N] = X[T][K] . W^T for prompt chunks, reading the same tile16 copy and the
// same dequantisation as the batched decode - but where a decode wave's A fragments meet one
// B column block (<= 16 rows), here they serve TM / 16 token groups: the per-weight VALU work
// is spread over TM tokens and the kernel is paced by the matrix cores, not by issue.
//
// Block = 8 waves x 2 tiles (256 weight rows) x TM tokens; per 128-k half step h of 256-k step
// s (the chunks 8s + 4h + kq cover k [256s + 128h, +128) for every type, see chunk_runs):
//   X[t0 .. t0 + TM)[that k range] f16 staged in LDS (double buffered, the next half's global
//   loads held in registers during this half's MFMAs), each wave's two tiles' raw weights one
//   half ahead (ping-pong, fixed roles), dequantised once per half into A fragments; per token
//   group g and run m ONE ds_read_b128 (the B operand, 16 tokens x 8 k) feeds the MFMAs of both
//   tiles (LDS at half rate: 512 B per 16-cycle MFMA per SIMD).
// Split-K (grid z) for the narrow projections: partial tiles meet by atomic add.
// Epilogues: STORE (+ resid), ADD (residual in place), SWIGLU (the tile16 SwiGLU copy's tile =
// 8 gate + 8 up rows of the same features: lane kq < 2 takes up from lane + 32 and writes
// silu(g) * u as f16 in the 4-group k order - the next gemm_t16's X).
// Staged X rows are 128 halves (no pad) with their 16-B units XOR-swizzled by the token's row in
// its 16-row group (unit u of row r at u ^ (r & 15)): ds_read_b128 serves a wave in lane groups
// {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ... - two kq values x 8 token rows per group - and
// no uniform pitch keeps those 16 lanes apart (136 halves: 2-way, measured 2.1 conflict cycles
// per LDS instruction); the swizzle makes them conflict-free for the Q4_K / Q5_K / Q6_K runs
// (Q8_0's stay 2-way).
static constexpr int kT16Pitch = 128;

// KW = 2: the block's K range in two halves, one group of NWV waves each (two waves per SIMD where
// the grid holds at most one block per CU), the groups' tiles summed through LDS at the end - the
// second wave per SIMD without split-K atomics.
template <int QT, int EPI, int TM, int NWV, int KW>
__global__ __launch_bounds__(NWV * 64 * KW) void gemm_t16_kernel(GemmT16Args a) {
  constexpr int NG = TM / 16, NT = NWV * 64;  // NT: the threads of one K group
  constexpr int XL = TM * 16 / NT;  // 16-B X pieces per thread per half step
  constexpr int SB = t16_step_bytes(QT);
  __shared__ __attribute__((aligned(16))) __half xs[2][KW][TM * kT16Pitch];
  // (wave-uniform by construction; readfirstlane tells the compiler, so the weight tiles' buffer
  // resources stay scalar instead of waterfall loops)
  const int kg = KW > 1 ? __builtin_amdgcn_readfirstlane((int)threadIdx.x / NT) : 0;  // this thread's K group
  const int tid = threadIdx.x - kg * NT, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int K = a.w.K, steps = K >> 8;
  const int ntiles = (a.w.rows + 15) >> 4;
  const int tile0 = blockIdx.x * 2 * NWV + 2 * wave;  // this wave's tiles: tile0, tile0 + 1
  const int t0 = blockIdx.y * TM;
  if (a.seg_dev) {  // grouped form: this expert's rows of the gathered buffers
    const int r0 = a.seg_dev[0];
    a.T = a.seg_dev[1] - r0;
    if (t0 >= a.T) return;  // whole block, before any barrier
    a.x += (size_t)r0 * K;
    if (a.out) a.out += (size_t)r0 * a.ldo;
    if (a.out_h) a.out_h += (size_t)r0 * a.ldh;
  }
  const int spz = (steps + (int)gridDim.z - 1) / (int)gridDim.z;
  const int sb0 = blockIdx.z * spz, se = min(steps, sb0 + spz);
  if (sb0 >= se) return;  // whole block, before any barrier
  const int spg = (se - sb0) / KW;  // steps per K group (the launcher keeps them whole)
  const int sb = sb0 + kg * spg;    // this group's first step
  const int nh = 2 * spg;
  const size_t tstride = a.tile_stride ? a.tile_stride : (size_t)steps * SB;
  auto tile_base = [&](int t) __attribute__((always_inline)) {  // (stacked segments: Q|K|V)
    t = min(t, ntiles - 1);
    const uint8_t* b = a.w.base;
    if (a.nwseg > 1 && t >= a.wseg_tiles[0]) {
      t -= a.wseg_tiles[0];
      b = a.wseg_base[1];
      if (a.nwseg > 2 && t >= a.wseg_tiles[1]) {
        t -= a.wseg_tiles[1];
        b = a.wseg_base[2];
      }
    }
    return b + (size_t)t * tstride + (size_t)a.step0 * SB;
  };
  const uint8_t* wt0 = tile_base(tile0);
  const uint8_t* wt1 = tile_base(tile0 + 1);
  f4_t acc[2][NG];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[j][g] = f4_t{0.f, 0.f, 0.f, 0.f};
  static_assert(XL >= 2 && XL <= 8 && XL * NT == TM * 16, "X pieces per thread");
  // X piece p = tid + NT j: token p / 16, 16-B column p % 16 of the 128-k slice (rows past T
  // load row T - 1: finite values whose outputs are never stored). Named registers, not an
  // array: the array was put in scratch.
  uint4 x0, x1, x2, x3, x4, x5, x6, x7;
  // the X and weight loads go through buffer resources - per-lane 32-bit voffsets fixed for the
  // kernel, the step's offset a uniform soffset - instead of 64-bit address arithmetic per load:
  // 257 -> 240 VALU per 64 MFMAs in the main loop of this VALU-bound kernel; 387-token admission
  // 12.8 -> 11.2 ms (profiles/README.md, round 6)
  const auto rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(a.x), 0, 0x7FFFFFFF, 0x00020000);
  int xvo[XL];  // bytes: T x K x 2 stays far below 2 GB (T <= 4096 rows, K <= 28672)
#pragma unroll
  for (int j = 0; j < XL; ++j) xvo[j] = (min(t0 + ((tid + NT * j) >> 4), a.T - 1) * K + 8 * (tid & 15)) * 2;
  auto xld = [&](int j, int k0) __attribute__((always_inline)) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsx, xvo[j], k0 * 2, 0));
  };
  auto load_x = [&](int i) __attribute__((always_inline)) {
    const int k0 = (sb + (i >> 1)) * 256 + 128 * (i & 1);
    x0 = xld(0, k0);
    x1 = xld(1, k0);
    if constexpr (XL > 2) x2 = xld(XL > 2 ? 2 : 0, k0);
    if constexpr (XL > 3) x3 = xld(XL > 3 ? 3 : 0, k0);
    if constexpr (XL > 4) x4 = xld(XL > 4 ? 4 : 0, k0);
    if constexpr (XL > 5) x5 = xld(XL > 5 ? 5 : 0, k0);
    if constexpr (XL > 6) x6 = xld(XL > 6 ? 6 : 0, k0);
    if constexpr (XL > 7) x7 = xld(XL > 7 ? 7 : 0, k0);
  };
  auto store_x = [&](int buf) __attribute__((always_inline)) {
    __half* d = &xs[buf][kg][(tid >> 4) * kT16Pitch + 8 * ((tid & 15) ^ ((tid >> 4) & 15))];
    constexpr int J = (NT / 16) * kT16Pitch;  // piece j + 1 is NT / 16 tokens further (same swizzle)
    *reinterpret_cast<uint4*>(d) = x0;
    *reinterpret_cast<uint4*>(d + J) = x1;
    if constexpr (XL > 2) *reinterpret_cast<uint4*>(d + 2 * J) = x2;
    if constexpr (XL > 3) *reinterpret_cast<uint4*>(d + 3 * J) = x3;
    if constexpr (XL > 4) *reinterpret_cast<uint4*>(d + 4 * J) = x4;
    if constexpr (XL > 5) *reinterpret_cast<uint4*>(d + 5 * J) = x5;
    if constexpr (XL > 6) *reinterpret_cast<uint4*>(d + 6 * J) = x6;
    if constexpr (XL > 7) *reinterpret_cast<uint4*>(d + 7 * J) = x7;
  };
  const auto rw0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wt0), 0, 0x7FFFFFFF, 0x00020000);
  const auto rw1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wt1), 0, 0x7FFFFFFF, 0x00020000);
  auto load_w = [&](int i, BRawT<QT>& w0, BRawT<QT>& w1) __attribute__((always_inline)) {
    const int s = sb + (i >> 1), h = i & 1;
    tload_rs<QT, false>(w0, rw0, s * SB, h, lane, r16, kq);  // (cached: each tile serves several token blocks)
    tload_rs<QT, false>(w1, rw1, s * SB, h, lane, r16, kq);
  };
  auto half = [&](int i, const BRawT<QT>& w0, const BRawT<QT>& w1) __attribute__((always_inline)) {
    const int s = sb + (i >> 1), h = i & 1;
    const int c = 8 * s + 4 * h + kq;
    int off_lo, off_hi;
    chunk_runs<QT>(c, off_lo, off_hi);
    off_lo -= 256 * s + 128 * h;
    off_hi -= 256 * s + 128 * h;
    HFrag F0, F1;
    dequant_frags<QT>(w0, c, F0);
    dequant_frags<QT>(w1, c, F1);
    const __half* xb = &xs[i & 1][kg][r16 * kT16Pitch];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int u = (((m < 2 ? off_lo : off_hi) >> 3) + (m & 1)) ^ r16;  // swizzled 16-B unit
        const uint4 bv = *reinterpret_cast<const uint4*>(xb + g * 16 * kT16Pitch + 8 * u);
        const int dw = 2 * (m & 1), sh = (m >> 1) * 2;
        const uint4 a0 = make_uint4(F0.w[4 * dw + sh], F0.w[4 * dw + sh + 1], F0.w[4 * dw + 4 + sh], F0.w[4 * dw + 5 + sh]);
        const uint4 a1 = make_uint4(F1.w[4 * dw + sh], F1.w[4 * dw + sh + 1], F1.w[4 * dw + 4 + sh], F1.w[4 * dw + 5 + sh]);
        acc[0][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, a0), __builtin_bit_cast(h8_t, bv), acc[0][g], 0, 0, 0);
        acc[1][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, a1), __builtin_bit_cast(h8_t, bv), acc[1][g], 0, 0, 0);
      }
    }
  };
  BRawT<QT> wa0, wa1, wb0, wb1;  // ping-pong weight buffers with fixed roles (no rotating copy)
  load_x(0);
  load_w(0, wa0, wa1);
  store_x(0);
  lds_barrier();
  // nh is even (whole 256-k steps). The loads past the last half are clamped repeats and the
  // last stores go to the buffer nobody reads any more: no conditional around a load (a
  // load under a branch drains vmcnt at the join, and the conditional X slice went to scratch)
  for (int i = 0; i < nh; i += 2) {
    // even half: compute from A, load B (and the next X slice)
    load_w(i + 1, wb0, wb1);
    load_x(i + 1);
    half(i, wa0, wa1);
    store_x((i + 1) & 1);
    lds_barrier();
    // odd half: compute from B, load A
    load_w(min(i + 2, nh - 1), wa0, wa1);
    load_x(min(i + 2, nh - 1));
    half(i + 1, wb0, wb1);
    store_x(i & 1);
    lds_barrier();
  }
  if constexpr (KW > 1) {  // group 1's tiles into LDS (the X buffers are free), group 0 adds them
    static_assert(2 * NG * NT * 16 <= sizeof(xs), "the K groups' reduction fits the X buffers");
    f4_t* red = reinterpret_cast<f4_t*>(&xs[0][0][0]);
    if (kg == 1) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < NG; ++g) red[((j * NG + g) * NWV + wave) * 64 + lane] = acc[j][g];
    }
    lds_barrier();
    if (kg == 1) return;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[j][g] += red[((j * NG + g) * NWV + wave) * 64 + lane];
  }
  // ---- epilogue: acc[j][g][e] = (weight row 16 tile + 4 kq + e, token t0 + 16 g + r16)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tile = tile0 + j;
    if (tile >= ntiles) continue;  // wave-uniform
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int t = t0 + 16 * g + r16;
      const f4_t v = acc[j][g];
      if constexpr (EPI == GEMM_SWIGLU) {
        f4_t u;
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = __shfl_xor(v[e], 32);
        const int f = 8 * tile + 4 * kq;
        if (kq < 2 && t < a.T && f < (a.w.rows >> 1)) {
          float hv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = v[e] / (1.f + __expf(-v[e])) * u[e];
          const __half2 p0 = __floats2half2_rn(hv[0], hv[2]), p1 = __floats2half2_rn(hv[1], hv[3]);
          *reinterpret_cast<uint2*>(a.out_h + (size_t)t * a.ldh + f) =
              make_uint2(__builtin_bit_cast(unsigned, p0), __builtin_bit_cast(unsigned, p1));
        }
      } else {
        const int n = 16 * tile + 4 * kq;
        if (t < a.T && n < a.w.rows) {
          float* o = a.out + (size_t)t * a.ldo + n;
          if (gridDim.z > 1) {  // split-K partials (STORE outputs pre-zeroed, resid added once)
            f4_t w = v;
            if (EPI == GEMM_STORE && a.resid && blockIdx.z == 0) {
              const float4 r = *reinterpret_cast<const float4*>(a.resid + (size_t)t * a.ldo + n);
              w += f4_t{r.x, r.y, r.z, r.w};
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) atomicAdd(o + e, w[e]);
          } else {
            float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
            if (EPI == GEMM_ADD) r = *reinterpret_cast<const float4*>(o);
            else if (a.resid) r = *reinterpret_cast<const float4*>(a.resid + (size_t)t * a.ldo + n);
            *reinterpret_cast<float4*>(o) = make_float4(r.x + v[0], r.y + v[1], r.z + v[2], r.w + v[3]);
          }
        }
      }
    }
  }
}

// two K groups per block for the narrow prefill projections (LFK_T16_KW=0/1 A/B; read once)
static bool t16_kw() {
  static const bool on = [] {
    const char* e = std::getenv("LFK_T16_KW");
    return e ? e[0] != '0' : true;
  }();
  return on;
}

template <int QT, int EPI>
static void launch_gemm_t16(const GemmT16Args& a, hipStream_t s) {
  // block shape (waves x 32 rows, TM tokens), measured over T = 384-2304 on the 8B shapes
  // (profiles/README.md, round 3): the SwiGLU gate/up (28672 rows) on 8 x 64 (8 x 128 from
  // 2048 tokens: twice the fragment reuse once the grid is many rounds deep); the 4096- and
  // 1024-row projections on 4 x 64 - 4 blocks per CU - then split over K (partials by atomic
  // add) only while the grid does not cover the CUs, >= 2 steps (512 k) per part.
  // a.cfg = waves * 1000 + tokens pins one (tools/gemm_bench.py --cfg).
  const int ntiles = (a.w.rows + 15) / 16, steps = a.w.K / 256, cus = bmm_cus();
  // grouped: size the shape and split for the expected rows, launch for the most
  const int rows = a.seg_dev ? std::max(1, std::min(a.T, a.rows_hint > 0 ? a.rows_hint : a.T)) : a.T;
  int nw = 4, tm = 64;
  const int pin_nw = a.cfg / 1000, pin_tm = a.cfg % 1000;
  if (((pin_nw == 8 && (pin_tm == 128 || pin_tm == 64)) || (pin_nw == 4 && (pin_tm == 64 || pin_tm == 128)))) {
    nw = pin_nw;
    tm = pin_tm;
  } else if (EPI == GEMM_SWIGLU) {
    // (round 6, tools/gemm_bench.py --only gateup, alternating twice: T = 300 4 x 64 121 / 120 us vs
    // 8 x 64 134 / 135; T = 512 4 x 128 168 / 167 vs 181 / 177; T = 1024 4 x 128 303 / 304 vs 317 /
    // 322; T = 387 all within 2 %; T = 2304 8 x 128 best)
    nw = rows >= 2048 ? 8 : rows >= 448 || rows <= 320 ? 4 : 8;
    tm = rows >= 448 ? 128 : 64;
  }
  const int gx = (ntiles + 2 * nw - 1) / (2 * nw), gy = (a.T + tm - 1) / tm, gy_busy = (rows + tm - 1) / tm;
  // split-K (partials by atomic add) only for long K, up to two resident rounds: at K = 4096 the
  // atomics cost more than the idle CUs (Q / Wo at T = 387: 57 us split in 2 vs 37 us whole at
  // T = 512), at K = 14336 the second wave per SIMD pays (down: 115 us split in 2 at T = 387 vs
  // 152 us whole at T = 512; profiles/README.md, round 6); tiny grids (a lone K / V) still split
  // two K groups per block where the grid leaves CUs with one 4-wave block or none (whole steps
  // per group; the grouped MoE form keeps its split-K sizing)
  const int kw = EPI != GEMM_SWIGLU && nw == 4 && tm == 64 && a.cfg == 0 && !a.seg_dev && t16_kw() &&
                         gx * gy_busy <= cus && steps % 2 == 0 ? 2 : 1;
  int split = 1;
  if (EPI != GEMM_SWIGLU && kw == 1)
    while (steps / (split * 2) >= 2 &&
           ((steps / (split * 2) >= 12 && gx * gy_busy * split * 2 <= 2 * cus) || gx * gy_busy * split * 4 <= cus))
      split *= 2;
  const int spz = (steps + split - 1) / split;
  split = (steps + spz - 1) / spz;  // no empty parts
  if (a.seg_dev && split > 1 && EPI != GEMM_STORE) throw std::runtime_error("gemm_t16: grouped split-K needs STORE");
  if (split > 1 && EPI == GEMM_STORE && !a.out_zeroed) {
    if (a.seg_dev) throw std::runtime_error("gemm_t16: grouped split-K STORE needs a pre-zeroed output");
    const hipError_t e = hipMemset2DAsync(a.out, sizeof(float) * a.ldo, 0, sizeof(float) * a.w.rows, a.T, s);
    if (e != hipSuccess) throw std::runtime_error("gemm_t16: memset failed");
  }
  const dim3 grid(gx, gy, split);
  if (nw == 8 && tm == 128) hipLaunchKernelGGL((gemm_t16_kernel<QT, EPI, 128, 8, 1>), grid, dim3(512), 0, s, a);
  else if (nw == 4 && tm == 128) hipLaunchKernelGGL((gemm_t16_kernel<QT, EPI, 128, 4, 1>), grid, dim3(256), 0, s, a);
  else if (nw == 8) hipLaunchKernelGGL((gemm_t16_kernel<QT, EPI, 64, 8, 1>), grid, dim3(512), 0, s, a);
  else if (kw == 2) hipLaunchKernelGGL((gemm_t16_kernel<QT, EPI, 64, 4, 2>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((gemm_t16_kernel<QT, EPI, 64, 4, 1>), grid, dim3(256), 0, s, a);
}

template <int QT>
static void gemm_t16_epi(const GemmT16Args& a, int epi, hipStream_t s) {
  switch (epi) {
    case GEMM_STORE: launch_gemm_t16<QT, GEMM_STORE>(a, s); break;
    case GEMM_ADD: launch_gemm_t16<QT, GEMM_ADD>(a, s); break;
    case GEMM_SWIGLU: launch_gemm_t16<QT, GEMM_SWIGLU>(a, s); break;
    default: throw std::runtime_error("gemm_t16: bad epilogue");
  }
}

void gemm_t16(const GemmT16Args& a, int epi, hipStream_t s) {
  if (a.T <= 0) return;
  if (!bmm_supported(a.w.type, a.w.K) || !a.w.base || !a.x) throw std::runtime_error("gemm_t16: unsupported type / K");
  if (a.w.rows % 16) throw std::runtime_error("gemm_t16: rows must be a multiple of 16");
  if (a.nwseg < 1 || a.nwseg > 3) throw std::runtime_error("gemm_t16: 1-3 stacked segments");
  if ((long long)a.T * a.w.K * 2 >= (1LL << 31)) throw std::runtime_error("gemm_t16: X exceeds the 2 GB buffer offsets");
  if (a.nwseg > 1) {
    int t = a.wseg_tiles[0];
    for (int i = 1; i < a.nwseg; ++i) {
      if (!a.wseg_base[i] || a.wseg_tiles[i] < 1) throw std::runtime_error("gemm_t16: stacked segment");
      t += a.wseg_tiles[i];
    }
    if (a.wseg_tiles[0] < 1 || t * 16 != a.w.rows || a.tile_stride || a.step0 || a.seg_dev)
      throw std::runtime_error("gemm_t16: stacked segments must cover the rows (plain matrices)");
  }
  if (epi == GEMM_SWIGLU) {
    if (!a.out_h || a.ldh % 4 || a.ldh < a.w.rows / 2) throw std::runtime_error("gemm_t16: SwiGLU output");
  } else if (!a.out || a.ldo % 4 || a.ldo < a.w.rows || (a.resid && epi != GEMM_STORE)) {
    throw std::runtime_error("gemm_t16: output");
  }
  if (reinterpret_cast<uintptr_t>(a.x) % 16) throw std::runtime_error("gemm_t16: X must be 16-byte aligned");
  switch (a.w.type) {
    case T_Q4_K: gemm_t16_epi<T_Q4_K>(a, epi, s); break;
    case T_Q5_K: gemm_t16_epi<T_Q5_K>(a, epi, s); break;
    case T_Q6_K: gemm_t16_epi<T_Q6_K>(a, epi, s); break;
    default: gemm_t16_epi<T_Q8_0>(a, epi, s); break;
  }
}

}  // namespace lfk
