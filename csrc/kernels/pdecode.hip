// Persistent decode step: see pdecode.h for the dataflow and the reasons.
//
// Workgroup = 8 waves on one CU: wave 0 is the LOADER (LDS-DMA of this CU's
// weight slices into an nslot-deep ring, in consumption order, whole token),
// waves 1..7 are CONSUMERS (granule gathers, integer-dot row slices out of the
// ring, epilogues, attention). The loader never joins a barrier: the ring is
// driven by two LDS counters (filled = items landed, freed = consumer-wave
// releases), the consumers meet at an LDS counter barrier (csync).
//
// Ring row format (pd_pack_rows): one row of a quantised matrix, its fields back to
// back, every field 16-B aligned, and EVERY type in the same chunk order: chunk c of
// superblock sb (32 weights, 16 B of 4-bit data) multiplies x[sb*256 + 64g + 16h + i] (lo,
// i < 16) and x[... + 32] (hi), g = (c & 7) >> 1, h = c & 1 - the native Q4_K order. Q6_K
// and Q8_0 rows are re-laid into it at pack time (lossless), so a consumer wave holds
// the activation chunks of its blocks in registers for a whole stage whatever the types.
//   Q4_K: meta[nsb][16] | qs[nsb][128]
//   Q5_K: meta[nsb][16] | qh[nsb][32] | qs[nsb][128]
//   Q6_K: sc[nsb][16] | d[nsb] (f16, padded to 16 B) | qh'[chunk][8] | ql'[chunk][16]
//         (ql' byte i: low 4 bits of lo value i | of hi value i << 4; qh' = two words, the
//         2 high bits of value 4k+m of a half at bit 8m+2k)
//   Q8_0: d[nb] (f16, padded to 16 B) | qs'[chunk][32] (lo half from block 8sb+2g, hi half
//         from block 8sb+2g+1, bytes [16h, 16h+16) of each)
// Activations are int8 with ONE f32 scale per 8 values (finer than the per-32
// blocks of the launch-per-op path), so a q8 block never straddles two
// producing CUs: every CU quantises exactly the 8-blocks it owns.
#include <cfloat>

#include "pdecode.h"
#include "qdot.h"

namespace lfk {

namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) int gi32;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
// LDS-qualified pointers for the out-of-line item code (a generic pointer argument
// would compile the ring and activation reads to flat loads)
#define LDS_AS __attribute__((address_space(3)))
typedef LDS_AS const uint8_t lds_u8;
typedef LDS_AS const int8_t lds_i8;
typedef LDS_AS const float lds_cf;
typedef LDS_AS float lds_f;
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int4 lds_i4(LDS_AS const void* p) {
  const i32x4_t v = *reinterpret_cast<LDS_AS const i32x4_t*>(p);
  return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 lds_f2(LDS_AS const void* p) {
  const f32x2_t v = *reinterpret_cast<LDS_AS const f32x2_t*>(p);
  return make_float2(v.x, v.y);
}
// The launch arguments live in a device buffer read through the constant address space
// (s_load, scalar-cached): kept as a by-value kernel argument, the compiler re-loaded
// fields from the kernarg segment inside the hot loops under SGPR pressure.
typedef const __attribute__((address_space(4))) PDecodeArgs CA;
__device__ __forceinline__ long long clk() { return (long long)__builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ uint32_t pd_row_bytes_dev(int type, int K) {
  switch (type) {
    case T_Q4_K: return (uint32_t)(K / 256) * 144;
    case T_Q5_K: return (uint32_t)(K / 256) * 176;
    case T_Q6_K: return (uint32_t)(K / 256) * 208 + (((K / 256) * 2 + 15) & ~15);
    default: return (uint32_t)(K / 32) * 32 + (((K / 32) * 2 + 15) & ~15);
  }
}
__device__ __forceinline__ size_t dump_stride(CA& a) { return (size_t)2 * a.nq + 2 * a.nkv + 2 * a.d + a.F; }
// descriptors through the constant address space: wave-uniform indices -> s_load (a vector
// load would be counted by vmcnt and make the loader's waits drain its own LDS-DMA stream)
typedef const __attribute__((address_space(4))) PdItem citem;
typedef const __attribute__((address_space(4))) PdLayer clayer;
__device__ __forceinline__ PdItem item_at(CA& a, int i) {
  citem* p = (citem*)a.items + i;
  PdItem r;
  r.off = p->off; r.row_bytes = p->row_bytes; r.dma_kb = p->dma_kb; r.rows = p->rows; r.row0 = p->row0;
  r.stage = p->stage; r.type = p->type;
  return r;
}
__device__ __forceinline__ PdLayer layer_at(CA& a, int l) {
  clayer* p = (clayer*)a.layers + l;
  PdLayer r;
  r.wbase = p->wbase; r.cu_bytes = p->cu_bytes; r.item0 = p->item0; r.nitems = p->nitems;
  r.attn_norm = p->attn_norm; r.ffn_norm = p->ffn_norm;
  return r;
}

constexpr int kThreads = kPdThreads;
constexpr int kLoaders = kPdLoaderWaves;        // loader waves (each its own vmcnt budget of in-flight DMA)
constexpr int kNCW = kPdConsumerWaves;          // consumer waves
constexpr int kAttW = 4;                 // consumer waves that read keys (16 keys each per pass)
constexpr long long kSpinTicks = 4000000;  // 40 ms of the 100 MHz wall clock per wait

// LDS control words (ints at the start of the dynamic region)
// Per ring slot: C_FILLED0 + slot = index + 1 of the last item landed in it (written by
// the loader wave that owns the item), C_FREED0 + slot = consumer-wave releases of it,
// cumulative. Per slot, not one sum: with one sum a wave running several items ahead could
// make a slot look free while a slower wave still reads it (measured: the loader then
// overwrote live ring bytes in stages of 8+ items).
enum Ctl : int { C_CBAR = 0, C_ABORT = 1, C_FILLED0 = 8, C_FREED0 = 16, C_NWORDS = 32 };
constexpr int kCtlBytes = C_NWORDS * 4;

__device__ __forceinline__ void gst(u64* p, unsigned tag, unsigned v) {
  __hip_atomic_store((gu64*)p, ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 gld(const u64* p) {
  return __hip_atomic_load((gu64*)const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int lds_ld(int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(int* p, int v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool global_abort(const int* err) {
  return __hip_atomic_load((gi32*)const_cast<int*>(err + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void raise_abort(int* err, int* ctl, int code) {
  __hip_atomic_store((gi32*)err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gi32*)(err + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lds_st(ctl + C_ABORT, 1);
}

// one 1-KiB LDS-DMA transfer: lane l's 16 B land at lds_dst + 16 l (non-temporal:
// every weight byte is read once per token by one CU)
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void vm_wait_dyn(int n) {
#define LFK_VW(k) case k: vm_wait<k>(); break;
  switch (n) {
    LFK_VW(0) LFK_VW(1) LFK_VW(2) LFK_VW(3) LFK_VW(4) LFK_VW(5) LFK_VW(6) LFK_VW(7)
    LFK_VW(8) LFK_VW(9) LFK_VW(10) LFK_VW(11) LFK_VW(12) LFK_VW(13) LFK_VW(14) LFK_VW(15)
    LFK_VW(16) LFK_VW(17) LFK_VW(18) LFK_VW(19) LFK_VW(20) LFK_VW(21) LFK_VW(22) LFK_VW(23)
    LFK_VW(24) LFK_VW(25) LFK_VW(26) LFK_VW(27) LFK_VW(28) LFK_VW(29) LFK_VW(30) LFK_VW(31)
    LFK_VW(32) LFK_VW(33) LFK_VW(34) LFK_VW(35) LFK_VW(36) LFK_VW(37) LFK_VW(38) LFK_VW(39)
    LFK_VW(40) LFK_VW(41) LFK_VW(42) LFK_VW(43) LFK_VW(44) LFK_VW(45) LFK_VW(46) LFK_VW(47)
    default: vm_wait<0>(); break;
  }
#undef LFK_VW
}

// ------------------------------------------------------------------ ring row dots
struct X8 {
  int lo[4], hi[4];
  float s[4];     // x scales of the 8-blocks: lo first / second half, hi first / second half
  float slo, shi; // scaled sums of the 16 lo / hi values (for the min / -32 terms)
};

__device__ __forceinline__ void load_x8(X8& X, lds_i8* xq, lds_cf* xs, int off_lo, int off_hi) {
  const int4 a = lds_i4(xq + off_lo);
  const int4 b = lds_i4(xq + off_hi);
  X.lo[0] = a.x; X.lo[1] = a.y; X.lo[2] = a.z; X.lo[3] = a.w;
  X.hi[0] = b.x; X.hi[1] = b.y; X.hi[2] = b.z; X.hi[3] = b.w;
  const float2 sa = lds_f2(xs + (off_lo >> 3));
  const float2 sb = lds_f2(xs + (off_hi >> 3));
  X.s[0] = sa.x; X.s[1] = sa.y; X.s[2] = sb.x; X.s[3] = sb.y;
  const int ones = 0x01010101;
  X.slo = sa.x * (float)dot4(a.x, ones, dot4(a.y, ones, 0)) + sa.y * (float)dot4(a.z, ones, dot4(a.w, ones, 0));
  X.shi = sb.x * (float)dot4(b.x, ones, dot4(b.y, ones, 0)) + sb.y * (float)dot4(b.z, ones, dot4(b.w, ones, 0));
}

__device__ __forceinline__ int pad16(int b) { return (b + 15) & ~15; }
__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// x offsets of chunk c (the one chunk order of the ring row format)
__device__ __forceinline__ void chunk_x_offsets(int c, int& off_lo, int& off_hi) {
  const int sb = c >> 3, j = c & 7;
  off_lo = sb * 256 + 64 * (j >> 1) + 16 * (j & 1);
  off_hi = off_lo + 32;
}

// Ring row chunk c split into its LDS loads (rload) and its integer math (rdot), so a
// wave can issue the loads of several units before the first dot (ILP: one unit at a time
// left each wave latency-bound on LDS round trips and DPP chains).
template <int T> struct RRaw;
template <> struct RRaw<T_Q4_K> { int4 q, m; };
template <> struct RRaw<T_Q5_K> { int4 q, m, qh; };
template <> struct RRaw<T_Q6_K> { int4 ql; uint2 qh; int sc_lo, sc_hi; unsigned d; };
template <> struct RRaw<T_Q8_0> { int4 qa, qb; unsigned d_lo, d_hi; };

template <int T>
__device__ __forceinline__ void rload(RRaw<T>& R, lds_u8* row, int nsb, int c) {
  const int sb = c >> 3, j = c & 7;
  if constexpr (T == T_Q4_K) {
    R.m = lds_i4(row + 16 * sb);
    R.q = lds_i4(row + nsb * 16 + 16 * c);
  } else if constexpr (T == T_Q5_K) {
    R.m = lds_i4(row + 16 * sb);
    R.qh = lds_i4(row + nsb * 16 + 32 * sb + 16 * (j & 1));
    R.q = lds_i4(row + nsb * 48 + 16 * c);
  } else if constexpr (T == T_Q6_K) {
    const int off_d = nsb * 16, off_qh = off_d + pad16(2 * nsb), off_ql = off_qh + 64 * nsb;
    R.ql = lds_i4(row + off_ql + 16 * c);
    const f32x2_t qh = *reinterpret_cast<LDS_AS const f32x2_t*>(row + off_qh + 8 * c);
    R.qh = make_uint2(__float_as_uint(qh.x), __float_as_uint(qh.y));
    const int si = 16 * sb + 4 * (j >> 1) + (j & 1);
    R.sc_lo = (int)*reinterpret_cast<LDS_AS const signed char*>(row + si);
    R.sc_hi = (int)*reinterpret_cast<LDS_AS const signed char*>(row + si + 2);
    R.d = *reinterpret_cast<LDS_AS const unsigned short*>(row + off_d + 2 * sb);
  } else {  // Q8_0: nsb is the number of 32-blocks
    const int off_qs = pad16(2 * nsb);
    R.qa = lds_i4(row + off_qs + 32 * c);
    R.qb = lds_i4(row + off_qs + 32 * c + 16);
    const int bl = 8 * sb + 2 * (j >> 1);
    R.d_lo = *reinterpret_cast<LDS_AS const unsigned short*>(row + 2 * bl);
    R.d_hi = *reinterpret_cast<LDS_AS const unsigned short*>(row + 2 * bl + 2);
  }
}

template <int T>
__device__ __forceinline__ float rdot(const RRaw<T>& R, int c, const X8& X) {
  const int j = c & 7;
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int g = j >> 1;
    const unsigned dd = (unsigned)R.m.x;
    const float d = h2f(dd & 0xFFFF), dmin = h2f(dd >> 16);
    float sc_lo, m_lo, sc_hi, m_hi;
    scale_min_pair(g, (unsigned)R.m.y, (unsigned)R.m.z, (unsigned)R.m.w, sc_lo, m_lo, sc_hi, m_hi);
    const int qv[4] = {R.q.x, R.q.y, R.q.z, R.q.w};
    int lo[4], hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = qv[i] & 0x0F0F0F0F;
      hi[i] = (qv[i] >> 4) & 0x0F0F0F0F;
      if constexpr (T == T_Q5_K) {
        const int hv = (i == 0 ? R.qh.x : i == 1 ? R.qh.y : i == 2 ? R.qh.z : R.qh.w);
        lo[i] |= ((hv >> (2 * g)) & 0x01010101) << 4;
        hi[i] |= ((hv >> (2 * g + 1)) & 0x01010101) << 4;
      }
    }
    const int dla = dot4(lo[1], X.lo[1], dot4(lo[0], X.lo[0], 0));
    const int dlb = dot4(lo[3], X.lo[3], dot4(lo[2], X.lo[2], 0));
    const int dha = dot4(hi[1], X.hi[1], dot4(hi[0], X.hi[0], 0));
    const int dhb = dot4(hi[3], X.hi[3], dot4(hi[2], X.hi[2], 0));
    return d * (sc_lo * (X.s[0] * (float)dla + X.s[1] * (float)dlb) + sc_hi * (X.s[2] * (float)dha + X.s[3] * (float)dhb)) -
           dmin * (m_lo * X.slo + m_hi * X.shi);
  } else if constexpr (T == T_Q6_K) {
    const int lv[4] = {R.ql.x, R.ql.y, R.ql.z, R.ql.w};
    int lo[4], hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (lv[i] & 0x0F0F0F0F) | (((int)(R.qh.x >> (2 * i)) & 0x03030303) << 4);
      hi[i] = ((lv[i] >> 4) & 0x0F0F0F0F) | (((int)(R.qh.y >> (2 * i)) & 0x03030303) << 4);
    }
    const int dla = dot4(lo[1], X.lo[1], dot4(lo[0], X.lo[0], 0));
    const int dlb = dot4(lo[3], X.lo[3], dot4(lo[2], X.lo[2], 0));
    const int dha = dot4(hi[1], X.hi[1], dot4(hi[0], X.hi[0], 0));
    const int dhb = dot4(hi[3], X.hi[3], dot4(hi[2], X.hi[2], 0));
    const float d = h2f(R.d & 0xFFFF);
    return d * ((float)R.sc_lo * (X.s[0] * (float)dla + X.s[1] * (float)dlb - 32.f * X.slo) +
                (float)R.sc_hi * (X.s[2] * (float)dha + X.s[3] * (float)dhb - 32.f * X.shi));
  } else {
    const int a0 = dot4(R.qa.y, X.lo[1], dot4(R.qa.x, X.lo[0], 0));
    const int a1 = dot4(R.qa.w, X.lo[3], dot4(R.qa.z, X.lo[2], 0));
    const int b0 = dot4(R.qb.y, X.hi[1], dot4(R.qb.x, X.hi[0], 0));
    const int b1 = dot4(R.qb.w, X.hi[3], dot4(R.qb.z, X.hi[2], 0));
    return h2f(R.d_lo & 0xFFFF) * (X.s[0] * (float)a0 + X.s[1] * (float)a1) +
           h2f(R.d_hi & 0xFFFF) * (X.s[2] * (float)b0 + X.s[3] * (float)b1);
  }
}

// Stage mapping of the consumer waves: the activation is cut into blocks of 64 chunks (one
// chunk per lane); wpb waves share a block (each a residue class of the item rows) and the
// ngroup = kNCW / wpb block groups cover all blocks (group gi: blocks gi and gi + ngroup).
// A wave loads the activation chunks of its (at most two) blocks into registers once per
// stage; per item it runs its rows x blocks with every LDS load issued before the first
// dot, sums its blocks per row and reduces each row once. part[row * ngroup + gi] is
// summed in a fixed order by the stage epilogue (deterministic).
struct StageMap {
  int nch, nblk, wpb, ngroup, gi, rc, nsb4;  // nsb4: K / 256
  bool active, v0, v1;                       // v0/v1: this lane's chunk of block 0/1 exists
  int c0, c1;                                // this lane's chunk in block 0/1 (clamped)
};

__device__ __forceinline__ StageMap stage_map(int K, int cw, int lane) {
  StageMap m;
  m.nch = K >> 5;
  m.nblk = (m.nch + 63) >> 6;
  m.nsb4 = K >> 8;
  m.wpb = max(1, kNCW / m.nblk);
  m.ngroup = kNCW / m.wpb;
  m.gi = cw / m.wpb;
  m.rc = cw - m.gi * m.wpb;
  m.active = m.gi < m.ngroup;
  const int b0 = m.gi, b1 = m.gi + m.ngroup;
  const int c0 = b0 * 64 + lane, c1 = b1 * 64 + lane;
  m.v0 = m.active && c0 < m.nch;
  m.v1 = m.active && b1 < m.nblk && c1 < m.nch;
  m.c0 = min(c0, m.nch - 1);
  m.c1 = min(c1, m.nch - 1);
  return m;
}

template <int T>
__device__ __forceinline__ void item_rows(lds_u8* slot, const PdItem& it, const StageMap& m, const X8 (&xb)[2],
                                          lds_f* part, int lane) {
  const int nsb = (T == T_Q8_0) ? m.nch : m.nsb4;
  const int rows = it.rows;
  for (int j0 = m.rc; j0 < rows; j0 += 2 * m.wpb) {
    const int j1 = j0 + m.wpb;
    const bool has1 = j1 < rows;
    lds_u8* r0 = slot + (size_t)j0 * it.row_bytes;
    lds_u8* r1 = slot + (size_t)min(j1, rows - 1) * it.row_bytes;
    RRaw<T> R00, R01, R10, R11;
    rload<T>(R00, r0, nsb, m.c0);
    rload<T>(R01, r0, nsb, m.c1);
    rload<T>(R10, r1, nsb, m.c0);
    rload<T>(R11, r1, nsb, m.c1);
    float v0 = m.v0 ? rdot<T>(R00, m.c0, xb[0]) : 0.f;
    float v1 = m.v0 ? rdot<T>(R10, m.c0, xb[0]) : 0.f;
    v0 += m.v1 ? rdot<T>(R01, m.c1, xb[1]) : 0.f;
    v1 += m.v1 ? rdot<T>(R11, m.c1, xb[1]) : 0.f;
    v0 = row_sum16(v0);
    v1 = row_sum16(v1);
    const float t0 = (readlane_f(v0, 0) + readlane_f(v0, 16)) + (readlane_f(v0, 32) + readlane_f(v0, 48));
    const float t1 = (readlane_f(v1, 0) + readlane_f(v1, 16)) + (readlane_f(v1, 32) + readlane_f(v1, 48));
    if (lane == 0) {
      part[(it.row0 + j0) * m.ngroup + m.gi] = t0;
      if (has1) part[(it.row0 + j1) * m.ngroup + m.gi] = t1;
    }
  }
}

// ------------------------------------------------------------------ LDS carve
struct Lds {
  int* ctl;
  float* xres;   // [64] this CU's residual rows
  float* part;   // [part_floats]
  int8_t* xq;    // activation (union with the attention scratch)
  float* xs;
  float* ssq;
  char* act;
  uint8_t* ring;
  unsigned ring_lds;  // LDS byte address of the ring
};

__device__ __forceinline__ Lds carve(char* smem, CA& a) {
  Lds L;
  L.ctl = reinterpret_cast<int*>(smem);
  L.xres = reinterpret_cast<float*>(smem + kCtlBytes);
  L.part = reinterpret_cast<float*>(smem + kCtlBytes + 256);
  char* p = smem + kCtlBytes + 256 + ((a.part_floats * 4 + 15) & ~15);
  L.act = p;
  const int actn = (max(max(a.d, a.nq), a.F) + 63) & ~63;
  L.xq = reinterpret_cast<int8_t*>(p);
  L.xs = reinterpret_cast<float*>(p + actn);
  L.ssq = reinterpret_cast<float*>(p + actn + actn / 2);
  L.ring = reinterpret_cast<uint8_t*>(p + a.act_bytes);
  L.ring_lds = (unsigned)(uintptr_t)(L.ring);
  return L;
}

// ------------------------------------------------------------------ loader waves
// kLoaders waves split the items (item n -> wave n % kLoaders). Each keeps up to kInflight
// of its items of LDS-DMA in flight (items <= 15 KiB: at most 4 x 15 = 60 one-KiB
// transfers, vmcnt is a 6-bit counter) and publishes an item (its slot's C_FILLED word)
// once vmcnt shows that only the transfers of its newer items remain. One wave could keep
// ~45 KiB in flight, which at ~2.4 us issue-to-land under a chip-wide stream is ~17 GB/s
// per CU (measured); two double that budget.
constexpr int kInflight = 3;

__device__ void loader(CA& a, const Lds& S, int u, int lw) {
  const int lane = threadIdx.x & 63;
  int* ctl = S.ctl;
  int qn[kInflight + 1], qkb[kInflight + 1];  // FIFO of this wave's in-flight items (oldest first)
  int qc = 0;
  auto publish = [&](int item) {
    if (lane == 0) lds_st(ctl + C_FILLED0 + item % a.nslot, item + 1);
  };
  auto publish_oldest = [&](int newer_kb) {
    vm_wait_dyn(newer_kb);
    publish(qn[0]);
#pragma unroll
    for (int i = 0; i < kInflight; ++i) { qn[i] = qn[i + 1]; qkb[i] = qkb[i + 1]; }
    --qc;
  };
  auto drain = [&]() {
    vm_wait<0>();
#pragma unroll
    for (int i = 0; i <= kInflight; ++i)
      if (i < qc) publish(qn[i]);
    qc = 0;
  };
  long long lac[3] = {0, 0, 0};  // blocked on slots, waiting for landings, issuing
  int n = 0;
  for (int l = 0; l < a.n_layer; ++l) {
    const PdLayer Ly = layer_at(a, l);
    const uint8_t* span = Ly.wbase + (size_t)u * Ly.cu_bytes;
    long long* tl = a.tl ? a.tl + ((size_t)u * a.n_layer + l) * kPdStamps : nullptr;
    long long* ti = (a.tli && l == 2) ? a.tli + (size_t)u * kPdItemStamps * 8 : nullptr;
    for (int k = 0; k < Ly.nitems; ++k, ++n) {
      if (n % kLoaders != lw) continue;
      const long long c0 = clk();
      if (tl && lane == 0 && (k == 0 || k == Ly.nitems - 1)) tl[k == 0 ? 10 : 11] = wall_clock64();
      const PdItem it = item_at(a, Ly.item0 + k);
      const int slot = n % a.nslot;
      if (n >= a.nslot) {
        // every consumer wave has released every earlier item of this slot
        int* freed = ctl + C_FREED0 + slot;
        const int need = (n / a.nslot) * kNCW;
        if (lds_ld(freed) < need) {
          drain();  // about to block on the consumers: land and publish what is in flight first
          const long long t0 = wall_clock64();
          while (lds_ld(freed) < need) {
            if (lds_ld(ctl + C_ABORT)) return;
            if (wall_clock64() - t0 > 4 * kSpinTicks) {  // consumers gone without a word: give up
              if (lane == 0) raise_abort(a.err, ctl, 91);
              return;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
      }
      if (ti && lane == 0 && k < kPdItemStamps) ti[k * 8 + 0] = wall_clock64();
      const long long c1 = clk();
      lac[0] += c1 - c0;
      const uint8_t* src = span + it.off + lane * 16;
      const unsigned dst = __builtin_amdgcn_readfirstlane(S.ring_lds + (unsigned)(slot * a.slot_bytes));
      if (!(a.dbg_mode & 2))
        for (int kb = 0; kb < it.dma_kb; ++kb) glds16(src + kb * 1024, dst + kb * 1024);
#pragma unroll
      for (int i = 0; i <= kInflight; ++i) {  // constant indices only: the FIFO stays in registers
        if (i == qc) { qn[i] = n; qkb[i] = it.dma_kb; }
      }
      ++qc;
      const long long c2 = clk();
      lac[2] += c2 - c1;
      if (qc > kInflight) {
        int newer = 0;
#pragma unroll
        for (int i = 1; i <= kInflight; ++i) newer += qkb[i];
        publish_oldest(newer);
      }
      lac[1] += clk() - c2;
    }
  }
  drain();
  if (a.acct && lw == 0 && lane == 0)
    for (int i = 0; i < 3; ++i) a.acct[(size_t)u * 16 + 8 + i] = lac[i];
}

// ------------------------------------------------------------------ consumer helpers
struct Cons {
  CA& a;
  const Lds& S;
  int u, cw, lane;
  unsigned ep;
  int phase;     // csync generation
  int n;         // next ring item
  bool ok;

  __device__ Cons(CA& a_, const Lds& S_, int u_, int cw_, unsigned ep_)
      : a(a_), S(S_), u(u_), cw(cw_), lane(threadIdx.x & 63), ep(ep_), phase(0), n(0), ok(true) {}

  __device__ bool aborted() { return lds_ld(S.ctl + C_ABORT) != 0; }
  // another CU gave up: stop this CU too (the loader watches the LDS word)
  __device__ bool bail() {
    lds_st(S.ctl + C_ABORT, 1);
    ok = false;
    return false;
  }

  // LDS counter barrier of the consumer waves
  __device__ bool csync() {
    const long long c0 = clk();
    const bool r = csync_();
    ac[2] += clk() - c0;
    return r;
  }
  __device__ bool csync_() {
    phase += kNCW;
    if (lane == 0) lds_add(S.ctl + C_CBAR, 1);
    long long t0 = 0;
    for (int spins = 0; lds_ld(S.ctl + C_CBAR) < phase; ++spins) {
      if (lds_ld(S.ctl + C_ABORT)) { ok = false; return false; }
      if ((spins & 63) == 63) {
        const long long t = wall_clock64();
        if (t0 == 0) t0 = t;
        else if (t - t0 > kSpinTicks) return fail(80);
      }
      __builtin_amdgcn_s_sleep(0);
    }
    return true;
  }

  __device__ bool fail(int code) {
    if (lane == 0) raise_abort(a.err, S.ctl, code);
    ok = false;
    return false;
  }

  // sweep granules [g0, g1) of gb (this wave's share), calling fn(i, value) for each
  template <class Fn>
  __device__ bool sweep(const u64* gb, int g0, int g1, int code, Fn fn) {
    const long long c0 = clk();
    const bool r = sweep_(gb, g0, g1, code, fn);
    ac[3] += clk() - c0;
    return r;
  }
  template <class Fn>
  __device__ bool sweep_(const u64* gb, int g0, int g1, int code, Fn fn) {
    constexpr int U = 8;
    for (int base = g0; base < g1; base += 64 * U) {
      u64 v[U];
      long long t0 = 0;
      for (int spins = 0;; ++spins) {
        bool good = true;
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const int i = base + k * 64 + lane;
          v[k] = gld(gb + min(i, g1 - 1));
          good &= (i >= g1) || ((unsigned)(v[k] >> 32) == ep);
        }
        if (__all(good)) break;
        const long long t = wall_clock64();
        if (t0 == 0) t0 = t;
        if (t - t0 > kSpinTicks) return fail(code);
        if ((spins & 15) == 15 && (aborted() || global_abort(a.err))) return bail();
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int i = base + k * 64 + lane;
        if (i < g1) fn(i, (unsigned)v[k]);
      }
    }
    return true;
  }

  // all consumer waves split [0, total) of one hop buffer, then meet at csync
  template <class Fn>
  __device__ bool gather(const u64* gb, int total, int code, Fn fn) {
    const int per = (((total + kNCW - 1) / kNCW) + 63) & ~63;
    const int g0 = min(total, cw * per), g1 = min(total, g0 + per);
    if (g0 < g1 && !sweep(gb, g0, g1, code, fn)) return false;
    return csync();
  }

  // decode of a q8 record [n/4 int8x4][n/8 f32 scales](+[1 ssq]) into the activation at `base`
  __device__ void q8_store(int base, int n4, int n8, int k, unsigned v) {
    if (k < n4) {
      *reinterpret_cast<unsigned*>(S.xq + base + 4 * k) = v;
    } else if (k < n4 + n8) {
      S.xs[(base >> 3) + (k - n4)] = __uint_as_float(v);
    }
  }

  long long* ti = nullptr;  // per-item stamps of one layer (cw 0, lane 0)
  int ti_k = 0;
  long long ac[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // cycle accounting (see PDecodeArgs::acct)
  StageMap sm;   // this wave's blocks / row class in the current stage
  X8 xb[2];      // activation chunks of those blocks (registers, whole stage)

  // stage with K inputs begins: map this wave and load its activation chunks once
  __device__ void begin_stage(int K) {
    sm = stage_map(K, cw, lane);
    int lo, hi;
    chunk_x_offsets(sm.c0, lo, hi);
    load_x8(xb[0], (lds_i8*)S.xq, (lds_cf*)S.xs, lo, hi);
    chunk_x_offsets(sm.c1, lo, hi);
    load_x8(xb[1], (lds_i8*)S.xq, (lds_cf*)S.xs, lo, hi);
  }

  // wait for ring item n, run this wave's rows of it, release it
  __device__ bool consume_item(const PdItem& it) {
    const int need = n + 1;
    int* filled = S.ctl + C_FILLED0 + n % a.nslot;
    if (ti && ti_k < kPdItemStamps) ti[ti_k * 8 + 2] = wall_clock64();
    const long long c0 = clk();
    if (lds_ld(filled) < need) {
      long long t0 = wall_clock64();
      while (lds_ld(filled) < need) {
        if (lds_ld(S.ctl + C_ABORT)) { ok = false; return false; }
        if (wall_clock64() - t0 > kSpinTicks) return fail(90);
        __builtin_amdgcn_s_sleep(0);
      }
    }
    if (ti && ti_k < kPdItemStamps) ti[ti_k * 8 + 3] = wall_clock64();
    lds_u8* slot = (lds_u8*)(S.ring + (size_t)(n % a.nslot) * a.slot_bytes);
    const long long c1 = clk();
    if (sm.active && !(a.dbg_mode & 1)) {
      lds_f* part = (lds_f*)S.part;
      switch (it.type) {
        case T_Q4_K: item_rows<T_Q4_K>(slot, it, sm, xb, part, lane); break;
        case T_Q5_K: item_rows<T_Q5_K>(slot, it, sm, xb, part, lane); break;
        case T_Q6_K: item_rows<T_Q6_K>(slot, it, sm, xb, part, lane); break;
        default: item_rows<T_Q8_0>(slot, it, sm, xb, part, lane); break;
      }
    }
    const long long c2 = clk();
    ac[1] += c1 - c0;
    ac[0] += c2 - c1;
    ac[4] += 1;
    // every LDS read of the slot has returned before the release (the add is a release)
    if (lane == 0) lds_add(S.ctl + C_FREED0 + n % a.nslot, 1);
    if (ti && ti_k < kPdItemStamps) ti[ti_k * 8 + 4] = wall_clock64();
    ++ti_k;
    ++n;
    return true;
  }

  // stage total of per-CU row j (its block groups summed in a fixed order)
  __device__ float row_total(int j, int K) const {
    const StageMap m = stage_map(K, 0, 0);
    float s = 0.f;
    for (int g = 0; g < m.ngroup; ++g) s += S.part[j * m.ngroup + g];
    return s;
  }

  // publish n (multiple of 8, <= 64 per call) values v (lane j holds value j) as a q8 record:
  // [n/4 int8x4][n/8 scales](+ssq); lanes >= n hold anything
  __device__ void publish_q8(u64* rec, float v, int n, int j0_rec4, int j0_rec8, int rec8_base) {
    const float amax = max8(fabsf(v));
    const float sc = amax * (1.f / 127.f);
    const float inv = sc > 0.f ? 1.f / sc : 0.f;
    const int q = __float2int_rn(v * inv) & 0xFF;
    // pack 4 lanes -> lane 4i
    const int q1 = __shfl_down(q, 1), q2 = __shfl_down(q, 2), q3 = __shfl_down(q, 3);
    if (lane < n && (lane & 3) == 0) gst(rec + j0_rec4 + (lane >> 2), ep, (unsigned)(q | (q1 << 8) | (q2 << 16) | (q3 << 24)));
    if (lane < n && (lane & 7) == 0) gst(rec + rec8_base + j0_rec8 + (lane >> 3), ep, __float_as_uint(sc));
  }
};

// HX record of CU u: the CU's NXU residual rows times the norm weight, q8 per 8, + sum of squares
__device__ void publish_hx(Cons& C, u64* hx, const float* norm_w) {
  CA& a = C.a;
  const int nx = a.nxu;
  const int rec = nx / 4 + nx / 8 + 1;
  u64* r = hx + (size_t)C.u * rec;
  float ss = 0.f;
  for (int j0 = 0; j0 < nx; j0 += 64) {
    const int j = j0 + C.lane;
    const float v = j < nx ? C.S.xres[j] : 0.f;
    ss += v * v;
    const float t = j < nx ? v * norm_w[C.u * nx + j] : 0.f;
    C.publish_q8(r, t, min(64, nx - j0), j0 / 4, j0 / 8, nx / 4);
  }
  ss = wave_sum_fast(ss);
  if (C.lane == 0) gst(r + nx / 4 + nx / 8, C.ep, __float_as_uint(ss));
}

// gather an HX hop into the activation; rms into ctl[C_RMS]
__device__ bool gather_hx(Cons& C, const u64* hx) {
  CA& a = C.a;
  const int nx = a.nxu, n4 = nx / 4, n8 = nx / 8, rec = n4 + n8 + 1;
  if (!C.gather(hx, a.ncu * rec, 10, [&](int i, unsigned v) {
        const int uu = i / rec, k = i - uu * rec;
        if (k == n4 + n8) C.S.ssq[uu] = __uint_as_float(v);
        else C.q8_store(uu * nx, n4, n8, k, v);
      }))
    return false;
  return true;
}

__device__ float hx_rms(Cons& C) {
  // fixed-order sum of the per-CU partial sums of squares (identical on every wave)
  float s = 0.f;
  for (int i = C.lane; i < C.a.ncu; i += 64) s += C.S.ssq[i];
  s = wave_sum_fast(s);
  return rsqrtf(s / (float)C.a.d + C.a.eps);
}

// ------------------------------------------------------------------ attention
struct AttLds {
  h2v* q;      // [G * hd / 2] (q * scale, f16 pairs)
  h2v* knew;   // [hd / 2]
  h2v* vnew;
  __half* vs;  // [kAttW][16][hd + 8]
  float* ps;   // [kAttW][G][16]
  float* wm;   // [kAttW][G]
  float* wl;
  float* wo;   // [kAttW][G][hd]
};

__device__ AttLds att_carve(const Lds& S, int G, int hd) {
  AttLds A;
  char* p = S.act;
  A.q = reinterpret_cast<h2v*>(p); p += G * hd * 2;
  A.knew = reinterpret_cast<h2v*>(p); p += hd * 2;
  A.vnew = reinterpret_cast<h2v*>(p); p += hd * 2;
  A.vs = reinterpret_cast<__half*>(p); p += kAttW * 16 * (hd + 8) * 2;
  A.ps = reinterpret_cast<float*>(p); p += kAttW * G * 16 * 4;
  A.wm = reinterpret_cast<float*>(p); p += kAttW * G * 4;
  A.wl = reinterpret_cast<float*>(p); p += kAttW * G * 4;
  A.wo = reinterpret_cast<float*>(p);
  return A;
}

template <int G>
__device__ bool attention_split(Cons& C, int l, int g, int s, int S_, int KPS, int L) {
  constexpr int HD = 128, DPL = HD / 4, NLD = DPL / 8;
  CA& a = C.a;
  const Lds& S = C.S;
  AttLds A = att_carve(S, G, HD);
  u64* gl = a.gran + (size_t)l * a.gran_layer;
  // q / k_new / v_new of the group: records of CUs [g*cpg, (g+1)*cpg)
  const int nq2 = a.nqu / 2, nk2 = a.nku / 2, rec = nq2 + 2 * nk2;
  const u64* src = gl + a.off_qkv + (size_t)g * a.cpg * rec;
  if (!C.gather(src, a.cpg * rec, 20, [&](int i, unsigned v) {
        const int ci = i / rec, k = i - ci * rec;
        const h2v hv = __builtin_bit_cast(h2v, v);
        if (k < nq2) A.q[ci * nq2 + k] = hv;
        else if (k < nq2 + nk2) A.knew[ci * nk2 + (k - nq2)] = hv;
        else A.vnew[ci * nk2 + (k - nq2 - nk2)] = hv;
      }))
    return false;
  const int k0 = s * KPS, k1 = min(L, k0 + KPS);
  const int cw = C.cw, lane = C.lane, kw = lane >> 2, sub = lane & 3;
  const __half* kc = a.k_cache + (size_t)l * a.kv_layer + (size_t)g * a.n_ctx * HD;
  const __half* vc = a.v_cache + (size_t)l * a.kv_layer + (size_t)g * a.n_ctx * HD;
  if (cw < kAttW) {
    float m[G], lsum[G], o[G][2];
#pragma unroll
    for (int h = 0; h < G; ++h) { m[h] = -FLT_MAX; lsum[h] = 0.f; o[h][0] = 0.f; o[h][1] = 0.f; }
    __half* vs = A.vs + (size_t)cw * 16 * (HD + 8);
    float* ps = A.ps + cw * G * 16;
    for (int kb = k0 + cw * 16; kb < k1; kb += 16 * kAttW) {
      const int key = kb + kw;
      const bool valid = key < k1;
      const bool is_new = key == L - 1;
      const size_t row = (size_t)min(key, a.n_ctx - 1) * HD + sub * DPL;
      uint4 kr[NLD], vr[NLD];
#pragma unroll
      for (int i = 0; i < NLD; ++i) {
        kr[i] = *reinterpret_cast<const uint4*>(kc + row + 8 * i);
        vr[i] = *reinterpret_cast<const uint4*>(vc + row + 8 * i);
      }
#pragma unroll
      for (int i = 0; i < NLD; ++i) {  // the new key comes from the gathered granules (branch-free select)
        const uint4 kn = *reinterpret_cast<const uint4*>(A.knew + (sub * DPL + 8 * i) / 2);
        const uint4 vn = *reinterpret_cast<const uint4*>(A.vnew + (sub * DPL + 8 * i) / 2);
        kr[i] = is_new ? kn : kr[i];
        vr[i] = is_new ? vn : vr[i];
      }
#pragma unroll
      for (int i = 0; i < NLD; ++i) *reinterpret_cast<uint4*>(vs + kw * (HD + 8) + sub * DPL + 8 * i) = vr[i];
      float sc[G];
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const uint4* q4 = reinterpret_cast<const uint4*>(A.q + h * (HD / 2) + sub * (DPL / 2));
        float p0 = 0.f, p1 = 0.f;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
          const uint4 qq = q4[i];
          p0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.x), __builtin_bit_cast(h2v, kr[i].x), p0, false);
          p1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.y), __builtin_bit_cast(h2v, kr[i].y), p1, false);
          p0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.z), __builtin_bit_cast(h2v, kr[i].z), p0, false);
          p1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, qq.w), __builtin_bit_cast(h2v, kr[i].w), p1, false);
        }
        float t = p0 + p1;
        t += dpp_f<0xB1>(t);
        t += dpp_f<0x4E>(t);  // quad sum: every lane of the key's quad holds the score
        sc[h] = t;
      }
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float sv = valid ? sc[h] : -FLT_MAX;
        const float mb = wave_max_fast(sv);
        const float mn = fmaxf(m[h], mb);
        const float f = __expf(m[h] - mn);
        const float e = valid ? __expf(sv - mn) : 0.f;
        // each key appears in 4 lanes (its quad): sum the quad leaders only
        lsum[h] = lsum[h] * f + wave_sum_fast(sub == 0 ? e : 0.f);
        o[h][0] *= f;
        o[h][1] *= f;
        m[h] = mn;
        if (sub == 0) ps[h * 16 + kw] = e;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const __half2 hv = *reinterpret_cast<const __half2*>(vs + k * (HD + 8) + 2 * lane);
        const float v0 = __low2float(hv), v1 = __high2float(hv);
#pragma unroll
        for (int h = 0; h < G; ++h) {
          const float p = ps[h * 16 + k];
          o[h][0] += p * v0;
          o[h][1] += p * v1;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
      A.wo[(cw * G + h) * HD + 2 * lane] = o[h][0];
      A.wo[(cw * G + h) * HD + 2 * lane + 1] = o[h][1];
      if (lane == 0) { A.wm[cw * G + h] = m[h]; A.wl[cw * G + h] = lsum[h]; }
    }
  }
  if (!C.csync()) return false;
  // combine the attention waves -> this split's partial (unnormalised o, m, l) per head
  u64* rec_out = gl + a.off_att + ((size_t)g * a.smax + s) * G * (HD + 2);
  for (int e = cw * 64 + lane; e < G * (HD + 2); e += kNCW * 64) {
    const int h = e / (HD + 2), dd = e - h * (HD + 2);
    float M = -FLT_MAX;
#pragma unroll
    for (int w = 0; w < kAttW; ++w) M = fmaxf(M, A.wm[w * G + h]);
    float val;
    if (dd == HD) {
      val = M;
    } else {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < kAttW; ++w) {
        const float f = A.wm[w * G + h] == -FLT_MAX ? 0.f : __expf(A.wm[w * G + h] - M);
        acc += f * (dd == HD + 1 ? A.wl[w * G + h] : A.wo[(w * G + h) * HD + dd]);
      }
      val = acc;
    }
    gst(rec_out + e, C.ep, __float_as_uint(val));
  }
  (void)S_;
  return true;
}

// merge of query head h = g*G + j over the S_ splits -> q8 record of o_h (48 granules for hd 128)
template <int G>
__device__ bool merge_head(Cons& C, int l, int g, int j, int S_) {
  constexpr int HD = 128;
  CA& a = C.a;
  u64* gl = a.gran + (size_t)l * a.gran_layer;
  if (C.cw >= 2) return true;  // 128 lanes = the head's dims
  const int dd = C.cw * 64 + C.lane;
  const u64* base = gl + a.off_att + (size_t)g * a.smax * G * (HD + 2) + j * (HD + 2);
  float M = -FLT_MAX, num = 0.f, den = 0.f;
  constexpr int B = 8;
  for (int s0 = 0; s0 < S_; s0 += B) {
    u64 vo[B], vm[B], vl[B];
    long long t0 = 0;
    for (int spins = 0;; ++spins) {
      bool good = true;
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const int s = min(s0 + i, S_ - 1);
        const u64* r = base + (size_t)s * G * (HD + 2);
        vo[i] = gld(r + dd);
        vm[i] = gld(r + HD);
        vl[i] = gld(r + HD + 1);
        good &= ((unsigned)(vo[i] >> 32) == C.ep) && ((unsigned)(vm[i] >> 32) == C.ep) &&
                ((unsigned)(vl[i] >> 32) == C.ep);
      }
      if (__all(good)) break;
      const long long t = wall_clock64();
      if (t0 == 0) t0 = t;
      if (t - t0 > kSpinTicks) return C.fail(30);
      if ((spins & 15) == 15 && (C.aborted() || global_abort(a.err))) return C.bail();
      __builtin_amdgcn_s_sleep(1);
    }
    float mb = M;
#pragma unroll
    for (int i = 0; i < B; ++i) if (s0 + i < S_) mb = fmaxf(mb, __uint_as_float((unsigned)vm[i]));
    const float r = __expf(M - mb);
    num *= r;
    den *= r;
#pragma unroll
    for (int i = 0; i < B; ++i) {
      if (s0 + i < S_) {
        const float f = __expf(__uint_as_float((unsigned)vm[i]) - mb);
        num += f * __uint_as_float((unsigned)vo[i]);
        den += f * __uint_as_float((unsigned)vl[i]);
      }
    }
    M = mb;
  }
  const float ov = num / den;
  const int h = g * G + j;
  if (a.dbg) a.dbg[(size_t)l * dump_stride(a) + a.nq + 2 * a.nkv + h * HD + dd] = ov;
  u64* rec = gl + a.off_o + (size_t)h * (HD / 4 + HD / 8);
  // lane group of wave cw covers dims [64cw, 64cw + 64): int8x4 records 16cw.., scales 8cw..
  C.publish_q8(rec, ov, 64, C.cw * 16, C.cw * 8, HD / 4);
  return true;
}

// ------------------------------------------------------------------ the kernel
template <int G>
__global__ __launch_bounds__(kThreads) void pdecode_kernel(const PDecodeArgs* ap) {
  CA& a = *(CA*)(ap);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds S = carve(smem, a);
  const int b = blockIdx.x;
  const int u = (a.ncu % 8 == 0) ? (b % 8) * (a.ncu / 8) + b / 8 : b;  // CU group g <-> one XCD (speed only)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long t_kernel0 = clk();
  if (threadIdx.x < C_NWORDS) S.ctl[threadIdx.x] = 0;
  __syncthreads();  // the only block-wide barrier: control words are zero before any wave runs
  if (wave < kLoaders) {
    loader(a, S, u, wave);
    return;
  }
  const unsigned ep = __hip_atomic_load((gu32*)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Cons C(a, S, u, wave - kLoaders, ep);
  const int g = u / a.cpg, gi = u - g * a.cpg;
  const int pos = *a.pos, L = pos + 1;
  const int S_ = min(a.smax, (L + 63) / 64);
  const int KPS = (L + S_ - 1) / S_;
  const int nx = a.nxu;

  // prologue: this CU's residual rows, HX of layer 0
  if (C.cw == 0) {
    if (C.lane < nx) S.xres[C.lane] = a.x[u * nx + C.lane];
    for (int j = 64 + C.lane; j < nx; j += 64) S.xres[j] = a.x[u * nx + j];
    publish_hx(C, a.gran + a.off_hx, layer_at(a, 0).attn_norm);
  }
  // Every layer is four stages (QKV, Wo, gate/up, down), each: hand-off of its input into
  // the LDS activation -> the stage's ring items -> epilogue (publishes the next input).
  // One loop, so the item code exists once in the binary.
  int n_item = 0;  // first item of the current layer in the layer's item list
  for (int l = 0; l < a.n_layer && C.ok; ++l) {
    const PdLayer Ly = layer_at(a, l);
    u64* gl = a.gran + (size_t)l * a.gran_layer;
    long long* tl = (a.tl && C.cw == 0 && C.lane == 0) ? a.tl + ((size_t)u * a.n_layer + l) * kPdStamps : nullptr;
#define PD_T(i) do { if (tl) tl[i] = wall_clock64(); } while (0)
    PD_T(0);
    C.ti = (a.tli && l == 2 && C.cw == 0 && C.lane == 0) ? a.tli + (size_t)u * kPdItemStamps * 8 : nullptr;
    C.ti_k = 0;
    int k = 0;           // next item of this layer
    float xscale = 1.f;  // RMSNorm scale of the stage input (1 for o and h)
    (void)n_item;
    for (int st = 0; st < 4 && C.ok; ++st) {
      // ---- input hand-off
      if (st == 0) {
        if (!gather_hx(C, gl + a.off_hx)) break;
        xscale = hx_rms(C);
      } else if (st == 1) {
        if (gi < S_) {  // attention split of kv head g
          const long long c0 = clk();
          if (!attention_split<G>(C, l, g, gi, S_, KPS, L)) break;
          C.ac[5] += clk() - c0;
        }
        if (gi >= a.cpg - G) {  // merge of one query head
          const long long c0 = clk();
          if (!merge_head<G>(C, l, g, gi - (a.cpg - G), S_)) break;
          C.ac[6] += clk() - c0;
        }
        const int hd = a.hd, n4 = hd / 4, n8 = hd / 8, rec = n4 + n8;
        if (!C.gather(gl + a.off_o, a.n_head * rec, 40, [&](int i, unsigned v) {
              const int h = i / rec, kk = i - h * rec;
              C.q8_store(h * hd, n4, n8, kk, v);
            }))
          break;
        xscale = 1.f;
      } else if (st == 2) {
        if (!gather_hx(C, gl + a.off_hx2)) break;
        xscale = hx_rms(C);
      } else {
        const int nf = a.nfu, n4 = nf / 4, n8 = nf / 8, rec = n4 + n8;
        if (!C.gather(gl + a.off_hh, a.ncu * rec, 60, [&](int i, unsigned v) {
              const int uu = i / rec, kk = i - uu * rec;
              C.q8_store(uu * nf, n4, n8, kk, v);
            }))
          break;
        xscale = 1.f;
      }
      PD_T(2 * st + 1);
      // ---- the stage's ring items
      const int K = st == 1 ? a.nq : (st == 3 ? a.F : a.d);
      C.begin_stage(K);
      const int last_stage = st == 0 ? PD_V : (st == 1 ? PD_WO : (st == 2 ? PD_UP : PD_DOWN));
      bool good = true;
      for (; k < Ly.nitems; ++k) {
        const PdItem it = item_at(a, Ly.item0 + k);
        if (it.stage > last_stage) break;
        if (!C.consume_item(it)) { good = false; break; }
      }
      if (!good || !C.csync()) break;
      PD_T(2 * st + 2);
      // ---- epilogue (consumer wave 0)
      if (C.cw != 0) continue;
      if (st == 0) {
        const int nrow = a.nqu + 2 * a.nku;
        const int nq2 = a.nqu / 2, nk2 = a.nku / 2;
        u64* rec = gl + a.off_qkv + (size_t)u * (nq2 + 2 * nk2);
        for (int j0 = 0; j0 < nrow; j0 += 64) {
          const int j = j0 + C.lane;
          const int jj = min(j, nrow - 1);
          float v = C.row_total(jj, a.d) * xscale;
          const bool isq = jj < a.nqu, isk = !isq && jj < a.nqu + a.nku;
          const int grow = isq ? u * a.nqu + jj : u * a.nku + (jj - a.nqu - (isk ? 0 : a.nku));
          const int dim = grow % a.hd;
          const float partner = __shfl_xor(v, 1);
          if (isq || isk) {
            const float2 cs = a.rope[(size_t)pos * (a.hd / 2) + dim / 2];
            v = (dim & 1) ? partner * cs.y + v * cs.x : v * cs.x - partner * cs.y;
          }
          if (a.dbg && j < nrow) {
            float* db = a.dbg + (size_t)l * dump_stride(a);
            const int di = isq ? grow : (isk ? a.nq + grow : a.nq + a.nkv + grow);
            db[di] = v;
          }
          if (isq) v *= a.attn_scale;
          if (!isq && j < nrow) {
            const int kvh = grow / a.hd;
            __half* cache =
                (isk ? a.k_cache : a.v_cache) + (size_t)l * a.kv_layer + ((size_t)kvh * a.n_ctx + pos) * a.hd + dim;
            *cache = __float2half(v);
          }
          const float vn = __shfl_xor(v, 1);
          if (j < nrow && (j & 1) == 0) {
            const h2v pr = {(_Float16)v, (_Float16)vn};
            const int gidx = isq ? jj / 2 : (isk ? nq2 + (jj - a.nqu) / 2 : nq2 + nk2 + (jj - a.nqu - a.nku) / 2);
            gst(rec + gidx, ep, __builtin_bit_cast(unsigned, pr));
          }
        }
      } else if (st == 1) {
        for (int j = C.lane; j < nx; j += 64) S.xres[j] += C.row_total(j, a.nq);
        if (a.dbg)
          for (int j = C.lane; j < nx; j += 64)
            a.dbg[(size_t)l * dump_stride(a) + 2 * a.nq + 2 * a.nkv + u * nx + j] = S.xres[j];
        publish_hx(C, gl + a.off_hx2, Ly.ffn_norm);
      } else if (st == 2) {
        const int nf = a.nfu;
        u64* rec = gl + a.off_hh + (size_t)u * (nf / 4 + nf / 8);
        for (int j0 = 0; j0 < nf; j0 += 64) {
          const int j = j0 + C.lane;
          const int jj = min(j, nf - 1);
          const float gv = C.row_total(jj, a.d) * xscale, uv = C.row_total(nf + jj, a.d) * xscale;
          const float h = j < nf ? silu_f(gv) * uv : 0.f;
          if (a.dbg && j < nf) a.dbg[(size_t)l * dump_stride(a) + 2 * a.nq + 2 * a.nkv + a.d + u * nf + j] = h;
          C.publish_q8(rec, h, min(64, nf - j0), j0 / 4, j0 / 8, nf / 4);
        }
      } else {
        for (int j = C.lane; j < nx; j += 64) S.xres[j] += C.row_total(j, a.F);
        if (a.dbg)
          for (int j = C.lane; j < nx; j += 64)
            a.dbg[(size_t)l * dump_stride(a) + 2 * a.nq + 2 * a.nkv + a.d + a.F + u * nx + j] = S.xres[j];
        if (l + 1 < a.n_layer) {
          publish_hx(C, a.gran + (size_t)(l + 1) * a.gran_layer + a.off_hx, layer_at(a, l + 1).attn_norm);
        } else {
          for (int j = C.lane; j < nx; j += 64) a.x[u * nx + j] = S.xres[j];
        }
      }
    }
#undef PD_T
  }
  if (a.acct && C.cw == 0 && C.lane == 0) {
    C.ac[7] = clk() - t_kernel0;
    for (int i = 0; i < 8; ++i) a.acct[(size_t)u * 16 + i] = C.ac[i];
  }
  if (u == 0 && C.cw == 0 && C.lane == 0)
    __hip_atomic_store((gu32*)a.epoch, ep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ microbenchmark
// item code alone: one workgroup per CU, ring slot and activation filled with junk that
// decodes to finite values, every consumer wave runs `iters` items of `rows` rows (type T,
// K inputs); out[block * 8 + cw] = shader cycles per item of consumer wave cw
template <int T>
__global__ __launch_bounds__(kThreads) void pd_item_bench_kernel(int rows, int K, int iters, long long* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nch = K >> 5;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xs = reinterpret_cast<float*>(smem + 16384);
  float* part = reinterpret_cast<float*>(smem + 16384 + 8192);
  uint8_t* slot = reinterpret_cast<uint8_t*>(smem + 16384 + 8192 + 4096);
  for (int i = threadIdx.x; i < K; i += blockDim.x) xq[i] = (int8_t)((i * 37) & 63);
  for (int i = threadIdx.x; i < K / 8; i += blockDim.x) xs[i] = 0.01f;
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) slot[i] = (uint8_t)(i * 13 + 7) & 0x3B;
  __syncthreads();
  if (wave < kLoaders) return;
  const int cw = wave - kLoaders;
  const StageMap m = stage_map(K, cw, lane);
  X8 xb[2];
  int lo, hi;
  chunk_x_offsets(m.c0, lo, hi);
  load_x8(xb[0], (lds_i8*)xq, (lds_cf*)xs, lo, hi);
  chunk_x_offsets(m.c1, lo, hi);
  load_x8(xb[1], (lds_i8*)xq, (lds_cf*)xs, lo, hi);
  PdItem it;
  it.off = 0; it.rows = (uint16_t)rows; it.row0 = 0; it.stage = 0; it.type = (uint8_t)T;
  it.row_bytes = pd_row_bytes_dev(T, K);
  it.dma_kb = 0;
  const long long t0 = clk();
  for (int i = 0; i < iters; ++i) {
    if (m.active) item_rows<T>((lds_u8*)slot, it, m, xb, (lds_f*)part, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const long long t1 = clk();
  if (lane == 0) out[blockIdx.x * 8 + cw] = (t1 - t0) / iters;
  (void)nch;
}

// ------------------------------------------------------------------ packing
__global__ void pd_pack_kernel(uint8_t* region, uint32_t cu_bytes, uint32_t stage_off, int rows_cu, QMat src,
                               const int* map, uint32_t rb) {
  const int i = blockIdx.x;
  const int cu = i / rows_cu, j = i - cu * rows_cu;
  const int r = map ? map[i] : i;
  uint8_t* d = region + (size_t)cu * cu_bytes + stage_off + (size_t)j * rb;
  const Planes& P = src.P;
  const uint8_t* b = src.base;
  auto cp = [&](size_t doff, const uint8_t* s, size_t n) {
    for (size_t k = threadIdx.x; k < n; k += blockDim.x) d[doff + k] = s[k];
  };
  const int K = src.K;
  if (src.type == T_Q4_K) {
    const int nsb = K / 256;
    cp(0, b + P.p1 + (size_t)r * P.s1, nsb * 16);
    cp(nsb * 16, b + P.p0 + (size_t)r * P.s0, nsb * 128);
  } else if (src.type == T_Q5_K) {
    const int nsb = K / 256;
    cp(0, b + P.p2 + (size_t)r * P.s2, nsb * 16);
    cp(nsb * 16, b + P.p1 + (size_t)r * P.s1, nsb * 32);
    cp(nsb * 48, b + P.p0 + (size_t)r * P.s0, nsb * 128);
  } else if (src.type == T_Q6_K) {
    // sc and d natively; ql/qh re-laid into the ring chunk order (see the format comment)
    const int nsb = K / 256, od = nsb * 16, oh = od + ((2 * nsb + 15) & ~15), ol = oh + nsb * 64;
    cp(0, b + P.p2 + (size_t)r * P.s2, nsb * 16);
    cp(od, b + P.p3 + (size_t)r * P.s3, nsb * 2);
    const uint8_t* qlr = b + P.p0 + (size_t)r * P.s0;
    const uint8_t* qhr = b + P.p1 + (size_t)r * P.s1;
    auto q6 = [&](int sb, int p) -> int {  // 6-bit value of position p of superblock sb (ggml order)
      const int n = p >> 7, t = (p & 127) >> 5, l = p & 31;
      const uint8_t* ql = qlr + sb * 128 + n * 64;
      const uint8_t qh = qhr[sb * 64 + n * 32 + l];
      const int lo4 = (t & 1) ? ql[l + 32] : ql[l];
      return ((t < 2) ? (lo4 & 15) : (lo4 >> 4)) | (((qh >> (2 * t)) & 3) << 4);
    };
    for (int c = threadIdx.x; c < K / 32; c += blockDim.x) {
      const int sb = c >> 3, j = c & 7, lo = 64 * (j >> 1) + 16 * (j & 1);
      unsigned qh_lo = 0, qh_hi = 0;
      for (int i = 0; i < 16; ++i) {
        const int va = q6(sb, lo + i), vb = q6(sb, lo + 32 + i);
        d[ol + 16 * c + i] = (uint8_t)((va & 15) | ((vb & 15) << 4));
        const int sh = 8 * (i & 3) + 2 * (i >> 2);
        qh_lo |= (unsigned)((va >> 4) & 3) << sh;
        qh_hi |= (unsigned)((vb >> 4) & 3) << sh;
      }
      for (int i = 0; i < 4; ++i) {
        d[oh + 8 * c + i] = (uint8_t)(qh_lo >> (8 * i));
        d[oh + 8 * c + 4 + i] = (uint8_t)(qh_hi >> (8 * i));
      }
    }
  } else {  // Q8_0: d natively; qs re-laid into the ring chunk order
    const int nb = K / 32, oq = (2 * nb + 15) & ~15;
    cp(0, b + P.p1 + (size_t)r * P.s1, nb * 2);
    const uint8_t* qs = b + P.p0 + (size_t)r * P.s0;
    for (int c = threadIdx.x; c < nb; c += blockDim.x) {
      const int sb = c >> 3, j = c & 7, bl = 8 * sb + 2 * (j >> 1), h = j & 1;
      for (int i = 0; i < 16; ++i) {
        d[oq + 32 * c + i] = qs[32 * bl + 16 * h + i];
        d[oq + 32 * c + 16 + i] = qs[32 * (bl + 1) + 16 * h + i];
      }
    }
  }
}

}  // namespace

uint32_t pd_row_bytes(int type, int K) {
  switch (type) {
    case T_Q4_K: return (uint32_t)(K / 256) * 144;
    case T_Q5_K: return (uint32_t)(K / 256) * 176;
    case T_Q6_K: return (uint32_t)(K / 256) * 208 + (((K / 256) * 2 + 15) & ~15);
    case T_Q8_0: return (uint32_t)(K / 32) * 32 + (((K / 32) * 2 + 15) & ~15);
  }
  return 0;
}

void pd_pack_rows(uint8_t* region, uint32_t cu_bytes, uint32_t stage_off, int rows_cu, int ncu, const QMat& src,
                  const int* map_dev, hipStream_t s) {
  if (rows_cu <= 0) return;
  hipLaunchKernelGGL(pd_pack_kernel, dim3(rows_cu * ncu), dim3(256), 0, s, region, cu_bytes, stage_off, rows_cu, src,
                     map_dev, pd_row_bytes(src.type, src.K));
}

size_t pdecode_lds_bytes(const PDecodeArgs& a) {
  return kCtlBytes + 256 + (size_t)((a.part_floats * 4 + 15) & ~15) + (size_t)a.act_bytes + (size_t)a.nslot * a.slot_bytes;
}

void pd_item_bench(int type, int rows, int K, int iters, int blocks, long long* out, hipStream_t s) {
  const size_t lds = 16384 + 8192 + 4096 + 16384;
  switch (type) {
    case T_Q4_K: hipLaunchKernelGGL(pd_item_bench_kernel<T_Q4_K>, dim3(blocks), dim3(kThreads), lds, s, rows, K, iters, out); break;
    case T_Q6_K: hipLaunchKernelGGL(pd_item_bench_kernel<T_Q6_K>, dim3(blocks), dim3(kThreads), lds, s, rows, K, iters, out); break;
    default: hipLaunchKernelGGL(pd_item_bench_kernel<T_Q8_0>, dim3(blocks), dim3(kThreads), lds, s, rows, K, iters, out); break;
  }
}

bool pdecode_resident(const PDecodeArgs& a) {
  const size_t lds = pdecode_lds_bytes(a);
  if (lds > 160 * 1024) return false;
  const int G = a.n_head / a.n_kv_head;
  int per_cu = 0;
  hipError_t e = hipErrorInvalidValue;
  if (G == 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pdecode_kernel<4>, kThreads, lds);
  if (G == 8) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pdecode_kernel<8>, kThreads, lds);
  return e == hipSuccess && per_cu >= 1;
}

void pdecode(const PDecodeArgs& a, const PDecodeArgs* a_dev, hipStream_t s) {
  const size_t lds = pdecode_lds_bytes(a);
  const int G = a.n_head / a.n_kv_head;
  switch (G) {
    case 4: hipLaunchKernelGGL(pdecode_kernel<4>, dim3(a.ncu), dim3(kThreads), lds, s, a_dev); break;
    case 8: hipLaunchKernelGGL(pdecode_kernel<8>, dim3(a.ncu), dim3(kThreads), lds, s, a_dev); break;
    default: throw std::runtime_error("pdecode: gqa group must be 4 or 8");
  }
}

}  // namespace lfk
