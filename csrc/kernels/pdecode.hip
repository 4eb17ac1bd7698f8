// Persistent decode step: see pdecode.h for the dataflow and the reasons.
//
// Workgroup = 8 waves on one CU: wave 0 is the LOADER (LDS-DMA of this CU's
// weight slices into an nslot-deep ring, in consumption order, whole token),
// waves 1..7 are CONSUMERS (granule gathers, integer-dot row slices out of the
// ring, epilogues, attention). The loader never joins a barrier: the ring is
// driven by two LDS counters (filled = items landed, freed = consumer-wave
// releases), the consumers meet at an LDS counter barrier (csync).
//
// Ring row format (pd_pack_rows): one row of a quantised matrix = its planar
// fields back to back, every field 16-B aligned:
//   Q4_K: meta[nsb][16] | qs[nsb][128]
//   Q5_K: meta[nsb][16] | qh[nsb][32] | qs[nsb][128]
//   Q6_K: sc[nsb][16] | d[nsb] (f16, padded to 16 B) | qh[nsb][64] | ql[nsb][128]
//   Q8_0: d[nb] (f16, padded to 16 B) | qs[nb][32]
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
// descriptors through the constant address space: wave-uniform indices -> s_load (a vector
// load would be counted by vmcnt and make the loader's waits drain its own LDS-DMA stream)
typedef const __attribute__((address_space(4))) PdItem citem;
typedef const __attribute__((address_space(4))) PdLayer clayer;
__device__ __forceinline__ PdItem item_at(const PDecodeArgs& a, int i) {
  citem* p = (citem*)a.items + i;
  PdItem r;
  r.off = p->off; r.row_bytes = p->row_bytes; r.dma_kb = p->dma_kb; r.rows = p->rows; r.row0 = p->row0;
  r.stage = p->stage; r.type = p->type;
  return r;
}
__device__ __forceinline__ PdLayer layer_at(const PDecodeArgs& a, int l) {
  clayer* p = (clayer*)a.layers + l;
  PdLayer r;
  r.wbase = p->wbase; r.cu_bytes = p->cu_bytes; r.item0 = p->item0; r.nitems = p->nitems;
  r.attn_norm = p->attn_norm; r.ffn_norm = p->ffn_norm;
  return r;
}

constexpr int kThreads = 512;
constexpr int kNCW = kThreads / 64 - 1;  // consumer waves
constexpr int kAttW = 4;                 // consumer waves that read keys (16 keys each per pass)
constexpr long long kSpinTicks = 4000000;  // 40 ms of the 100 MHz wall clock per wait

// LDS control words (ints at the start of the dynamic region)
// C_FREED0 + slot: consumer-wave releases of that ring slot, cumulative. Per slot, not one sum:
// with one sum a wave running several items ahead could make a slot look free while a slower
// wave still reads it (the loader then overwrote live ring bytes: measured, stages of 8+ items)
enum Ctl : int { C_FILLED = 0, C_CBAR = 2, C_ABORT = 3, C_FREED0 = 8, C_NWORDS = 16 };

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

__device__ __forceinline__ void load_x8(X8& X, const int8_t* xq, const float* xs, int off_lo, int off_hi) {
  const int4 a = *reinterpret_cast<const int4*>(xq + off_lo);
  const int4 b = *reinterpret_cast<const int4*>(xq + off_hi);
  X.lo[0] = a.x; X.lo[1] = a.y; X.lo[2] = a.z; X.lo[3] = a.w;
  X.hi[0] = b.x; X.hi[1] = b.y; X.hi[2] = b.z; X.hi[3] = b.w;
  const float2 sa = *reinterpret_cast<const float2*>(xs + (off_lo >> 3));
  const float2 sb = *reinterpret_cast<const float2*>(xs + (off_hi >> 3));
  X.s[0] = sa.x; X.s[1] = sa.y; X.s[2] = sb.x; X.s[3] = sb.y;
  const int ones = 0x01010101;
  X.slo = sa.x * (float)dot4(a.x, ones, dot4(a.y, ones, 0)) + sa.y * (float)dot4(a.z, ones, dot4(a.w, ones, 0));
  X.shi = sb.x * (float)dot4(b.x, ones, dot4(b.y, ones, 0)) + sb.y * (float)dot4(b.z, ones, dot4(b.w, ones, 0));
}

__device__ __forceinline__ int pad16(int b) { return (b + 15) & ~15; }
__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// x offsets of chunk c (32 weights of a row = 16 B of 4-bit data) for each type
template <int T>
__device__ __forceinline__ void chunk_x_offsets(int c, int& off_lo, int& off_hi) {
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

// dot of chunk c of one ring row (LDS) with the activation chunk X
template <int T>
__device__ __forceinline__ float rdot(const uint8_t* row, int nsb, int c, const X8& X) {
  const int sb = c >> 3, j = c & 7;
  if constexpr (T == T_Q4_K || T == T_Q5_K) {
    const int g = j >> 1;
    const int4 m = *reinterpret_cast<const int4*>(row + 16 * sb);
    int4 q, qh;
    if constexpr (T == T_Q4_K) {
      q = *reinterpret_cast<const int4*>(row + nsb * 16 + 16 * c);
    } else {
      qh = *reinterpret_cast<const int4*>(row + nsb * 16 + 32 * sb + 16 * (j & 1));
      q = *reinterpret_cast<const int4*>(row + nsb * 48 + 16 * c);
    }
    const unsigned dd = (unsigned)m.x;
    const float d = h2f(dd & 0xFFFF), dmin = h2f(dd >> 16);
    float sc_lo, m_lo, sc_hi, m_hi;
    scale_min_pair(g, (unsigned)m.y, (unsigned)m.z, (unsigned)m.w, sc_lo, m_lo, sc_hi, m_hi);
    const int qv[4] = {q.x, q.y, q.z, q.w};
    int lo[4], hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = qv[i] & 0x0F0F0F0F;
      hi[i] = (qv[i] >> 4) & 0x0F0F0F0F;
      if constexpr (T == T_Q5_K) {
        const int hv = (i == 0 ? qh.x : i == 1 ? qh.y : i == 2 ? qh.z : qh.w);
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
    const int n = j >> 2, o = 16 * (j & 3);
    const int off_d = nsb * 16, off_qh = off_d + pad16(2 * nsb), off_ql = off_qh + 64 * nsb;
    const int4 ql = *reinterpret_cast<const int4*>(row + off_ql + 16 * c);
    const int4 qh = *reinterpret_cast<const int4*>(row + off_qh + 64 * sb + 32 * n + (o & 31));
    const int si = 8 * n + (o >> 4);
    const int sc_lo = (int)*reinterpret_cast<const signed char*>(row + 16 * sb + si);
    const int sc_hi = (int)*reinterpret_cast<const signed char*>(row + 16 * sb + si + 4);
    const float d = h2f(*reinterpret_cast<const unsigned short*>(row + off_d + 2 * sb));
    const int s = (o >= 32) ? 2 : 0;
    const int lv[4] = {ql.x, ql.y, ql.z, ql.w};
    const int hv[4] = {qh.x, qh.y, qh.z, qh.w};
    int lo[4], hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (lv[i] & 0x0F0F0F0F) | (((hv[i] >> s) & 0x03030303) << 4);
      hi[i] = ((lv[i] >> 4) & 0x0F0F0F0F) | (((hv[i] >> (s + 4)) & 0x03030303) << 4);
    }
    const int dla = dot4(lo[1], X.lo[1], dot4(lo[0], X.lo[0], 0));
    const int dlb = dot4(lo[3], X.lo[3], dot4(lo[2], X.lo[2], 0));
    const int dha = dot4(hi[1], X.hi[1], dot4(hi[0], X.hi[0], 0));
    const int dhb = dot4(hi[3], X.hi[3], dot4(hi[2], X.hi[2], 0));
    return d * ((float)sc_lo * (X.s[0] * (float)dla + X.s[1] * (float)dlb - 32.f * X.slo) +
                (float)sc_hi * (X.s[2] * (float)dha + X.s[3] * (float)dhb - 32.f * X.shi));
  } else {  // Q8_0: nsb is the number of 32-blocks here
    const int off_qs = pad16(2 * nsb);
    const int4 qa = *reinterpret_cast<const int4*>(row + off_qs + 32 * c);
    const int4 qb = *reinterpret_cast<const int4*>(row + off_qs + 32 * c + 16);
    const float d = h2f(*reinterpret_cast<const unsigned short*>(row + 2 * c));
    const int a0 = dot4(qa.y, X.lo[1], dot4(qa.x, X.lo[0], 0));
    const int a1 = dot4(qa.w, X.lo[3], dot4(qa.z, X.lo[2], 0));
    const int b0 = dot4(qb.y, X.hi[1], dot4(qb.x, X.hi[0], 0));
    const int b1 = dot4(qb.w, X.hi[3], dot4(qb.z, X.hi[2], 0));
    return d * (X.s[0] * (float)a0 + X.s[1] * (float)a1 + X.s[2] * (float)b0 + X.s[3] * (float)b1);
  }
}

// All (row, 64-chunk block) units of one ring item, round-robin over the consumer
// waves; each unit's wave-reduced partial goes to part[(row0 + r) * nblk + b] (summed
// in a fixed order by the stage epilogue: deterministic).
template <int T>
__device__ __forceinline__ void item_units(const uint8_t* slot, const PdItem& it, int K, const int8_t* xq,
                                           const float* xs, float* part, int cw, int lane) {
  const int nch = K >> 5;
  const int nblk = (nch + 63) >> 6;
  const int nsb = (T == T_Q8_0) ? nch : (K >> 8);
  const int units = it.rows * nblk;
  for (int t = cw; t < units; t += kNCW) {
    const int r = t / nblk, b = t - r * nblk;
    const int c = b * 64 + lane;
    float v = 0.f;
    if (c < nch) {
      int off_lo, off_hi;
      chunk_x_offsets<T>(c, off_lo, off_hi);
      X8 X;
      load_x8(X, xq, xs, off_lo, off_hi);
      v = rdot<T>(slot + (size_t)r * it.row_bytes, nsb, c, X);
    }
    v = wave_sum_fast(v);
    if (lane == 0) part[(it.row0 + r) * nblk + b] = v;
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

__device__ __forceinline__ Lds carve(char* smem, const PDecodeArgs& a) {
  Lds L;
  L.ctl = reinterpret_cast<int*>(smem);
  L.xres = reinterpret_cast<float*>(smem + 64);
  L.part = reinterpret_cast<float*>(smem + 64 + 256);
  char* p = smem + 64 + 256 + ((a.part_floats * 4 + 15) & ~15);
  L.act = p;
  const int actn = (max(max(a.d, a.nq), a.F) + 63) & ~63;
  L.xq = reinterpret_cast<int8_t*>(p);
  L.xs = reinterpret_cast<float*>(p + actn);
  L.ssq = reinterpret_cast<float*>(p + actn + actn / 2);
  L.ring = reinterpret_cast<uint8_t*>(p + a.act_bytes);
  L.ring_lds = (unsigned)(uintptr_t)(L.ring);
  return L;
}

// ------------------------------------------------------------------ loader wave
__device__ void loader(const PDecodeArgs& a, const Lds& S, int u) {
  const int lane = threadIdx.x & 63;
  int* ctl = S.ctl;
  int n = 0, pend = -1;
  for (int l = 0; l < a.n_layer; ++l) {
    const PdLayer Ly = layer_at(a, l);
    const uint8_t* span = Ly.wbase + (size_t)u * Ly.cu_bytes;
    long long* tl = a.tl ? a.tl + ((size_t)u * a.n_layer + l) * kPdStamps : nullptr;
    for (int k = 0; k < Ly.nitems; ++k, ++n) {
      if (tl && lane == 0 && (k == 0 || k == Ly.nitems - 1)) tl[k == 0 ? 10 : 11] = wall_clock64();
      const PdItem it = item_at(a, Ly.item0 + k);
      const int slot = n % a.nslot;
      if (n >= a.nslot) {
        // every consumer wave has released every earlier item of this slot
        int* freed = ctl + C_FREED0 + slot;
        const int need = (n / a.nslot) * kNCW;
        if (lds_ld(freed) < need) {
          // about to block on the consumers: land and publish what is in flight first
          vm_wait<0>();
          if (pend >= 0) { if (lane == 0) lds_st(ctl + C_FILLED, pend + 1); pend = -1; }
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
      const uint8_t* src = span + it.off + lane * 16;
      const unsigned dst = __builtin_amdgcn_readfirstlane(S.ring_lds + (unsigned)(slot * a.slot_bytes));
      for (int kb = 0; kb < it.dma_kb; ++kb) glds16(src + kb * 1024, dst + kb * 1024);
      if (pend >= 0) {  // the previous item has landed once at most this item's transfers remain
        vm_wait_dyn(it.dma_kb);
        if (lane == 0) lds_st(ctl + C_FILLED, pend + 1);
      }
      pend = n;
    }
  }
  vm_wait<0>();
  if (pend >= 0 && lane == 0) lds_st(ctl + C_FILLED, pend + 1);
}

// ------------------------------------------------------------------ consumer helpers
struct Cons {
  const PDecodeArgs& a;
  const Lds& S;
  int u, cw, lane;
  unsigned ep;
  int phase;     // csync generation
  int n;         // next ring item
  bool ok;

  __device__ Cons(const PDecodeArgs& a_, const Lds& S_, int u_, int cw_, unsigned ep_)
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

  // wait for ring item n, run its units, release it
  __device__ bool consume_item(const PdItem& it) {
    const int need = n + 1;
    if (lds_ld(S.ctl + C_FILLED) < need) {
      long long t0 = wall_clock64();
      while (lds_ld(S.ctl + C_FILLED) < need) {
        if (lds_ld(S.ctl + C_ABORT)) { ok = false; return false; }
        if (wall_clock64() - t0 > kSpinTicks) return fail(90);
        __builtin_amdgcn_s_sleep(0);
      }
    }
    const uint8_t* slot = S.ring + (size_t)(n % a.nslot) * a.slot_bytes;
    const int K = it.stage == PD_WO ? a.nq : (it.stage == PD_DOWN ? a.F : a.d);
    switch (it.type) {
      case T_Q4_K: item_units<T_Q4_K>(slot, it, K, S.xq, S.xs, S.part, cw, lane); break;
      case T_Q5_K: item_units<T_Q5_K>(slot, it, K, S.xq, S.xs, S.part, cw, lane); break;
      case T_Q6_K: item_units<T_Q6_K>(slot, it, K, S.xq, S.xs, S.part, cw, lane); break;
      default: item_units<T_Q8_0>(slot, it, K, S.xq, S.xs, S.part, cw, lane); break;
    }
    // every LDS read of the slot has returned before the release (the add is a release)
    if (lane == 0) lds_add(S.ctl + C_FREED0 + n % a.nslot, 1);
    ++n;
    return true;
  }

  // consume the items [k0, k1) of layer l's item list
  __device__ bool consume(const PdLayer& Ly, int k0, int k1) {
    for (int k = k0; k < k1; ++k)
      if (!consume_item(item_at(a, Ly.item0 + k))) return false;
    return csync();
  }

  // stage total of per-CU row j (sum of its blocks in a fixed order)
  __device__ float row_total(int j, int K) const {
    const int nblk = ((K >> 5) + 63) >> 6;
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += S.part[j * nblk + b];
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
  const PDecodeArgs& a = C.a;
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
  const PDecodeArgs& a = C.a;
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
  const PDecodeArgs& a = C.a;
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
  const PDecodeArgs& a = C.a;
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
  if (a.dbg) a.dbg[(size_t)l * pd_dump_stride(a) + a.nq + 2 * a.nkv + h * HD + dd] = ov;
  u64* rec = gl + a.off_o + (size_t)h * (HD / 4 + HD / 8);
  // lane group of wave cw covers dims [64cw, 64cw + 64): int8x4 records 16cw.., scales 8cw..
  C.publish_q8(rec, ov, 64, C.cw * 16, C.cw * 8, HD / 4);
  return true;
}

// ------------------------------------------------------------------ the kernel
template <int G>
__global__ __launch_bounds__(kThreads) void pdecode_kernel(PDecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds S = carve(smem, a);
  const int b = blockIdx.x;
  const int u = (a.ncu % 8 == 0) ? (b % 8) * (a.ncu / 8) + b / 8 : b;  // CU group g <-> one XCD (speed only)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < C_NWORDS) S.ctl[threadIdx.x] = 0;
  __syncthreads();  // the only block-wide barrier: control words are zero before any wave runs
  if (wave == 0) {
    loader(a, S, u);
    return;
  }
  const unsigned ep = __hip_atomic_load((gu32*)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Cons C(a, S, u, wave - 1, ep);
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
  for (int l = 0; l < a.n_layer && C.ok; ++l) {
    const PdLayer Ly = layer_at(a, l);
    u64* gl = a.gran + (size_t)l * a.gran_layer;
    long long* tl = (a.tl && C.cw == 0 && C.lane == 0) ? a.tl + ((size_t)u * a.n_layer + l) * kPdStamps : nullptr;
#define PD_T(i) do { if (tl) tl[i] = wall_clock64(); } while (0)
    PD_T(0);
    // item ranges of the stages (items are stage-ordered)
    int kq = 0, kw0 = 0, kg0 = 0, kd0 = 0;
    {
      int k = 0;
      while (k < Ly.nitems && item_at(a, Ly.item0 + k).stage <= PD_V) ++k;
      kw0 = k;
      while (k < Ly.nitems && item_at(a, Ly.item0 + k).stage == PD_WO) ++k;
      kg0 = k;
      while (k < Ly.nitems && item_at(a, Ly.item0 + k).stage <= PD_UP) ++k;
      kd0 = k;
    }
    // ---- QKV
    if (!gather_hx(C, gl + a.off_hx)) break;
    PD_T(1);
    const float rms_a = hx_rms(C);
    if (!C.consume(Ly, kq, kw0)) break;
    PD_T(2);
    if (C.cw == 0) {
      const int nrow = a.nqu + 2 * a.nku;
      const int nq2 = a.nqu / 2, nk2 = a.nku / 2;
      u64* rec = gl + a.off_qkv + (size_t)u * (nq2 + 2 * nk2);
      for (int j0 = 0; j0 < nrow; j0 += 64) {
        const int j = j0 + C.lane;
        const int jj = min(j, nrow - 1);
        float v = C.row_total(jj, a.d) * rms_a;
        const bool isq = jj < a.nqu, isk = !isq && jj < a.nqu + a.nku;
        const int grow = isq ? u * a.nqu + jj : u * a.nku + (jj - a.nqu - (isk ? 0 : a.nku));
        const int dim = grow % a.hd;
        const float partner = __shfl_xor(v, 1);
        if (isq || isk) {
          const float2 cs = a.rope[(size_t)pos * (a.hd / 2) + dim / 2];
          v = (dim & 1) ? partner * cs.y + v * cs.x : v * cs.x - partner * cs.y;
        }
        if (a.dbg && j < nrow) {
          float* db = a.dbg + (size_t)l * pd_dump_stride(a);
          const int di = isq ? grow : (isk ? a.nq + grow : a.nq + a.nkv + grow);
          db[di] = v;
        }
        if (isq) v *= a.attn_scale;
        if (!isq && j < nrow) {
          const int kvh = grow / a.hd;
          __half* cache = (isk ? a.k_cache : a.v_cache) + (size_t)l * a.kv_layer + ((size_t)kvh * a.n_ctx + pos) * a.hd + dim;
          *cache = __float2half(v);
        }
        const float vn = __shfl_xor(v, 1);
        if (j < nrow && (j & 1) == 0) {
          const h2v pr = {(_Float16)v, (_Float16)vn};
          const int gidx = isq ? jj / 2 : (isk ? nq2 + (jj - a.nqu) / 2 : nq2 + nk2 + (jj - a.nqu - a.nku) / 2);
          gst(rec + gidx, ep, __builtin_bit_cast(unsigned, pr));
        }
      }
    }
    // ---- attention (splits) and merges
    if (gi < S_) {
      if (!attention_split<G>(C, l, g, gi, S_, KPS, L)) break;
    }
    if (gi >= a.cpg - G) {
      if (!merge_head<G>(C, l, g, gi - (a.cpg - G), S_)) break;
    }
    PD_T(3);
    // ---- Wo
    {
      const int hd = a.hd, n4 = hd / 4, n8 = hd / 8, rec = n4 + n8;
      if (!C.gather(gl + a.off_o, a.n_head * rec, 40, [&](int i, unsigned v) {
            const int h = i / rec, k = i - h * rec;
            C.q8_store(h * hd, n4, n8, k, v);
          }))
        break;
    }
    PD_T(4);
    if (!C.consume(Ly, kw0, kg0)) break;
    PD_T(5);
    if (C.cw == 0) {
      for (int j = C.lane; j < nx; j += 64) S.xres[j] += C.row_total(j, a.nq);
      if (a.dbg)
        for (int j = C.lane; j < nx; j += 64) a.dbg[(size_t)l * pd_dump_stride(a) + 2 * a.nq + 2 * a.nkv + u * nx + j] = S.xres[j];
      publish_hx(C, gl + a.off_hx2, Ly.ffn_norm);
    }
    // ---- gate/up + SwiGLU
    if (!gather_hx(C, gl + a.off_hx2)) break;
    PD_T(6);
    const float rms_f = hx_rms(C);
    if (!C.consume(Ly, kg0, kd0)) break;
    PD_T(7);
    if (C.cw == 0) {
      const int nf = a.nfu;
      u64* rec = gl + a.off_hh + (size_t)u * (nf / 4 + nf / 8);
      for (int j0 = 0; j0 < nf; j0 += 64) {
        const int j = j0 + C.lane;
        const int jj = min(j, nf - 1);
        const float gv = C.row_total(jj, a.d) * rms_f, uv = C.row_total(nf + jj, a.d) * rms_f;
        const float h = j < nf ? silu_f(gv) * uv : 0.f;
        if (a.dbg && j < nf) a.dbg[(size_t)l * pd_dump_stride(a) + 2 * a.nq + 2 * a.nkv + a.d + u * nf + j] = h;
        C.publish_q8(rec, h, min(64, nf - j0), j0 / 4, j0 / 8, nf / 4);
      }
    }
    // ---- down
    {
      const int nf = a.nfu, n4 = nf / 4, n8 = nf / 8, rec = n4 + n8;
      if (!C.gather(gl + a.off_hh, a.ncu * rec, 60, [&](int i, unsigned v) {
            const int uu = i / rec, k = i - uu * rec;
            C.q8_store(uu * nf, n4, n8, k, v);
          }))
        break;
    }
    PD_T(8);
    if (!C.consume(Ly, kd0, Ly.nitems)) break;
    PD_T(9);
#undef PD_T
    if (C.cw == 0) {
      for (int j = C.lane; j < nx; j += 64) S.xres[j] += C.row_total(j, a.F);
      if (a.dbg)
        for (int j = C.lane; j < nx; j += 64)
          a.dbg[(size_t)l * pd_dump_stride(a) + 2 * a.nq + 2 * a.nkv + a.d + a.F + u * nx + j] = S.xres[j];
      if (l + 1 < a.n_layer) {
        publish_hx(C, a.gran + (size_t)(l + 1) * a.gran_layer + a.off_hx, layer_at(a, l + 1).attn_norm);
      } else {
        for (int j = C.lane; j < nx; j += 64) a.x[u * nx + j] = S.xres[j];
      }
    }
  }
  if (u == 0 && C.cw == 0 && C.lane == 0)
    __hip_atomic_store((gu32*)a.epoch, ep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    const int nsb = K / 256, od = nsb * 16, oh = od + ((2 * nsb + 15) & ~15);
    cp(0, b + P.p2 + (size_t)r * P.s2, nsb * 16);
    cp(od, b + P.p3 + (size_t)r * P.s3, nsb * 2);
    cp(oh, b + P.p1 + (size_t)r * P.s1, nsb * 64);
    cp(oh + nsb * 64, b + P.p0 + (size_t)r * P.s0, nsb * 128);
  } else {  // Q8_0
    const int nb = K / 32, oq = (2 * nb + 15) & ~15;
    cp(0, b + P.p1 + (size_t)r * P.s1, nb * 2);
    cp(oq, b + P.p0 + (size_t)r * P.s0, nb * 32);
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
  return 64 + 256 + (size_t)((a.part_floats * 4 + 15) & ~15) + (size_t)a.act_bytes + (size_t)a.nslot * a.slot_bytes;
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

void pdecode(const PDecodeArgs& a, hipStream_t s) {
  const size_t lds = pdecode_lds_bytes(a);
  const int G = a.n_head / a.n_kv_head;
  switch (G) {
    case 4: hipLaunchKernelGGL(pdecode_kernel<4>, dim3(a.ncu), dim3(kThreads), lds, s, a); break;
    case 8: hipLaunchKernelGGL(pdecode_kernel<8>, dim3(a.ncu), dim3(kThreads), lds, s, a); break;
    default: throw std::runtime_error("pdecode: gqa group must be 4 or 8");
  }
}

}  // namespace lfk
