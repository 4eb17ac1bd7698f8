// Weight-ring microbenchmark for the batched decode's wave-owned gate/up (bmm.hip wt_body): does
// an LDS-DMA weight ring (global -> LDS loads with no VGPR destination, D steps in flight per
// wave) overlap the Q4_K dequantisation + MFMA with the HBM stream better than the register ring
// (PD steps of raw weights in VGPRs)? Same shape as the kernel: 256 blocks x 7 busy waves, each
// wave one tile16 tile = 16 contiguous 2560-B steps (73.4 MB per launch), every launch on a fresh
// region of a 1.5 GB buffer (the Infinity Cache holds none of it), random quant bytes and random
// f16 B operands in LDS (zero operands run the MFMAs at a clock they do not get on real data).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/ring_bench tools/ring_bench.hip && build/ring_bench
//
// Variants: stream (loads only), compute (dequant + MFMA on register-resident data, no loads),
// reg PD (the production register ring), dma D (per-wave LDS-DMA ring, D steps in flight; the
// wave reads its own slot back with ds_read after a counted vmcnt - no barrier: only the issuing
// wave reads a slot).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));

constexpr int kTiles = 1792, kSteps = 16, kSB = 2560, kWavesBusy = 7, kBlocks = 256;
constexpr int kXBytes = 16384;  // the B-operand region (random f16)

__device__ __forceinline__ h2_t as_h2(unsigned v) { return __builtin_bit_cast(h2_t, v); }
__device__ __forceinline__ unsigned as_u(h2_t v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ unsigned bytes02(unsigned x) { return __builtin_amdgcn_perm(0x64646464u, x, 0x04020400u); }
__device__ __forceinline__ unsigned bytes13(unsigned x) { return __builtin_amdgcn_perm(0x64646464u, x, 0x04030401u); }
__device__ __forceinline__ unsigned deq_pair(unsigned mp, h2_t bias, h2_t a, h2_t m) {
  const h2_t v = as_h2(mp) - bias;
  return as_u(v * a + m);
}

struct Raw {  // one chunk (h) of a step: 16 quant bytes + the (d*sc, -dmin*m) pair of its 2 sub-blocks
  int4 q;
  uint2 m;
};

struct HFrag {
  unsigned w[16];
};

__device__ __forceinline__ void dequant(const Raw& w, HFrag& F) {
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
}

// one 256-k step (bmm_step's IL form): 8 B-operand LDS reads, both chunks dequantised, 8 MFMAs
template <bool HALF = false>
__device__ __forceinline__ void step_compute(const Raw* wc, int s, int kq, const __half* xrow, f4_t& acc, f4_t& acc2) {
  auto frag = [](const HFrag& F, int m) {
    const int dw = 2 * (m & 1), sh = (m >> 1) * 2;
    return make_uint4(F.w[4 * dw + sh], F.w[4 * dw + sh + 1], F.w[4 * dw + 4 + sh], F.w[4 * dw + 5 + sh]);
  };
  uint4 xr[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 8 * s + 4 * h + kq, j = c & 7;
    const int off_lo = (64 * (j >> 1) + 16 * (j & 1)) & 4095, off_hi = off_lo + 32;
    const uint4* xl = reinterpret_cast<const uint4*>(xrow + off_lo);
    const uint4* xh = reinterpret_cast<const uint4*>(xrow + off_hi);
    xr[h][0] = xl[0]; xr[h][1] = xl[1]; xr[h][2] = xh[0]; xr[h][3] = xh[1];
  }
  HFrag F0, F1;
  dequant(wc[0], F0);
  if constexpr (HALF) {
#pragma unroll
    for (int i = 0; i < 16; ++i) F1.w[i] = F0.w[i] ^ (unsigned)wc[1].q.x;
  } else {
    dequant(wc[1], F1);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, frag(F0, m)), __builtin_bit_cast(h8_t, xr[0][m]), acc, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, frag(F1, m)), __builtin_bit_cast(h8_t, xr[1][m]), acc2, 0, 0, 0);
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7FFFFFFF, 0x00020000);
}

// register load of one step (the production tload_rs form: nt quant planes, cached scale pairs)
__device__ __forceinline__ void rload(Raw* w, __amdgpu_buffer_rsrc_t rs, int so, int lane, int r16, int kq) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const v4i_t t = __builtin_bit_cast(v4i_t, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, so + h * 1024, 2));
    w[h].q = make_int4(t.x, t.y, t.z, t.w);
    const v2i_t u = __builtin_bit_cast(v2i_t, __builtin_amdgcn_raw_buffer_load_b64(rs, r16 * 32 + 8 * (kq >> 1), so + 2048 + 16 * h, 0));
    w[h].m = make_uint2((unsigned)u.x, (unsigned)u.y);
  }
}

// LDS-DMA of one step into an LDS slot (lane-linear: lane l's 16 B of a 1 KB piece land at
// slot + l * 16, its 4 B of a 256-B piece at slot + l * 4). M0 carries the wave-uniform LDS address.
// (M0 is compiler-reserved: saved and restored inside the statement that sets it)
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma_step(const unsigned char* p, unsigned slot, int lane) {
  slot = __builtin_amdgcn_readfirstlane(slot);  // (wave-uniform; the compiler cannot tell)
  dma16(p + lane * 16, slot);
  dma16(p + 1024 + lane * 16, slot + 1024);
  dma4(p + 2048 + lane * 4, slot + 2048);
  dma4(p + 2304 + lane * 4, slot + 2304);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


// the loader's counted wait: n = DMA instructions allowed to stay outstanding (a multiple of 21)
__device__ __forceinline__ void vm_wait_rt(int n) {
  if (n >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  else if (n >= 42) asm volatile("s_waitcnt vmcnt(42)" ::: "memory");
  else if (n >= 21) asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// MODE 8: one loader wave (wave 7) streams every tile's step s of the block into phase slot s % (D + 1)
// by LDS-DMA (3 pieces per step block: 2 x 1 KB quant, 512 B scale pairs on 32 lanes), D phases ahead;
// 7 consumer waves compute; one raw barrier per phase (the loader's counted vmcnt makes the phase's
// data visible; the consumers' lgkmcnt(0) frees the slot the loader refills next)
template <int D>
__device__ __forceinline__ void engine_body(const unsigned char* base, char* smem, const __half* xrow, int blk, int wave,
                                            int lane, int r16, int kq, f4_t& acc, f4_t& acc2) {
  constexpr int NS = D + 1, PH = kWavesBusy * kSB;  // slots, bytes per phase
  static_assert(3 * kWavesBusy * (D - 1) <= 63, "vmcnt range");
  char* ring = smem + kXBytes;
  const unsigned ring_lds = (unsigned)(size_t)ring;
  const unsigned char* tb = base + (size_t)blk * kWavesBusy * kSteps * kSB;
  auto issue = [&](int ph) {  // loader: phase ph of every tile
    const unsigned slot = __builtin_amdgcn_readfirstlane(ring_lds + (ph % NS) * PH);
#pragma unroll
    for (int c = 0; c < kWavesBusy; ++c) {
      const unsigned char* p = tb + ((size_t)c * kSteps + ph) * kSB;
      dma16(p + lane * 16, slot + c * kSB);
      dma16(p + 1024 + lane * 16, slot + c * kSB + 1024);
      if (lane < 32) dma16(p + 2048 + lane * 16, slot + c * kSB + 2048);
    }
  };
  const bool loader = wave == kWavesBusy;
  if (loader) {
#pragma unroll
    for (int p = 0; p < D; ++p) issue(p);
    vm_wait_rt(21 * (D - 1));  // phase 0 landed
  }
  lds_barrier();
#pragma unroll
  for (int p = 0; p < kSteps; ++p) {
    if (loader) {
      if (p + D < kSteps) issue(p + D);
      const int after = (p + D < kSteps ? p + D : kSteps - 1) - (p + 1);  // phases issued after p + 1
      if (p + 1 < kSteps) vm_wait_rt(21 * (after > 0 ? after : 0));
    } else {
      const char* slot = ring + (p % NS) * PH + wave * kSB;
      Raw w[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        w[h].q = *reinterpret_cast<const int4*>(slot + h * 1024 + lane * 16);
        w[h].m = *reinterpret_cast<const uint2*>(slot + 2048 + r16 * 32 + 8 * (2 * h + (kq >> 1)));
      }
      step_compute(w, p, kq, xrow, acc, acc2);
    }
    lds_barrier();
  }
}

// MODE 0 stream only, 1 compute only, 2 register ring (PD), 3 LDS-DMA ring (PD = slots in flight)
template <int MODE, int PD>
__global__ __launch_bounds__(512, 1) void ring_kernel(const unsigned char* base, const __half* xsrc, float* out, int dump) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __half* xs = reinterpret_cast<__half*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, blk = blockIdx.x;
  for (int i = tid; i < kXBytes / 16; i += 512)
    reinterpret_cast<uint4*>(xs)[i] = reinterpret_cast<const uint4*>(xsrc)[i];
  __syncthreads();
  if constexpr (MODE == 8) {
    const int r16 = lane & 15, kq = lane >> 4;
    f4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = acc;
    engine_body<PD>(base, smem, xs + r16 * 512, blk, wave, lane, r16, kq, acc, acc2);
    acc += acc2;
    if (dump == 1 && wave < kWavesBusy) reinterpret_cast<f4_t*>(out)[blk * 512 + tid] = acc;
    else if (acc[0] == 1.2345f) out[blk * 512 + tid] = acc[1] + acc[2] + acc[3];
    return;
  }
  if (wave >= kWavesBusy) return;
  const int tile = blk * kWavesBusy + wave, r16 = lane & 15, kq = lane >> 4;
  const unsigned char* tp = base + (size_t)tile * kSteps * kSB;
  const auto rs = rsrc(tp);
  const __half* xrow = xs + r16 * 512;
  f4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = acc;
  if constexpr (MODE == 0) {
    constexpr int R = PD + 1;
    Raw buf[R][2];
    unsigned fold = 0;
#pragma unroll
    for (int p = 0; p < PD; ++p) rload(buf[p], rs, p * kSB, lane, r16, kq);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      rload(buf[(s + PD) % R], rs, (s + PD < kSteps ? s + PD : 0) * kSB, lane, r16, kq);
      const Raw* b = buf[s % R];
#pragma unroll
      for (int h = 0; h < 2; ++h) fold ^= b[h].q.x ^ b[h].q.y ^ b[h].q.z ^ b[h].q.w ^ b[h].m.x ^ b[h].m.y;
    }
    acc[0] = (float)fold;
  } else if constexpr (MODE == 7) {  // stream, plain global loads (stream_bench.hip's form)
    constexpr int R = PD + 1;
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    u4 bq[R][2];
    unsigned fold = 0;
    auto gl = [&](int s2, int r) {
      const unsigned char* p = tp + (size_t)s2 * kSB;
      bq[r][0] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p + lane * 16));
      bq[r][1] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p + 1024 + lane * 16));
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) gl(p, p);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      if (s + PD < kSteps) gl(s + PD, (s + PD) % R);
#pragma unroll
      for (int h = 0; h < 2; ++h) fold ^= bq[s % R][h].x ^ bq[s % R][h].y ^ bq[s % R][h].z ^ bq[s % R][h].w;
    }
    acc[0] = (float)fold;
  } else if constexpr (MODE == 9) {  // register ring PD over a step-major layout [step][tile]
    constexpr int R = PD + 1;
    Raw buf[R][2];
    const auto rb = rsrc(base);  // (kernel argument: uniform, no waterfall)
    const int vt = tile * kSB;   // the wave's tile inside a step band
    auto ld = [&](Raw* w, int s2) {
      const int so = s2 * kTiles * kSB;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const v4i_t t = __builtin_bit_cast(v4i_t, __builtin_amdgcn_raw_buffer_load_b128(rb, vt + lane * 16, so + h * 1024, 2));
        w[h].q = make_int4(t.x, t.y, t.z, t.w);
        const v2i_t u = __builtin_bit_cast(v2i_t, __builtin_amdgcn_raw_buffer_load_b64(rb, vt + r16 * 32 + 8 * (kq >> 1), so + 2048 + 16 * h, 0));
        w[h].m = make_uint2((unsigned)u.x, (unsigned)u.y);
      }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) ld(buf[p], p);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      ld(buf[(s + PD) % R], s + PD < kSteps ? s + PD : 0);
      __builtin_amdgcn_sched_barrier(0);
      step_compute(buf[s % R], s, kq, xrow, acc, acc2);
    }
  } else if constexpr (MODE == 10) {  // MODE 2 without the waterfall: buffer resource over the kernel argument
    constexpr int R = PD + 1;
    Raw buf[R][2];
    const auto rb = rsrc(base);
    const int vt = tile * kSteps * kSB;
    auto ld = [&](Raw* w, int s2) {
      const int so = s2 * kSB;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const v4i_t t = __builtin_bit_cast(v4i_t, __builtin_amdgcn_raw_buffer_load_b128(rb, vt + lane * 16, so + h * 1024, 2));
        w[h].q = make_int4(t.x, t.y, t.z, t.w);
        const v2i_t u = __builtin_bit_cast(v2i_t, __builtin_amdgcn_raw_buffer_load_b64(rb, vt + r16 * 32 + 8 * (kq >> 1), so + 2048 + 16 * h, 0));
        w[h].m = make_uint2((unsigned)u.x, (unsigned)u.y);
      }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) ld(buf[p], p);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      ld(buf[(s + PD) % R], s + PD < kSteps ? s + PD : 0);
      __builtin_amdgcn_sched_barrier(0);
      step_compute(buf[s % R], s, kq, xrow, acc, acc2);
    }
  } else if constexpr (MODE == 4) {  // register ring PD, half the dequantisation (chunk 0's fragments for both)
    constexpr int R = PD + 1;
    Raw buf[R][2];
#pragma unroll
    for (int p = 0; p < PD; ++p) rload(buf[p], rs, p * kSB, lane, r16, kq);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      rload(buf[(s + PD) % R], rs, (s + PD < kSteps ? s + PD : 0) * kSB, lane, r16, kq);
      __builtin_amdgcn_sched_barrier(0);
      Raw w2[2] = {buf[s % R][0], buf[s % R][1]};
      w2[1].q.x ^= buf[s % R][1].q.y ^ buf[s % R][1].q.z ^ buf[s % R][1].q.w ^ buf[s % R][1].m.x ^ buf[s % R][1].m.y;
      step_compute<true>(w2, s, kq, xrow, acc, acc2);
    }
  } else if constexpr (MODE == 1) {
    Raw w[2];
    rload(w, rs, 0, lane, r16, kq);
#pragma unroll 2
    for (int s = 0; s < kSteps; ++s) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // every word changes per step: nothing of the dequantisation is hoisted
        w[h].q.x += s; w[h].q.y ^= s; w[h].q.z += 3 * s; w[h].q.w ^= 5 * s;
        w[h].m.x ^= (unsigned)s << 3; w[h].m.y ^= (unsigned)s << 5;
      }
      step_compute(w, s, kq, xrow, acc, acc2);
    }
  } else if constexpr (MODE == 6) {  // MODE 2 with per-step s_memtime stamps (out: [wave][34] u64)
    constexpr int R = PD + 1;
    Raw buf[R][2];
    unsigned long long* st = reinterpret_cast<unsigned long long*>(out) + (size_t)(blk * kWavesBusy + wave) * 34;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int p = 0; p < PD; ++p) rload(buf[p], rs, p * kSB, lane, r16, kq);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      rload(buf[(s + PD) % R], rs, (s + PD < kSteps ? s + PD : 0) * kSB, lane, r16, kq);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PD) : "memory");
      const unsigned long long tw = __builtin_amdgcn_s_memtime();
      step_compute(buf[s % R], s, kq, xrow, acc, acc2);
      asm volatile("s_nop 0" ::"v"(acc[0]), "v"(acc2[0]));
      const unsigned long long tc = __builtin_amdgcn_s_memtime();
      if (lane == 0 && dump == 2) { st[2 + 2 * s] = tw - t0; st[3 + 2 * s] = tc - t0; }
    }
    if (lane == 0 && dump == 2) { st[0] = t0; st[1] = __builtin_amdgcn_s_memtime() - t0; }
  } else if constexpr (MODE == 2) {
    constexpr int R = PD + 1;
    Raw buf[R][2];
#pragma unroll
    for (int p = 0; p < PD; ++p) rload(buf[p], rs, p * kSB, lane, r16, kq);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      rload(buf[(s + PD) % R], rs, (s + PD < kSteps ? s + PD : 0) * kSB, lane, r16, kq);
      __builtin_amdgcn_sched_barrier(0);
      step_compute(buf[s % R], s, kq, xrow, acc, acc2);
    }
  } else {
    // this wave's ring: PD + 1 slots of kSB bytes past the x region
    constexpr int R = PD + 1;
    const unsigned ring = (unsigned)(size_t)(smem + kXBytes) + wave * R * kSB;
#pragma unroll
    for (int p = 0; p < PD; ++p) dma_step(tp + p * kSB, ring + p * kSB, lane);
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      dma_step(tp + (s + PD < kSteps ? s + PD : 0) * kSB, ring + ((s + PD) % R) * kSB, lane);
      vm_wait<4 * PD>();  // step s has landed (4 DMAs per step, PD steps issued after it)
      const char* slot = smem + kXBytes + (wave * R + s % R) * kSB;
      Raw w[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        w[h].q = *reinterpret_cast<const int4*>(slot + h * 1024 + lane * 16);
        w[h].m = *reinterpret_cast<const uint2*>(slot + 2048 + r16 * 32 + 8 * (2 * h + (kq >> 1)));
      }
      step_compute(w, s, kq, xrow, acc, acc2);
    }
    vm_wait<0>();
  }
  acc += acc2;
  if (dump == 1) reinterpret_cast<f4_t*>(out)[blk * 512 + tid] = acc;  // (dump 2: out holds the stamps only)
  else if (acc[0] == 1.2345f) out[blk * 512 + tid] = acc[1] + acc[2] + acc[3];
}

// (at least 81 KB, as the production launchers request: one block per CU, so every CU runs one
// block of 7 busy waves - with 16 KB the dispatcher may pack several blocks onto one CU)
static constexpr size_t lds_of(int mode, int pd) {
  const size_t need = kXBytes + (mode == 3 || mode == 8 ? (size_t)kWavesBusy * (pd + 1) * kSB : 0);
  return need > 83 * 1024 ? need : 83 * 1024;
}

// MODE 5: 16 waves per CU (1024 threads), two waves per tile (8 steps each), register ring PD
template <int PD>
__global__ __launch_bounds__(1024, 1) void ring16_kernel(const unsigned char* base, const __half* xsrc, float* out, int dump) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __half* xs = reinterpret_cast<__half*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, blk = blockIdx.x;
  for (int i = tid; i < kXBytes / 16; i += 1024)
    reinterpret_cast<uint4*>(xs)[i] = reinterpret_cast<const uint4*>(xsrc)[i];
  __syncthreads();
  if (wave >= 2 * kWavesBusy) return;
  const int tile = blk * kWavesBusy + (wave >> 1), half = wave & 1, r16 = lane & 15, kq = lane >> 4;
  const unsigned char* tp = base + ((size_t)tile * kSteps + half * (kSteps / 2)) * kSB;
  const auto rs = rsrc(tp);
  const __half* xrow = xs + r16 * 512;
  f4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = acc;
  constexpr int R = PD + 1, NS = kSteps / 2;
  Raw buf[R][2];
#pragma unroll
  for (int p = 0; p < PD; ++p) rload(buf[p], rs, p * kSB, lane, r16, kq);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    rload(buf[(s + PD) % R], rs, (s + PD < NS ? s + PD : 0) * kSB, lane, r16, kq);
    __builtin_amdgcn_sched_barrier(0);
    step_compute(buf[s % R], s, kq, xrow, acc, acc2);
  }
  acc += acc2;
  if (acc[0] == 1.2345f) out[blk * 1024 + tid] = acc[1] + acc[2] + acc[3];
}

template <int PD>
static double run16(const unsigned char* buf, size_t region, int nreg, const __half* x, float* out, hipStream_t st, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t lds = lds_of(2, PD);
  CK(hipFuncSetAttribute((const void*)ring16_kernel<PD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int i = 0; i < nreg; ++i) hipLaunchKernelGGL((ring16_kernel<PD>), dim3(kBlocks), dim3(1024), lds, st, buf + i * region, x, out, 0);
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((ring16_kernel<PD>), dim3(kBlocks), dim3(1024), lds, st, buf + (i % nreg) * region, x, out, 0);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / iters;
}


template <int MODE, int PD>
static double run(const unsigned char* buf, size_t region, int nreg, const __half* x, float* out, hipStream_t st, int iters) {
  const size_t lds = lds_of(MODE, PD);
  CK(hipFuncSetAttribute((const void*)ring_kernel<MODE, PD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < nreg; ++i) hipLaunchKernelGGL((ring_kernel<MODE, PD>), dim3(kBlocks), dim3(512), lds, st, buf + i * region, x, out, 0);
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((ring_kernel<MODE, PD>), dim3(kBlocks), dim3(512), lds, st, buf + (i % nreg) * region, x, out, 0);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3 / iters;
}

// correctness of the DMA ring: the same accumulators as the register ring on the same data
template <int MODE, int PD>
static std::vector<float> dump(const unsigned char* buf, const __half* x, float* out4, hipStream_t st) {
  const size_t lds = lds_of(MODE, PD);
  CK(hipFuncSetAttribute((const void*)ring_kernel<MODE, PD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipMemsetAsync(out4, 0, (size_t)kBlocks * 512 * 16, st));
  hipLaunchKernelGGL((ring_kernel<MODE, PD>), dim3(kBlocks), dim3(512), lds, st, buf, x, out4, 1);
  CK(hipStreamSynchronize(st));
  CK(hipGetLastError());
  std::vector<float> h((size_t)kBlocks * 512 * 4);
  CK(hipMemcpy(h.data(), out4, h.size() * 4, hipMemcpyDeviceToHost));
  return h;
}

// stream-only and compute-only launches side by side on two streams: do the CUs overlap them?
static double run_concurrent(const unsigned char* buf, size_t region, int nreg, const __half* x, float* out, float* out2,
                             hipStream_t st, hipStream_t st2, int iters, int which) {
  hipEvent_t e0, e1, j;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&j));
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  CK(hipStreamWaitEvent(st2, e0, 0));
  for (int i = 0; i < iters; ++i) {
    if (which & 1)
      hipLaunchKernelGGL((ring_kernel<0, 2>), dim3(kBlocks), dim3(512), kXBytes, st, buf + (i % nreg) * region, x, out, 0);
    if (which & 2)
      hipLaunchKernelGGL((ring_kernel<1, 2>), dim3(kBlocks), dim3(512), kXBytes, st2, buf + (i % nreg) * region, x, out2, 0);
  }
  CK(hipEventRecord(j, st2));
  CK(hipStreamWaitEvent(st, j, 0));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
  const bool memset_init = argc > 1 && argv[1][0] == 'm';
  const size_t bytes = (size_t)kTiles * kSteps * kSB;
  const size_t region = (bytes + 4095) / 4096 * 4096;
  const int nreg = argc > 2 ? atoi(argv[2]) : 20;
  unsigned char* buf;
  __half* x;
  float* out;
  CK(hipMalloc(&buf, region * nreg));
  CK(hipMalloc(&x, kXBytes));
  CK(hipMalloc(&out, kBlocks * 512 * 4));
  {
    std::vector<unsigned> h(region * nreg / 4);
    unsigned s = 12345u;
    for (auto& v : h) {
      s = s * 1664525u + 1013904223u;
      v = s;
    }
    // scale pairs: finite f16 (exponent bits kept away from inf / nan)
    for (size_t i = 0; i < h.size(); ++i) {
      const size_t off = (i * 4) % kSB;
      if (off >= 2048) h[i] &= 0x3BFF3BFFu;
    }
    CK(hipMemcpy(buf, h.data(), region * nreg, hipMemcpyHostToDevice));
    if (memset_init) {  // A/B: a constant fill (as tools/stream_bench.hip)
      CK(hipMemset(buf, 0x5a, region * nreg));
      printf("buffer: memset 0x5a\n");
    }
    std::vector<unsigned short> hx(kXBytes / 2);
    for (auto& v : hx) {
      s = s * 1664525u + 1013904223u;
      v = (unsigned short)(0x3000 | (s >> 22));  // small positive f16
    }
    CK(hipMemcpy(x, hx.data(), kXBytes, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  {
    float* out4;
    CK(hipMalloc(&out4, (size_t)kBlocks * 512 * 16));
    const std::vector<float> a = dump<2, 2>(buf, x, out4, st);
    for (int v = 0; v < 5; ++v) {
      const std::vector<float> b = v == 0 ? dump<3, 2>(buf, x, out4, st) : v == 1 ? dump<3, 4>(buf, x, out4, st)
                                   : v == 2 ? dump<2, 4>(buf, x, out4, st) : v == 3 ? dump<8, 2>(buf, x, out4, st)
                                                                                    : dump<8, 4>(buf, x, out4, st);
      double md = 0, mx = 0;
      size_t nan = 0;
      for (size_t i = 0; i < a.size(); ++i) {
        if (!(b[i] == b[i])) ++nan;
        md = std::max(md, (double)std::abs(a[i] - b[i]));
        mx = std::max(mx, (double)std::abs(a[i]));
      }
      printf("check %s vs reg PD2: max |diff| %.3g of max |acc| %.3g, nan %zu\n",
             v == 0 ? "dma D2" : v == 1 ? "dma D4" : v == 2 ? "reg PD4" : v == 3 ? "engine D2" : "engine D4", md, mx, nan);
    }
    {  // the stream variants really read every word: their folds against the host's
      const std::vector<float> s0 = dump<0, 2>(buf, x, out4, st);
      std::vector<unsigned> hb(kSteps * kSB / 4);
      CK(hipMemcpy(hb.data(), buf, hb.size() * 4, hipMemcpyDeviceToHost));  // tile 0 (block 0, wave 0)
      // lane 0: q words at [s][h*1024 + 0..15], m words at [s][2048 + 8*(2h)] (r16 = 0, kq = 0)
      unsigned f = 0;
      for (int st2 = 0; st2 < kSteps; ++st2)
        for (int h = 0; h < 2; ++h) {
          const unsigned* q = &hb[(st2 * kSB + h * 1024) / 4];
          const unsigned* m = &hb[(st2 * kSB + 2048 + 16 * h) / 4];
          f ^= q[0] ^ q[1] ^ q[2] ^ q[3] ^ m[0] ^ m[1];
        }
      printf("check stream fold: device %.6g host %.6g\n", s0[0], (double)(float)f);
    }
    CK(hipFree(out4));
  }
  float* out16;
  CK(hipMalloc(&out16, kBlocks * 1024 * 4));
  {  // per-step stamps of the register ring (MODE 6): where a wave's time goes
    unsigned long long* stamps;
    const size_t n = (size_t)kBlocks * kWavesBusy * 34;
    CK(hipMalloc(&stamps, n * 8));
    CK(hipFuncSetAttribute((const void*)ring_kernel<6, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(6, 2)));
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL((ring_kernel<6, 2>), dim3(kBlocks), dim3(512), lds_of(6, 2), st, buf + (size_t)(rep % nreg) * region, x,
                         (float*)stamps, 2);
      CK(hipStreamSynchronize(st));
    }
    std::vector<unsigned long long> h(n);
    CK(hipMemcpy(h.data(), stamps, n * 8, hipMemcpyDeviceToHost));
    unsigned long long tmin = ~0ull, tmax = 0;
    double wait[kSteps] = {0}, comp[kSteps] = {0}, life = 0;
    const int nw = kBlocks * kWavesBusy;
    for (int w = 0; w < nw; ++w) {
      const unsigned long long* r = &h[(size_t)w * 34];
      tmin = std::min(tmin, r[0]);
      tmax = std::max(tmax, r[0] + r[1]);
      life += r[1];
      unsigned long long prev = 0;
      for (int s2 = 0; s2 < kSteps; ++s2) {
        wait[s2] += (double)(r[2 + 2 * s2] - prev);
        comp[s2] += (double)(r[3 + 2 * s2] - r[2 + 2 * s2]);
        prev = r[3 + 2 * s2];
      }
    }
    printf("stamps (s_memtime ticks = 100 MHz? see below): wave life avg %.0f, first-start..last-end %llu\n", life / nw, tmax - tmin);
    for (int s2 = 0; s2 < kSteps; ++s2) printf("  step %2d: wait %7.1f  compute %7.1f\n", s2, wait[s2] / nw, comp[s2] / nw);
    CK(hipFree(stamps));
  }
  const int iters = argc > 3 ? atoi(argv[3]) : 60;
  {  // one stream launch alone, timed by its own events, on a region no launch touched yet
    hipEvent_t a0, a1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    CK(hipFuncSetAttribute((const void*)ring_kernel<0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(0, 2)));
    for (int r = nreg - 3; r < nreg; ++r) {
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(a0, st));
      hipLaunchKernelGGL((ring_kernel<0, 2>), dim3(kBlocks), dim3(512), lds_of(0, 2), st, buf + (size_t)r * region, x, out, 0);
      CK(hipEventRecord(a1, st));
      CK(hipEventSynchronize(a1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a0, a1));
      printf("single cold stream launch (region %d): %.2f us\n", r, ms * 1e3);
    }
  }
  auto rep = [&](const char* name, double us) {
    printf("%-22s %8.2f us  %6.2f TB/s\n", name, us, bytes / us * 1e-6);
    fflush(stdout);
  };
  for (int rnd = 0; rnd < 2; ++rnd) {
    printf("-- round %d (%.1f MB per launch)\n", rnd, bytes * 1e-6);
    rep("stream PD2", run<0, 2>(buf, region, nreg, x, out, st, iters));
    rep("stream global PD2", run<7, 2>(buf, region, nreg, x, out, st, iters));
    rep("compute only", run<1, 2>(buf, region, nreg, x, out, st, iters));
    rep("reg PD2", run<2, 2>(buf, region, nreg, x, out, st, iters));
    rep("reg PD2 no waterfall", run<10, 2>(buf, region, nreg, x, out, st, iters));
    rep("reg PD3 no waterfall", run<10, 3>(buf, region, nreg, x, out, st, iters));
    rep("step-major reg PD2", run<9, 2>(buf, region, nreg, x, out, st, iters));
    rep("step-major reg PD3", run<9, 3>(buf, region, nreg, x, out, st, iters));
    {
      hipStream_t st2;
      CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
      float* o2;
      CK(hipMalloc(&o2, kBlocks * 512 * 4));
      rep("2-stream: stream only", run_concurrent(buf, region, nreg, x, out, o2, st, st2, iters, 1));
      rep("2-stream: compute only", run_concurrent(buf, region, nreg, x, out, o2, st, st2, iters, 2));
      rep("2-stream: both", run_concurrent(buf, region, nreg, x, out, o2, st, st2, iters, 3));
      CK(hipFree(o2));
    }
    rep("reg PD2 half dequant", run<4, 2>(buf, region, nreg, x, out, st, iters));
    rep("16 waves reg PD2", run16<2>(buf, region, nreg, x, (float*)nullptr == nullptr ? out16 : out16, st, iters));
    rep("reg PD3", run<2, 3>(buf, region, nreg, x, out, st, iters));
    rep("reg PD4", run<2, 4>(buf, region, nreg, x, out, st, iters));
    rep("engine D2", run<8, 2>(buf, region, nreg, x, out, st, iters));
    rep("engine D3", run<8, 3>(buf, region, nreg, x, out, st, iters));
    rep("dma D2", run<3, 2>(buf, region, nreg, x, out, st, iters));
    rep("dma D3", run<3, 3>(buf, region, nreg, x, out, st, iters));
    rep("dma D4", run<3, 4>(buf, region, nreg, x, out, st, iters));
  }
  CK(hipFree(buf));
  CK(hipFree(x));
  CK(hipFree(out));
  return 0;
}
