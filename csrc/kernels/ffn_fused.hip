// Fused decode FFN: RMSNorm -> gate/up GEMV + SwiGLU -> down GEMV + residual,
// ONE launch instead of two (replaces upstream's
// rms_norm + mul + 2x mul_mat_vec_q + silu + mul + mul_mat_vec_q + add chain).
//
// Status: correct (tests/test_engine_gpu.py::test_fused_ffn_matches_unfused), OPT-IN via
// LFK_FFN_FUSED=1. At Llama-3-8B shapes on MI355X one fused launch took 31-33 us against
// 29-30 us for the two separate launches: the hand-off (sc1 drain ~2 us, then a fan-in
// poll that sees the last producer 2-4 us late under the chip-wide weight stream) costs
// what the boundary and the down kernel's x prologue cost.
//
// Why it was tried: a batch-1 decode GEMV launch pays ~1.3-1.7 us of kernel boundary plus a
// 2-3 us x prologue whose loads queue behind the chip-wide weight burst
// (tools/gemv_chain_timeline.py). Here the down projection's dependency on the
// SwiGLU output is a PARTIAL one - its split-K part kp only needs the 2048
// features h[kp*2048 .. +2048) - so it is carried by per-slice arrival counters
// inside the launch, and each wave issues its first down-projection weight
// loads BEFORE it waits for its slice: the weight stream runs across the seam.
//
// Geometry: one 1024-thread workgroup per CU (pinned by an LDS request above
// half of the 160 KiB), grid = CU count, so every workgroup is resident and a
// wait can never block a producer from being scheduled. Phase A (gate/up) and
// phase B (down) items are split into contiguous per-workgroup ranges.
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16, write-through form):
//   producer: h stored with sc1 (agent-scope relaxed atomic stores), every
//             storing wave drains vmcnt, workgroup barrier, ONE lane adds 1 to
//             the slice counter (agent-scope relaxed atomic);
//   consumer: ONE lane polls the counter (relaxed agent loads, s_sleep, bounded:
//             a timeout sets *err instead of hanging), barrier, then every load
//             of h is an sc1 load.
// Phase B adds into the residual x, which phase A's prologue reads: a second
// counter (prologues done) must reach the grid size before the first add.
// Counters of layer l are zeroed by the launch of the NEXT layer (the previous
// launch has completed at a kernel boundary), so replays need no memset node.
#include "gemv_dev.h"

namespace lfk {

static constexpr int kFfnSliceF = 2048;  // features per down split-K part (64 chunks of 32)
static constexpr int kSpinLimit = 1 << 20;
static constexpr size_t kOnePerCuLdsFfn = 80 * 1024 + 256;  // > half of the CU's LDS: one workgroup per CU

__device__ __forceinline__ int ld_acq_i32(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1_f(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded poll by the calling lane; returns false (and flags *err) on timeout
__device__ __forceinline__ bool wait_geq(const int* ctr, int target, int* err, int code) {
  for (int spins = 0; ld_acq_i32(ctr) < target; ++spins) {
    if (spins > kSpinLimit) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

template <int QG, int QD>
__global__ __launch_bounds__(1024) void ffn_fused_kernel(FfnFusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NR = 4, NF = 2, WPB = 16;
  const int d = a.w_gu.K, F = a.F;
  const int G = gridDim.x, b = blockIdx.x;
  const int wave = wave_id(), lane = threadIdx.x & 63;
  // LDS: phase A x (d int8 + d/32 f32 + red), then phase B h (F int8 + F/32 f32)
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + d);
  float* red = xd + (d >> 5);
  int& s_flag = *reinterpret_cast<int*>(red + 16);   // in the dynamic region (no static LDS: Guideline 17)
  int8_t* hq = reinterpret_cast<int8_t*>(smem + ((d + (d >> 5) * 4 + 128 + 15) & ~15));
  float* hd = reinterpret_cast<float*>(reinterpret_cast<char*>(hq) + F);

  // stamps (dbg_clk, microbenchmarks): entry, prologue, phase A done, published, waits done,
  // h in LDS, exit
  long long* tl = a.dbg_clk ? a.dbg_clk + (size_t)b * 8 : nullptr;
#define LFK_FT(i) do { if (tl && threadIdx.x == 0) tl[i] = wall_clock64(); } while (0)
  LFK_FT(0);
  int* ctr = a.counters;            // [nslice] slice arrivals, [31] prologues done
  const int nslice = (F + kFfnSliceF - 1) / kFfnSliceF;
  if (b == 0 && threadIdx.x < 32 && a.counters_clear) a.counters_clear[threadIdx.x] = 0;

  // ---- phase A: gate/up + SwiGLU over items [a0, a1)
  const int NA = F / NF;
  const int perA = (NA + G - 1) / G;
  const int a0 = min(NA, b * perA), a1 = min(NA, a0 + perA);
  GemvArgs ga;
  ga.w = a.w_gu; ga.n_out = F;
  const int groupsA = NA;
  XPrologue<true, 1024> xp;
  xp.load(a.x, a.norm_w, d);
  RowPtr R[NR];
  int slot = 0, f0 = 0;
  WStream<QG, NR, 1> ws;
  int item = a0 + wave;
  {
    const int it0 = min(item, NA - 1);
    item_rows<EPI_SWIGLU, NR>(ga, it0, groupsA, R, slot, f0);
    ws.load(R, 0, d >> 5, lane);
  }
  const float xs = xp.finish(a.x, a.norm_w, a.eps, d, xq, xd, red);
  LFK_FT(1);
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr + 31, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nchA = d >> 5;
  while (item < a1) {
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    ws.finish_rows(R, nchA, xq, xd, acc, lane);
    const int cf = f0;
    const int next = item + WPB;
    if (next < a1) {
      item_rows<EPI_SWIGLU, NR>(ga, next, groupsA, R, slot, f0);
      ws.load(R, 0, nchA, lane);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] *= xs;
    const float v = reduce_rows<NR>(acc, lane);
    const float u = __shfl(v, (lane + NF) & 63);
    if (lane < NF) st_sc1_f(a.h + cf + lane, silu(v) * u);
    item = next;
  }

  LFK_FT(2);
  // ---- phase B setup: this workgroup's down items [b0, b1), kp-major
  const int RG = a.w_down.rows / NR;       // row groups of 4
  const int NB = RG * nslice;
  const int perB = (NB + G - 1) / G;
  const int b0 = min(NB, b * perB), b1 = min(NB, b0 + perB);
  const int nchB = F >> 5;
  WStream<QD, NR, 1> wd;
  RowPtr RD[NR];
  int jb = b0 + wave;
  auto rows_of = [&](int j, int& kp) {
    kp = j / RG;
    const int rg = j - kp * RG;
#pragma unroll
    for (int r = 0; r < NR; ++r) RD[r] = row_ptr(a.w_down.base, a.w_down.P, (unsigned)min(rg * NR + r, a.w_down.rows - 1));
    return rg;
  };
  // ---- publish this workgroup's h (phase A) to its slice counters. The drain
  // comes BEFORE the phase-B weight prefetch: loads and stores share vmcnt on
  // gfx9, so a drain behind the prefetch would wait for the weights too.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0 && a0 < a1) {
    const int s_lo = (a0 * NF) / kFfnSliceF, s_hi = ((a1 - 1) * NF) / kFfnSliceF;
    for (int s = s_lo; s <= s_hi; ++s) __hip_atomic_fetch_add(ctr + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  LFK_FT(3);
  int kp = 0, rg = 0;
  if (b0 < b1) {  // prefetch the first down item's weights before any wait
    rg = rows_of(min(jb, b1 - 1), kp);
    wd.load(RD, kp * 64, nchB, lane);
  }
  if (b0 >= b1) return;

  // ---- phase B: wait for the slices this workgroup reads, then h -> q8 in LDS
  const int kp_lo = b0 / RG, kp_hi = (b1 - 1) / RG;
  if (threadIdx.x == 0) {
    int ok = 1;
    for (int s = kp_lo; s <= kp_hi && ok; ++s) {
      // producers of slice s: workgroups whose phase-A range meets its items
      const int i_lo = s * (kFfnSliceF / NF), i_hi = min(NA, (s + 1) * (kFfnSliceF / NF)) - 1;
      const int target = i_hi / perA - i_lo / perA + 1;
      ok = wait_geq(ctr + s, target, a.err, 1 + s);
    }
    if (ok) ok = wait_geq(ctr + 31, G, a.err, 64);
    s_flag = ok;
  }
  __syncthreads();
  LFK_FT(4);
  if (!s_flag) return;
  {
    // (kp_hi - kp_lo + 1) <= 2 slices of 2048 features: 512 threads x 4 features per slice
    const int t = threadIdx.x;
    for (int s = kp_lo + (t >> 9); s <= kp_hi; s += 2) {
      const int i = s * kFfnSliceF + (t & 511) * 4;
      if (i < F) {
        float4 v;
        v.x = ld_sc1_f(a.h + i); v.y = ld_sc1_f(a.h + i + 1); v.z = ld_sc1_f(a.h + i + 2); v.w = ld_sc1_f(a.h + i + 3);
        const float amax = max8(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        const float dsc = amax * (1.f / 127.f);
        const float id = dsc > 0.f ? 1.f / dsc : 0.f;
        const int q0 = __float2int_rn(v.x * id), q1 = __float2int_rn(v.y * id);
        const int q2 = __float2int_rn(v.z * id), q3 = __float2int_rn(v.w * id);
        *reinterpret_cast<int*>(hq + i) = (q0 & 0xFF) | ((q1 & 0xFF) << 8) | ((q2 & 0xFF) << 16) | ((q3 & 0xFF) << 24);
        if ((t & 7) == 0) hd[i >> 5] = dsc;
      }
    }
  }
  __syncthreads();
  LFK_FT(5);
  while (jb < b1) {
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    wd.dot(kp * 64, nchB, hq, hd, acc, lane);
    const int crg = rg;
    const int next = jb + WPB;
    if (next < b1) {
      rg = rows_of(next, kp);
      wd.load(RD, kp * 64, nchB, lane);
    }
    const float v = reduce_rows<NR>(acc, lane);
    if (lane < NR && crg * NR + lane < a.w_down.rows) atomicAdd(a.x + crg * NR + lane, v);
    jb = next;
  }
  LFK_FT(6);
#undef LFK_FT
}

static size_t ffn_lds(int d, int F) {
  const size_t a = (size_t)((d + (d >> 5) * 4 + 128 + 15) & ~15);
  const size_t need = a + F + (size_t)(F >> 5) * 4 + 16;
  return need > kOnePerCuLdsFfn ? need : kOnePerCuLdsFfn;
}

template <int QG, int QD>
static bool ffn_launch(const FfnFusedArgs& a, hipStream_t s, bool probe) {
  auto k = ffn_fused_kernel<QG, QD>;
  const size_t lds = ffn_lds(a.w_gu.K, a.F);
  if (probe) {
    // every workgroup must be resident: exactly one per CU, grid = CU count
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 1024, lds) != hipSuccess) return false;
    return per_cu == 1 && cus > 0;
  }
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipLaunchKernelGGL(k, dim3(cus), dim3(1024), lds, s, a);
  return true;
}

static bool ffn_dispatch(const FfnFusedArgs& a, hipStream_t s, bool probe) {
  const int tg = a.w_gu.type, td = a.w_down.type;
  if (tg == T_Q4_K && td == T_Q4_K) return ffn_launch<T_Q4_K, T_Q4_K>(a, s, probe);
  if (tg == T_Q4_K && td == T_Q6_K) return ffn_launch<T_Q4_K, T_Q6_K>(a, s, probe);
  if (tg == T_Q4_K && td == T_Q5_K) return ffn_launch<T_Q4_K, T_Q5_K>(a, s, probe);
  if (tg == T_Q8_0 && td == T_Q8_0) return ffn_launch<T_Q8_0, T_Q8_0>(a, s, probe);
  // other mixes (Q5_K/Q6_K gate-up) exceed 128 VGPRs at 1024 threads: unfused path
  return false;
}

bool ffn_fused_supported(const FfnFusedArgs& a) {
  if (a.w_gu.K % 256 || a.F % 32 || a.w_gu.rows != 2 * a.F || a.w_down.K != a.F) return false;
  if (a.w_gu.K > 16384) return false;                      // one-batch x prologue (XPrologue<., 1024>)
  if ((a.F + kFfnSliceF - 1) / kFfnSliceF > 31) return false;  // counter slots
  if (ffn_lds(a.w_gu.K, a.F) > 160 * 1024) return false;
  // opt-in (LFK_FFN_FUSED=1): measured on MI355X at Llama-3-8B shapes it is not faster than
  // the two launches it replaces - the sc1 drain (~2 us) and the fan-in poll under a saturated
  // weight stream (~3 us) cost what the kernel boundary + x prologue did (tools/ffn_fused_timeline.py)
  const char* e = getenv("LFK_FFN_FUSED");
  if (!e || e[0] != '1') return false;
  return ffn_dispatch(a, nullptr, true);
}

void ffn_fused(const FfnFusedArgs& a, hipStream_t s) {
  if (!ffn_dispatch(a, s, false)) throw std::runtime_error("ffn_fused: unsupported weight types");
}

}  // namespace lfk
