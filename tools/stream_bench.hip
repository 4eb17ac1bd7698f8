// HBM streaming microbenchmark for the batched decode projections' weight stream (bmm.hip's
// wave-owned gate/up: 256 blocks x 7 busy waves, each wave one tile16 tile = 16 contiguous
// 2560-B steps, PD steps in flight per wave). Which access pattern / depth reaches what rate on
// this chip, with nothing computed: the loaded words are XOR-folded into one register.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/stream_bench tools/stream_bench.hip && build/stream_bench
//
// Patterns (bytes per launch = the gate/up's 1792 tiles x 16 steps x 2560 B = 73.4 MB):
//   tile   the bmm layout: wave-owned contiguous tiles ([tile][step]), 2 x 1 KB 16-B/lane quant
//          loads + 2 x 512 B 8-B/lane scale loads per step
//   step   step-major ([step][tile]): at step s all waves read one contiguous 4.6 MB band
//   seq    one contiguous 287 KB range per block, the block's waves taking 1 KB pieces in turn
// Times are per launch, back to back on one stream (each includes one ~1.5 us kernel boundary).
// Each launch reads a fresh region of a 1.5 GiB buffer (the 256 MB Infinity Cache holds none).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kTiles = 1792, kSteps = 16, kSB = 2560, kWavesBusy = 7, kBlocks = 256;

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const unsigned char* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else return *reinterpret_cast<const u32x4*>(p);
}

struct Raw {
  u32x4 q0, q1;
  u32x2 m0, m1;
};

// pattern 0 = tile, 1 = step-major, 2 = seq (per-block contiguous)
template <int PAT>
__device__ __forceinline__ const unsigned char* step_ptr(const unsigned char* base, int tile, int s, int wave, int blk) {
  if constexpr (PAT == 0) return base + ((size_t)tile * kSteps + s) * kSB;
  else if constexpr (PAT == 1) return base + ((size_t)s * kTiles + tile) * kSB;
  else return base + (size_t)blk * kWavesBusy * kSteps * kSB + ((size_t)s * kWavesBusy + wave) * kSB;
}

template <int PAT, int PD, bool NT>
__global__ __launch_bounds__(512, 1) void stream_kernel(const unsigned char* base, unsigned* out) {
  constexpr int R = PD + 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, blk = blockIdx.x;
  if (wave >= kWavesBusy) return;
  const int tile = blk * kWavesBusy + wave, r16 = lane & 15, kq = lane >> 4;
  Raw buf[R];
  auto load = [&](Raw& b, int s) {
    const unsigned char* p = step_ptr<PAT>(base, tile, s, wave, blk);
    b.q0 = ld16<NT>(p + lane * 16);
    b.q1 = ld16<NT>(p + 1024 + lane * 16);
    b.m0 = *reinterpret_cast<const u32x2*>(p + 2048 + r16 * 32 + 8 * (kq >> 1));
    b.m1 = *reinterpret_cast<const u32x2*>(p + 2048 + r16 * 32 + 8 * (2 + (kq >> 1)));
  };
  unsigned acc = 0;
#pragma unroll
  for (int p = 0; p < PD; ++p) load(buf[p], p);
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    if (s + PD < kSteps) load(buf[(s + PD) % R], s + PD);
    const Raw& b = buf[s % R];
    acc ^= b.q0.x ^ b.q0.y ^ b.q0.z ^ b.q0.w ^ b.q1.x ^ b.q1.y ^ b.q1.z ^ b.q1.w ^ b.m0.x ^ b.m0.y ^ b.m1.x ^ b.m1.y;
  }
  if (acc == 0x9e3779b9u) out[blk * 512 + threadIdx.x] = acc;
}

template <int PAT, int PD, bool NT>
static double run(const unsigned char* buf, size_t region, int nreg, unsigned* out, hipStream_t st, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < nreg; ++i) hipLaunchKernelGGL((stream_kernel<PAT, PD, NT>), dim3(kBlocks), dim3(512), 0, st, buf + i * region, out);
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((stream_kernel<PAT, PD, NT>), dim3(kBlocks), dim3(512), 0, st, buf + (i % nreg) * region, out);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3 / iters;  // us per launch
}

int main() {
  const size_t bytes = (size_t)kTiles * kSteps * kSB;  // 73.4 MB
  const size_t region = (bytes + 4095) / 4096 * 4096;
  const int nreg = 20;                                  // 1.47 GB rotated
  unsigned char* buf;
  unsigned* out;
  CK(hipMalloc(&buf, region * nreg));
  CK(hipMalloc(&out, kBlocks * 512 * 4));
  CK(hipMemset(buf, 0x5a, region * nreg));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int iters = 60;
  auto rep = [&](const char* name, double us) {
    printf("%-22s %8.2f us  %6.2f TB/s\n", name, us, bytes / us * 1e-6);
    fflush(stdout);
  };
  for (int rnd = 0; rnd < 2; ++rnd) {
    printf("-- round %d (%.1f MB per launch)\n", rnd, bytes * 1e-6);
    rep("tile  PD1 nt", run<0, 1, true>(buf, region, nreg, out, st, iters));
    rep("tile  PD2 nt", run<0, 2, true>(buf, region, nreg, out, st, iters));
    rep("tile  PD3 nt", run<0, 3, true>(buf, region, nreg, out, st, iters));
    rep("tile  PD4 nt", run<0, 4, true>(buf, region, nreg, out, st, iters));
    rep("tile  PD6 nt", run<0, 6, true>(buf, region, nreg, out, st, iters));
    rep("tile  PD2 plain", run<0, 2, false>(buf, region, nreg, out, st, iters));
    rep("tile  PD4 plain", run<0, 4, false>(buf, region, nreg, out, st, iters));
    rep("step  PD2 nt", run<1, 2, true>(buf, region, nreg, out, st, iters));
    rep("step  PD4 nt", run<1, 4, true>(buf, region, nreg, out, st, iters));
    rep("seq   PD2 nt", run<2, 2, true>(buf, region, nreg, out, st, iters));
    rep("seq   PD4 nt", run<2, 4, true>(buf, region, nreg, out, st, iters));
    rep("seq   PD6 nt", run<2, 6, true>(buf, region, nreg, out, st, iters));
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
