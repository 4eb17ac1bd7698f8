// K/V load-shape microbenchmark for the batched decode attention (B = 6 rows x 8 kv heads,
// L = 700 keys, head_dim 128, f16 K and V): how fast does the chip pull one layer's 17 MB of
// K/V when
//   split : every (row, kv head) is cut into 64-key chunks, one 256-thread block per chunk
//           (the production attn_decode grid: 528 blocks, 32 KB each), vs
//   whole : ONE block per (row, kv head) reads all of its L keys (48 blocks of 1024 threads,
//           358 KB each; no cross-block merge would be needed), its waves issuing every load
//           up front, vs
//   whole2: two blocks per (row, kv head) (96 blocks, 179 KB each).
// Each launch reads a fresh KV region (layers rotated over 1.2 GB). Loads only (XOR-folded).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/attn_load_bench tools/attn_load_bench.hip && /tmp/attn_load_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kB = 6, kKV = 8, kL = 700, kCtx = 1024, kHD = 128;
constexpr size_t kRowBytes = kHD * 2;                               // one key's K (or V) row
constexpr size_t kSlotBytes = (size_t)kKV * kCtx * kRowBytes;       // one slot's K (or V) of a layer
constexpr size_t kLayerBytes = 2 * kB * kSlotBytes;                 // K and V of B slots

typedef unsigned u4 __attribute__((ext_vector_type(4)));

// split: block (kvh, chunk, row), 256 threads: lane = (key lane / 4, quarter lane % 4) as production
__global__ __launch_bounds__(256) void split_kernel(const unsigned char* base, unsigned* out) {
  const int kvh = blockIdx.x, chunk = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int key = min(chunk * 64 + wave * 16 + (lane >> 2), kL - 1);
  const unsigned char* k = base + (size_t)b * kSlotBytes + ((size_t)kvh * kCtx + key) * kRowBytes + (lane & 3) * 64;
  const unsigned char* v = k + (size_t)kB * kSlotBytes;
  u4 acc = {0, 0, 0, 0};
  u4 r[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(k) + i);
#pragma unroll
  for (int i = 0; i < 4; ++i) r[4 + i] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(v) + i);
#pragma unroll
  for (int i = 0; i < 8; ++i) acc ^= r[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[tid] = acc.x;
}

// whole: NB blocks per (row, kv head), 1024 threads; wave w takes 64-key chunks w, w + 16, ... of its
// block's key range; all of a wave's loads go out before any use (<= CPW chunks per wave)
template <int NB, int CPW>
__global__ __launch_bounds__(1024) void whole_kernel(const unsigned char* base, unsigned* out) {
  const int kvh = blockIdx.x, part = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int per = (kL + NB - 1) / NB, k0 = part * per, k1 = min(kL, k0 + per);
  u4 acc = {0, 0, 0, 0};
  u4 r[CPW][2][4];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    // chunk of 16 keys: wave w, pass c -> keys k0 + (c * 16 + w) * 16 + lane / 4
    const int key = min(k0 + (c * 16 + wave) * 16 + (lane >> 2), k1 - 1);
    const unsigned char* k = base + (size_t)b * kSlotBytes + ((size_t)kvh * kCtx + key) * kRowBytes + (lane & 3) * 64;
    const unsigned char* v = k + (size_t)kB * kSlotBytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[c][0][i] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(k) + i);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[c][1][i] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(v) + i);
  }
#pragma unroll
  for (int c = 0; c < CPW; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= r[c][0][i] ^ r[c][1][i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[tid] = acc.x;
}

template <typename F>
static double timeit(F launch, int nreg, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < nreg; ++i) launch(i);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) launch(i % nreg);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / iters;
}

int main() {
  const int nreg = 32;  // layers
  unsigned char* buf;
  unsigned* out;
  CK(hipMalloc(&buf, kLayerBytes * nreg));
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMemset(buf, 0x3c, kLayerBytes * nreg));
  const double mb = 2.0 * kB * kKV * kL * kRowBytes * 1e-6;
  printf("K/V bytes per launch (B %d, L %d): %.1f MB; region per layer %.1f MB x %d\n", kB, kL, mb, kLayerBytes * 1e-6, nreg);
  for (int rnd = 0; rnd < 2; ++rnd) {
    const double t0 = timeit([&](int i) {
      hipLaunchKernelGGL(split_kernel, dim3(kKV, (kL + 63) / 64, kB), dim3(256), 0, 0, buf + (size_t)i * kLayerBytes, out);
    }, nreg, 64);
    printf("split  (528 blocks x 32 KB)        %7.2f us  %5.2f TB/s\n", t0, mb / t0);
    const double t1 = timeit([&](int i) {
      hipLaunchKernelGGL((whole_kernel<1, 3>), dim3(kKV, 1, kB), dim3(1024), 0, 0, buf + (size_t)i * kLayerBytes, out);
    }, nreg, 64);
    printf("whole  (48 blocks x 358 KB)        %7.2f us  %5.2f TB/s\n", t1, mb / t1);
    const double t2 = timeit([&](int i) {
      hipLaunchKernelGGL((whole_kernel<2, 2>), dim3(kKV, 2, kB), dim3(1024), 0, 0, buf + (size_t)i * kLayerBytes, out);
    }, nreg, 64);
    printf("whole2 (96 blocks x 179 KB)        %7.2f us  %5.2f TB/s\n", t2, mb / t2);
    const double t3 = timeit([&](int i) {
      hipLaunchKernelGGL((whole_kernel<4, 1>), dim3(kKV, 4, kB), dim3(1024), 0, 0, buf + (size_t)i * kLayerBytes, out);
    }, nreg, 64);
    printf("whole4 (192 blocks x 90 KB)        %7.2f us  %5.2f TB/s\n", t3, mb / t3);
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
