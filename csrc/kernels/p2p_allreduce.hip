// One-shot push collectives for tensor-parallel messages (SURVEY §2.4 X7, §2.6 N0c,
// §5.8): the two per-layer all-reduces of a row-parallel decode step carry 16-32 KiB
// per row, where a ring all-reduce is latency-bound (2(N-1) dependent steps). Here
// every rank WRITES its buffer straight into every peer's receive slot over its
// point-to-point xGMI link (7 links used at once on an 8-GPU node), raises one flag
// per (rank, block) in each peer, then waits for the N flags in its OWN memory and
//   * all-reduce: sums the N slots locally in fixed rank order - every rank computes
//     bit-identical results (the TP ranks must stay in lock-step), or
//   * all-gather: copies slot p to dst[p * n ...] (the sampler's candidate blocks,
//     logit shards for the test hooks).
//
// Receive regions are exported/imported once with hipIpc* handles (one process per
// GPU, or several processes on one GPU in the IPC-only test mode); the kernel is
// graph-capturable: the epoch lives in device memory and advances on every launch.
//
// Slot reuse needs no second barrier because EVERY launch uses the same fixed grid
// (kP2PMaxBlocks blocks, whatever n is): all blocks share one epoch sequence, slot
// parity alternates per launch, and a rank writes parity e&1 again at epoch e+2 only
// after it saw every peer's flags of epoch e+1 - raised by a peer's launch e+1, which
// started after that peer's launch e (and its reads of the slot) completed (stream
// order). A per-launch block count would break this: blocks of different launches
// would advance different epochs and alias slot ranges.
//
// Memory model (why a peer's bytes are never read stale, across xGMI or on one GPU):
//   * the receive region is allocated hipDeviceMallocUncached (runtime/p2p.cpp): no L2 /
//     L1 of the owning GPU or of a writing peer keeps a line of it, so every store lands in
//     the owner's HBM and every load reads HBM - there is no previous-epoch line to hit;
//   * payload stores are plain (vectorised) stores into the peer's region, ordered before
//     the flag stores by a system-scope release fence + block barrier (the fence waits for
//     the stores to be acknowledged by the peer's memory);
//   * the reader polls its LOCAL flags with system-scope acquire loads and reads the slots
//     with system-scope loads; on a cacheable fallback region (hipMalloc, if the uncached
//     allocation is refused) the system scope still bypasses the non-coherent caches.
// Slot reuse (a rank overwriting a slot a slower peer still reads) is excluded by the epoch
// argument above.
// Every wait is bounded: a timeout sets *err and the launch completes (the engine
// then reports itself unhealthy) instead of hanging.
#include "kernels.h"

namespace lfk {

static constexpr int kP2PSpin = 1 << 22;

__device__ __forceinline__ float ld_sys(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void p2p_collective_kernel(P2PArgs a) {
  __shared__ int s_ep, s_ok;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int W = a.world, R = a.rank;
  const int chunk = ((a.n + kP2PMaxBlocks - 1) / kP2PMaxBlocks + 3) & ~3;
  const int i0 = min(a.n, b * chunk), i1 = min(a.n, i0 + chunk);
  if (tid == 0) {
    const int e = a.epochs[b] + 1;  // block-private word: plain access
    a.epochs[b] = e;
    s_ep = e;
    s_ok = 1;
  }
  __syncthreads();
  const int ep = s_ep, slot = ep & 1;
  const size_t FB = kP2PMaxBlocks;
  // 1. push this rank's chunk into slot [slot][R] of every rank (self included)
  const bool vec = ((reinterpret_cast<uintptr_t>(a.src) & 15) == 0) && (a.max_n % 4 == 0);
  const int v0 = i0, v1 = vec ? i0 + ((i1 - i0) & ~3) : i0;
  for (int p = 0; p < W; ++p) {
    float* dst = a.peers.data[p] + ((size_t)slot * W + R) * a.max_n;
    for (int i = v0 + 4 * tid; i < v1; i += 4 * blockDim.x)
      *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(a.src + i);
    for (int i = v1 + tid; i < i1; i += blockDim.x) dst[i] = a.src[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this thread's stores before the barrier
  __syncthreads();
  // 2. one flag per (slot, rank, block) in every rank
  if (tid < W)
    __hip_atomic_store(a.peers.flags[tid] + ((size_t)slot * W + R) * FB + b, ep, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every rank's flag in this rank's own region
  if (tid < W) {
    const int* f = a.peers.flags[R] + ((size_t)slot * W + tid) * FB + b;
    for (int spins = 0; __hip_atomic_load(const_cast<int*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < ep;
         ++spins) {
      if (spins > kP2PSpin) {
        __hip_atomic_store(a.err, 100 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (!s_ok) return;
  const float* mine = a.peers.data[R] + (size_t)slot * W * a.max_n;
  if (a.gather) {
    // 4a. rank p's chunk -> dst[p * n + i]
    for (int p = 0; p < W; ++p)
      for (int i = i0 + tid; i < i1; i += blockDim.x) a.dst[(size_t)p * a.n + i] = ld_sys(mine + (size_t)p * a.max_n + i);
    return;
  }
  // 4b. sum the W slots in rank order (bit-identical on every rank)
  for (int i = i0 + tid; i < i1; i += blockDim.x) {
    float v = 0.f;
    for (int p = 0; p < W; ++p) v += ld_sys(mine + (size_t)p * a.max_n + i);
    a.dst[i] = v;
  }
}

void p2p_collective(const P2PArgs& a, hipStream_t s) {
  if (a.world < 1 || a.world > kP2PMaxRanks) throw std::runtime_error("p2p: world must be 1..8");
  if (a.n <= 0) return;
  if (a.n > a.max_n) throw std::runtime_error("p2p: message larger than the slot");
  hipLaunchKernelGGL(p2p_collective_kernel, dim3(kP2PMaxBlocks), dim3(256), 0, s, a);
}

}  // namespace lfk
