// One-shot push all-reduce for decode-sized tensor-parallel messages (SURVEY
// §2.4 X7, §2.6 N0c, §5.8): the two per-layer all-reduces of a row-parallel
// decode step carry 16-32 KiB, where a ring all-reduce is latency-bound
// (2(N-1) dependent steps over a ring). Here every rank WRITES its partial
// straight into every peer's receive slot over its point-to-point xGMI link
// (7 links used at once on an 8-GPU node), raises one flag per (rank, block)
// in each peer, then waits for the N flags in its OWN memory and sums the N
// slots locally in fixed rank order - so every rank computes bit-identical
// results (the TP ranks must stay in lock-step).
//
// Receive regions are exported/imported once with hipIpc* handles (one process
// per GPU); the kernel is graph-capturable: the epoch (per block) lives in
// device memory and advances on every launch, and slots alternate with the
// epoch's parity. Slot reuse is safe without a second barrier: a rank writes
// slot s again at epoch e+2 only after it saw every peer's flag for e+1, which
// each peer raised after finishing its reads of epoch e (stream order).
//
// Memory model: data and flags are stored with system-scope atomics (write-
// through, visible to the peer agent), a system-scope release fence orders
// each thread's data stores before the block barrier and the flag stores;
// the reader polls its local flags with system-scope acquire loads and reads
// the slots with system-scope loads (bypassing an L2 that may hold the slot's
// previous epoch). Every wait is bounded: a timeout sets *err and the launch
// completes (the engine then reports itself unhealthy) instead of hanging.
#include "kernels.h"

namespace lfk {

static constexpr int kP2PSpin = 1 << 22;

__device__ __forceinline__ void st_sys(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void p2p_allreduce_kernel(P2PAllreduceArgs a) {
  __shared__ int s_ep, s_ok;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int W = a.world, R = a.rank;
  const int chunk = ((a.n + gridDim.x - 1) / gridDim.x + 3) & ~3;
  const int i0 = b * chunk, i1 = min(a.n, i0 + chunk);
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
  for (int p = 0; p < W; ++p) {
    float* dst = a.peers.data[p] + ((size_t)slot * W + R) * a.max_n;
    for (int i = i0 + tid; i < i1; i += blockDim.x) st_sys(dst + i, a.src[i]);
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
  // 4. sum the W slots in rank order (bit-identical on every rank)
  const float* mine = a.peers.data[R] + (size_t)slot * W * a.max_n;
  for (int i = i0 + tid; i < i1; i += blockDim.x) {
    float v = 0.f;
    for (int p = 0; p < W; ++p) v += ld_sys(mine + (size_t)p * a.max_n + i);
    a.dst[i] = v;
  }
}

void p2p_allreduce(const P2PAllreduceArgs& a, hipStream_t s) {
  if (a.world < 1 || a.world > kP2PMaxRanks) throw std::runtime_error("p2p_allreduce: world must be 1..8");
  if (a.n <= 0) return;
  if (a.n > a.max_n) throw std::runtime_error("p2p_allreduce: message larger than the slot");
  const int blocks = a.blocks > 0 ? a.blocks : 1;
  if (blocks > kP2PMaxBlocks) throw std::runtime_error("p2p_allreduce: too many blocks");
  hipLaunchKernelGGL(p2p_allreduce_kernel, dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace lfk
