// One-shot push collectives for tensor-parallel messages (SURVEY §2.4 X7, §2.6 N0c,
// §5.8): the two per-layer all-reduces of a row-parallel decode step carry 16-32 KiB
// per row, where a ring all-reduce is latency-bound (2(N-1) dependent steps). Here
// every rank WRITES its buffer straight into every peer's receive slot over its
// point-to-point xGMI link (7 links used at once on an 8-GPU node) as 8-byte granules
// {value, epoch}, and reads its OWN slots until every granule carries this launch's epoch:
//   * all-reduce: sums the N slots locally in fixed rank order - every rank computes
//     bit-identical results (the TP ranks must stay in lock-step), or
//   * all-gather: copies slot p to dst[p * n ...] (the sampler's candidate blocks,
//     logit shards for the test hooks).
// The data carries its own readiness (the LL form of a hand-off, MI355X_MICROARCH "granule"):
// no release fence behind the payload, no flag store, no flag poll before the payload reads -
// one memory round trip per element instead of store -> fence -> flag -> poll -> load (the
// round-3 form measured ~10 us per 2-rank collective on one GPU).
//
// Receive regions are exported/imported once with hipIpc* handles (one process per
// GPU, or several processes on one GPU in the IPC-only test mode); the kernel is
// graph-capturable: the epoch lives in device memory and advances on every launch.
//
// Slot reuse needs no second barrier because EVERY launch uses the same fixed grid
// (kP2PMaxBlocks blocks, whatever n is) and a block's chunk is fixed per n: all blocks
// advance one epoch sequence, slot parity alternates per launch, and rank R's block b writes
// parity e&1 again at epoch e+2 only after it received every peer's block-b granules of epoch
// e+1 - written by that peer's launch e+1, which started after the peer's launch e (and its
// block b's reads of parity e&1) completed (stream order). That needs every block to receive at
// least one granule from every peer in every launch, whatever n is: each block also exchanges
// one heartbeat granule of its own (index max_n + b of the slot). A granule of an older epoch is
// never taken for a newer one: the tag is the full 32-bit epoch.
//
// Memory model: the region is hipDeviceMallocUncached (runtime/p2p.cpp), so no L2 of either
// side keeps a line of it; each granule is one naturally aligned 8-byte system-scope atomic
// store (untorn: value and tag arrive together) and is read with 8-byte system-scope atomic
// loads. On a cacheable fallback region (hipMalloc, if the uncached allocation is refused) the
// system scope still bypasses the non-coherent caches.
// Every wait is bounded: a timeout sets *err, stores the rank's fault code into every rank's
// region (P2PPeers::fault) and the launch completes instead of hanging; every wait also polls
// the fault words between spins, so one rank's fault ends every rank's waits at once. A faulted
// group is poisoned: its outputs are stale from then on, every rank's engine reports the fault
// (check_device_err) and the leader refuses further steps.
#include "kernels.h"
#include "qdot.h"

namespace lfk {

// bounded waits, in wall_clock64 ticks (100 MHz): 20 s - ranks time-sliced on one GPU (the IPC
// rehearsal) can legitimately wait long for a peer's queue to run
static constexpr long long kP2PWaitTicks = 2000000000LL;

typedef unsigned long long u64_t;

__device__ __forceinline__ void p2p_collective_body(const P2PArgs& a) {
  __shared__ unsigned s_ep;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int W = a.world, R = a.rank;
  const int chunk = (a.n + kP2PMaxBlocks - 1) / kP2PMaxBlocks;
  const int i0 = min(a.n, b * chunk), i1 = min(a.n, i0 + chunk);
  if (tid == 0) {
    const int e = a.epochs[b] + 1;  // block-private word: plain access
    a.epochs[b] = e;
    s_ep = (unsigned)e;
  }
  __syncthreads();
  const unsigned ep = s_ep;
  const int slot = ep & 1;
  const size_t M = (size_t)a.stride;                   // granules per (slot, rank): data + heartbeats (+ fused)
  const int hb = a.max_n + b;                          // this block's heartbeat granule
  // 1. push this rank's chunk into slot [slot][R] of every rank (self included), then the block's
  //    heartbeat (last, so that a peer seeing it mostly finds the data there too)
  for (int i = i0 + tid; i < i1; i += blockDim.x) {
    const u64_t g = ((u64_t)ep << 32) | __float_as_uint(a.src[i]);
    if (a.accumulate) const_cast<float*>(a.src)[i] = 0.f;  // (this lane's own element, read above)
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      if (p < W)
        __hip_atomic_store(reinterpret_cast<u64_t*>(a.peers.data[p]) + ((size_t)slot * W + R) * M + i, g,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (tid < W)
    __hip_atomic_store(reinterpret_cast<u64_t*>(a.peers.data[tid]) + ((size_t)slot * W + R) * M + hb, (u64_t)ep << 32,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // 2. the block's heartbeats first - W lanes poll (sleeping between polls) while the rest of the
  //    block waits at the barrier, so a late peer costs polling traffic of W lanes per block, not
  //    of every lane (8 ranks sharing one GPU in the IPC rehearsal starved each other's queues)
  const u64_t* mine = reinterpret_cast<const u64_t*>(a.peers.data[R]) + (size_t)slot * W * M;
  __shared__ int s_ok;
  if (tid == 0) s_ok = 1;
  __syncthreads();
  if (tid < W) {
    const long long t0 = wall_clock64();
    for (int spins = 0;; ++spins) {
      const u64_t g = __hip_atomic_load(const_cast<u64_t*>(mine + (size_t)tid * M + hb), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM);
      if ((unsigned)(g >> 32) == ep) break;
      if ((spins & 255) == 255) {
        if (wall_clock64() - t0 > kP2PWaitTicks) {
          __hip_atomic_store(a.err, 100 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          p2p_raise(a.peers, W, R, 100 + tid);  // poison the group: every rank's waits end
          s_ok = 0;
          break;
        }
        if (p2p_poisoned(a.peers, W, R)) {  // some rank already failed: the group is dead
          s_ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (!s_ok) return;
  // 3. every rank's granule of each element, re-read (rarely) until it carries this epoch: the
  //    peer's data stores were issued before its heartbeat but may land after it
  for (int i = i0 + tid; i < i1; i += blockDim.x) {
    float v[kP2PMaxRanks];
    unsigned pending = (1u << W) - 1;
    const long long t0 = wall_clock64();
    for (int spins = 0; pending; ++spins) {
#pragma unroll
      for (int p = 0; p < kP2PMaxRanks; ++p) {
        if (p < W && (pending >> p & 1)) {
          const u64_t g = __hip_atomic_load(const_cast<u64_t*>(mine + (size_t)p * M + i), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM);
          if ((unsigned)(g >> 32) == ep) {
            v[p] = __uint_as_float((unsigned)g);
            pending &= ~(1u << p);
          }
        }
      }
      if (!pending) break;
      if ((spins & 255) == 255) {
        if (wall_clock64() - t0 > kP2PWaitTicks) {
          __hip_atomic_store(a.err, 100 + __builtin_ctz(pending), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          p2p_raise(a.peers, W, R, 100 + __builtin_ctz(pending));
          return;
        }
        if (p2p_poisoned(a.peers, W, R)) return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (a.gather) {
#pragma unroll
      for (int p = 0; p < kP2PMaxRanks; ++p)
        if (p < W) a.dst[(size_t)p * a.n + i] = v[p];
    } else {
      float sum = 0.f;  // rank order: bit-identical on every rank
#pragma unroll
      for (int p = 0; p < kP2PMaxRanks; ++p)
        if (p < W) sum += v[p];
      a.dst[i] = a.accumulate ? a.dst[i] + sum : sum;  // (dst identical on every rank: so is the result)
    }
  }
}

__global__ __launch_bounds__(256) void p2p_collective_kernel(P2PArgs a) {
  p2p_collective_body(a);
  // the fault words as this launch leaves them, mirrored to host-mapped memory (a fault a later
  // block raises is mirrored by the next launch)
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.fault_h) {
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      if (p < a.world)
        __hip_atomic_store(a.fault_h + p, __hip_atomic_load(a.peers.fault[a.rank] + p, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_SYSTEM),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

void p2p_collective(const P2PArgs& a, hipStream_t s) {
  if (a.world < 1 || a.world > kP2PMaxRanks) throw std::runtime_error("p2p: world must be 1..8");
  if (a.n <= 0) return;
  if (a.n > a.max_n) throw std::runtime_error("p2p: message larger than the slot");
  if (a.stride < a.max_n + kP2PMaxBlocks) throw std::runtime_error("p2p: slot stride");
  if (a.accumulate && a.gather) throw std::runtime_error("p2p: accumulate is an all-reduce mode");
  if (a.accumulate && a.src == a.dst) throw std::runtime_error("p2p: accumulate needs distinct src / dst");
  hipLaunchKernelGGL(p2p_collective_kernel, dim3(kP2PMaxBlocks), dim3(256), 0, s, a);
}

}  // namespace lfk
