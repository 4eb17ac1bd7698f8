// Host side of the one-shot P2P collectives: owns this rank's
// receive region (exported with a hipIpc handle) and the peers' imported
// regions; dispatches all-reduces and all-gathers of up to max_n floats to
// kernels/p2p_allreduce.hip. One process per GPU (or, in the IPC-only test mode,
// several per GPU): handles are exchanged by the caller (torch.distributed).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../kernels/kernels.h"

namespace lfk {

class P2PComm {
 public:
  // fused_n > 0: a further area of fused_n granules per (slot, rank) past the collective's, for
  // the GEMV epilogue all-reduce (gemv.hip, GemvArgs::tp_*), with its own per-item epochs
  P2PComm(int rank, int world, int max_n, int device, bool uncached = true, int fused_n = 0);
  ~P2PComm();
  P2PComm(const P2PComm&) = delete;
  P2PComm& operator=(const P2PComm&) = delete;

  std::string handle() const;                          // hipIpcMemHandle_t bytes of this rank's region
  void open(const std::vector<std::string>& handles);  // every rank's handle, in rank order
  bool ready() const { return ready_; }
  int max_n() const { return max_n_; }
  void allreduce(const float* src, float* dst, int n, hipStream_t s);
  // dst += the all-reduced src, and src is left zeroed (P2PArgs::accumulate)
  void allreduce_add(float* src, float* dst, int n, hipStream_t s);
  void allgather(const float* src, float* dst, int n, hipStream_t s);  // dst [world][n]
  int error() const;                                   // device error word (0 = ok)
  // the group's fault words as stored in this rank's region (fault[r]: rank r's code, 0 = none):
  // any rank's timed-out wait, or a host failure raise_fault() published
  // fresh = false: the host-mapped mirror the last collective launch left (no copy; the engine's
  // per-step check), true: a blocking read of the region itself
  std::vector<int> faults(bool fresh = true) const;
  std::string fault_report(bool fresh = true) const;   // "" = no rank faulted
  void raise_fault(int code);                          // this rank's code into every rank's region
  bool uncached() const { return uncached_; }          // region allocated hipDeviceMallocUncached
  // diagnostics: per rank (mapped pointer, allocation base, allocation size) as seen here
  std::vector<std::vector<unsigned long long>> mappings() const;
  void reset_error();
  // the fused area: granule stride per (slot, rank), its offset, per-item epochs, peers
  int stride() const { return max_n_ + kP2PMaxBlocks + fused_n_; }
  int fused_offset() const { return max_n_ + kP2PMaxBlocks; }
  int fused_n() const { return fused_n_; }
  int* fused_epochs() const { return fused_epochs_; }
  int* err_word() const { return err_; }
  const P2PPeers& peers() const { return peers_; }
  int rank() const { return rank_; }
  bool shared_device() const { return shared_device_; }  // some peer is on this rank's GPU (rehearsal)
  int world() const { return world_; }

 private:
  int rank_, world_, max_n_, device_, fused_n_ = 0;
  int* fused_epochs_ = nullptr;
  size_t data_bytes_ = 0, region_bytes_ = 0;
  void* region_ = nullptr;
  std::vector<void*> imported_;
  int* epochs_ = nullptr;
  int* err_ = nullptr;
  int* fault_h_ = nullptr;   // host-mapped mirror of this rank's fault words (P2PArgs::fault_h)
  int* fault_hd_ = nullptr;  // ... its device-side address
  P2PPeers peers_;
  bool ready_ = false;
  bool shared_device_ = false;
  bool uncached_ = false;
  void launch(const float* src, float* dst, int n, int gather, hipStream_t s, int accumulate = 0);
};

}  // namespace lfk
