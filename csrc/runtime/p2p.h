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
  P2PComm(int rank, int world, int max_n, int device, bool uncached = true);
  ~P2PComm();
  P2PComm(const P2PComm&) = delete;
  P2PComm& operator=(const P2PComm&) = delete;

  std::string handle() const;                          // hipIpcMemHandle_t bytes of this rank's region
  void open(const std::vector<std::string>& handles);  // every rank's handle, in rank order
  bool ready() const { return ready_; }
  int max_n() const { return max_n_; }
  void allreduce(const float* src, float* dst, int n, hipStream_t s);
  void allgather(const float* src, float* dst, int n, hipStream_t s);  // dst [world][n]
  int error() const;                                   // device error word (0 = ok)
  bool uncached() const { return uncached_; }          // region allocated hipDeviceMallocUncached
  // diagnostics: per rank (mapped pointer, allocation base, allocation size) as seen here
  std::vector<std::vector<unsigned long long>> mappings() const;
  void reset_error();

 private:
  int rank_, world_, max_n_, device_;
  size_t data_bytes_ = 0, region_bytes_ = 0;
  void* region_ = nullptr;
  std::vector<void*> imported_;
  int* epochs_ = nullptr;
  int* err_ = nullptr;
  P2PPeers peers_;
  bool ready_ = false;
  bool uncached_ = false;
  void launch(const float* src, float* dst, int n, int gather, hipStream_t s);
};

}  // namespace lfk
