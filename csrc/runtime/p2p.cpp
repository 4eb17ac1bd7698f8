#include "p2p.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace lfk {

static void p2pchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("p2p: ") + what + ": " + hipGetErrorString(e));
}

P2PComm::P2PComm(int rank, int world, int max_n, int device, bool uncached, int fused_n)
    : rank_(rank), world_(world), max_n_((max_n + 3) & ~3), device_(device), fused_n_(std::max(0, fused_n)),
      uncached_(uncached) {
  if (world < 1 || world > kP2PMaxRanks || rank < 0 || rank >= world) throw std::runtime_error("p2p: bad rank/world");
  if (max_n <= 0) throw std::runtime_error("p2p: bad max_n");
  p2pchk(hipSetDevice(device_), "hipSetDevice");
  // {value, epoch} granules: max_n data + kP2PMaxBlocks heartbeats (+ the fused area) per (slot, rank)
  data_bytes_ = sizeof(unsigned long long) * 2 * (size_t)world * (max_n_ + kP2PMaxBlocks + fused_n_);
  data_bytes_ = (data_bytes_ + 255) & ~(size_t)255;
  region_bytes_ = data_bytes_ + sizeof(int) * 2 * (size_t)world * kP2PMaxBlocks;
  // A whole, 2 MiB-granular allocation of its own, UNCACHED (hipDeviceMallocUncached): peers
  // store payloads and flags into it over xGMI while this GPU polls and reads it, so no L2 of
  // either side may hold a line of it (a stale line of the previous epoch is the classic
  // cross-device failure; the kernel's system-scope fences order the accesses, the memory type
  // keeps every one of them at the memory). Ranks sharing a GPU (the one-GPU IPC rehearsal)
  // import it the same way (tests/test_p2p_allreduce.py runs both region types).
  // An exported IPC handle names the underlying allocation: the region must BE that allocation
  // (checked below), or the peer's mapping would start at the allocation's base.
  region_bytes_ = (region_bytes_ + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
  if (!uncached_ || hipExtMallocWithFlags(&region_, region_bytes_, hipDeviceMallocUncached) != hipSuccess) {
    if (uncached_) (void)hipGetLastError();
    region_ = nullptr;
    p2pchk(hipMalloc(&region_, region_bytes_), "hipMalloc region");
    uncached_ = false;
  }
  {
    hipDeviceptr_t base = nullptr;
    size_t sz = 0;
    p2pchk(hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)region_), "hipMemGetAddressRange region");
    if ((void*)base != region_ || sz < region_bytes_)
      throw std::runtime_error("p2p: the receive region is not a whole allocation of its own (IPC peers would map "
                               "its base, not the region)");
  }
  p2pchk(hipMemset(region_, 0, region_bytes_), "hipMemset region");
  p2pchk(hipMalloc((void**)&epochs_, sizeof(int) * kP2PMaxBlocks), "hipMalloc epochs");
  p2pchk(hipMemset(epochs_, 0, sizeof(int) * kP2PMaxBlocks), "hipMemset epochs");
  if (fused_n_ > 0) {  // per-item epochs of the fused area (an item = one GEMV wave item, >= 1 row)
    p2pchk(hipMalloc((void**)&fused_epochs_, sizeof(int) * fused_n_), "hipMalloc fused epochs");
    p2pchk(hipMemset(fused_epochs_, 0, sizeof(int) * fused_n_), "hipMemset fused epochs");
  }
  p2pchk(hipMalloc((void**)&err_, sizeof(int) * 4), "hipMalloc err");
  p2pchk(hipMemset(err_, 0, sizeof(int) * 4), "hipMemset err");
  p2pchk(hipHostMalloc((void**)&fault_h_, sizeof(int) * kP2PMaxRanks, hipHostMallocMapped | hipHostMallocCoherent),
         "hipHostMalloc fault mirror");
  std::memset(fault_h_, 0, sizeof(int) * kP2PMaxRanks);
  p2pchk(hipHostGetDevicePointer((void**)&fault_hd_, fault_h_, 0), "hipHostGetDevicePointer fault mirror");
  p2pchk(hipDeviceSynchronize(), "sync");
}

P2PComm::~P2PComm() {
  for (void* p : imported_)
    if (p) (void)hipIpcCloseMemHandle(p);
  if (region_) (void)hipFree(region_);
  if (epochs_) (void)hipFree(epochs_);
  if (fused_epochs_) (void)hipFree(fused_epochs_);
  if (err_) (void)hipFree(err_);
  if (fault_h_) (void)hipHostFree(fault_h_);
}

std::string P2PComm::handle() const {
  hipIpcMemHandle_t h;
  p2pchk(hipIpcGetMemHandle(&h, region_), "hipIpcGetMemHandle");
  // + this rank's device index: peers on the same device (the one-GPU IPC rehearsal) are told apart
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h)) +
         std::string(reinterpret_cast<const char*>(&device_), sizeof(int));
}

void P2PComm::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("p2p: need one handle per rank");
  p2pchk(hipSetDevice(device_), "hipSetDevice");
  for (int p = 0; p < world_; ++p) {
    char* base = nullptr;
    if (p == rank_) {
      base = static_cast<char*>(region_);
    } else {
      if (handles[p].size() != sizeof(hipIpcMemHandle_t) + sizeof(int)) throw std::runtime_error("p2p: bad handle size");
      int pdev = -1;
      std::memcpy(&pdev, handles[p].data() + sizeof(hipIpcMemHandle_t), sizeof(int));
      shared_device_ = shared_device_ || pdev == device_;
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[p].data(), sizeof(h));
      void* ptr = nullptr;
      p2pchk(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      imported_.push_back(ptr);
      // the mapping must cover the peer's whole region (same layout on every rank)
      hipDeviceptr_t mbase = nullptr;
      size_t msz = 0;
      p2pchk(hipMemGetAddressRange(&mbase, &msz, (hipDeviceptr_t)ptr), "hipMemGetAddressRange peer");
      if ((char*)mbase + msz < (char*)ptr + region_bytes_)
        throw std::runtime_error("p2p: rank " + std::to_string(p) + "'s imported region is smaller than the layout");
      base = static_cast<char*>(ptr);
    }
    if (!base) throw std::runtime_error("p2p: no mapping for rank " + std::to_string(p));
    peers_.data[p] = reinterpret_cast<float*>(base);
    peers_.fault[p] = reinterpret_cast<int*>(base + data_bytes_);
  }
  ready_ = true;
}

void P2PComm::launch(const float* src, float* dst, int n, int gather, hipStream_t s, int accumulate) {
  if (!ready_) throw std::runtime_error("p2p: open() the peer handles first");
  P2PArgs a;
  a.peers = peers_;
  a.src = src; a.dst = dst; a.n = n; a.max_n = max_n_; a.rank = rank_; a.world = world_; a.gather = gather;
  a.accumulate = accumulate;
  a.stride = stride();
  a.epochs = epochs_; a.err = err_; a.fault_h = fault_hd_;
  p2p_collective(a, s);
}

void P2PComm::allreduce(const float* src, float* dst, int n, hipStream_t s) { launch(src, dst, n, 0, s); }

void P2PComm::allreduce_add(float* src, float* dst, int n, hipStream_t s) { launch(src, dst, n, 0, s, 1); }

void P2PComm::allgather(const float* src, float* dst, int n, hipStream_t s) { launch(src, dst, n, 1, s); }

std::vector<std::vector<unsigned long long>> P2PComm::mappings() const {
  std::vector<std::vector<unsigned long long>> out;
  for (int p = 0; p < world_; ++p) {
    void* ptr = p == rank_ ? region_ : (ready_ ? (void*)peers_.data[p] : nullptr);
    hipDeviceptr_t base = nullptr;
    size_t sz = 0;
    if (ptr && hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)ptr) != hipSuccess) {
      (void)hipGetLastError();
      base = nullptr;
      sz = 0;
    }
    out.push_back({(unsigned long long)(uintptr_t)ptr, (unsigned long long)(uintptr_t)base, (unsigned long long)sz});
  }
  return out;
}

int P2PComm::error() const {
  int e = 0;
  p2pchk(hipMemcpy(&e, err_, sizeof(int), hipMemcpyDeviceToHost), "read err");
  return e;
}

std::vector<int> P2PComm::faults(bool fresh) const {
  std::vector<int> f((size_t)world_, 0);
  if (!ready_) return f;
  if (!fresh) {
    for (int r = 0; r < world_; ++r) f[r] = __atomic_load_n(fault_h_ + r, __ATOMIC_ACQUIRE);
    return f;
  }
  p2pchk(hipMemcpy(f.data(), peers_.fault[rank_], sizeof(int) * world_, hipMemcpyDeviceToHost), "read faults");
  return f;
}

std::string P2PComm::fault_report(bool fresh) const {
  std::string out;
  const std::vector<int> f = faults(fresh);
  for (int r = 0; r < world_; ++r)
    if (f[r]) {
      const int c = f[r];
      const std::string what = c >= 1000 ? "its host failed a command" :
                               c >= 300 ? "its epilogue all-reduce wait for rank " + std::to_string(c % 100) + " timed out" :
                               "its collective wait for rank " + std::to_string(c % 100) + " timed out";
      out += (out.empty() ? "" : "; ") + std::string("rank ") + std::to_string(r) + ": " + what +
             " (code " + std::to_string(c) + ")";
    }
  return out;
}

void P2PComm::raise_fault(int code) {
  if (!ready_ || code == 0) return;
  for (int p = 0; p < world_; ++p)
    p2pchk(hipMemcpy(peers_.fault[p] + rank_, &code, sizeof(int), hipMemcpyHostToDevice), "raise fault");
}

void P2PComm::reset_error() {
  p2pchk(hipMemset(err_, 0, sizeof(int) * 4), "reset err");
  if (ready_) p2pchk(hipMemset(peers_.fault[rank_], 0, sizeof(int) * kP2PMaxRanks), "reset faults");
  std::memset(fault_h_, 0, sizeof(int) * kP2PMaxRanks);
}

}  // namespace lfk
