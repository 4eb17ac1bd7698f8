// Host control channel of a tensor-parallel engine group (SURVEY §2.5 TP, §3.5).
//
// Every rank of a row-split model must enqueue the same device work in the same order:
// its collectives pair with the other ranks'. Rank 0 owns the HTTP server, the admission
// queue and the continuous-batching scheduler; the follower ranks run no Python request
// path at all. Instead, every engine entry point on rank 0 publishes a small command
// (op + arguments: a prompt chunk, the slot list of a batch step, "one decode step") on
// this channel before it enqueues its own work, and each follower's native loop
// (Engine::follow) replays it. Cancellation, stop tokens and admission are decided on
// rank 0 only; the followers simply never receive the steps that did not happen.
//
// Transport: one POSIX shared-memory segment per group (the ranks of a TP group share a
// node - xGMI is intra-node), a single-slot mailbox with a sequence word, per-follower
// acknowledgements and a futex on the sequence word (followers sleep in the kernel
// between requests; a publish wakes them within microseconds). The leader waits only
// until every follower has COPIED the previous command, never for its execution, so
// the ranks run their GPU work concurrently.
#pragma once
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace lfk {

// Byte-buffer serialisation of one command.
class TPMsg {
 public:
  std::vector<uint8_t> buf;
  size_t rd = 0;
  template <class T>
  void put(const T& v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    buf.insert(buf.end(), p, p + sizeof(T));
  }
  template <class T>
  void put_vec(const std::vector<T>& v) {
    put<int64_t>((int64_t)v.size());
    const uint8_t* p = reinterpret_cast<const uint8_t*>(v.data());
    buf.insert(buf.end(), p, p + sizeof(T) * v.size());
  }
  template <class T>
  T get() {
    if (rd + sizeof(T) > buf.size()) throw std::runtime_error("tp channel: truncated command");
    T v;
    std::memcpy(&v, buf.data() + rd, sizeof(T));
    rd += sizeof(T);
    return v;
  }
  template <class T>
  std::vector<T> get_vec() {
    const int64_t n = get<int64_t>();
    if (n < 0 || rd + sizeof(T) * (size_t)n > buf.size()) throw std::runtime_error("tp channel: truncated command");
    std::vector<T> v((size_t)n);
    std::memcpy(v.data(), buf.data() + rd, sizeof(T) * (size_t)n);
    rd += sizeof(T) * (size_t)n;
    return v;
  }
};

class TPChannel {
 public:
  // rank 0: create the segment (payload capacity `cap` bytes); followers: attach to it
  static std::unique_ptr<TPChannel> create(const std::string& name, int world, size_t cap);
  static std::unique_ptr<TPChannel> attach(const std::string& name, int rank);
  ~TPChannel();
  TPChannel(const TPChannel&) = delete;
  TPChannel& operator=(const TPChannel&) = delete;

  // leader: wait until every follower copied the previous command, then publish this one
  void publish(const TPMsg& m);
  // follower: the next command (true), or false after timeout_ms without one
  bool receive(TPMsg& m, int timeout_ms);
  bool leader_alive() const;
  // follower: publish this rank's failure (message kept, first failure wins); leader: every
  // follower's published failure or exit, "" while the group is sound (a shared-memory read)
  void report_fault(const std::string& msg);
  std::string fault_report() const;
  int rank() const { return rank_; }
  int world() const;

 private:
  struct Hdr;
  TPChannel() = default;
  std::string name_;
  int rank_ = 0;
  int fd_ = -1;
  size_t bytes_ = 0;
  Hdr* h_ = nullptr;
  uint8_t* payload_ = nullptr;
  // fault_report()'s follower liveness probes (kill + /proc reads) run at most every 100 ms: the
  // engine asks after every step, and a fault flag in the shared header needs no probe
  mutable int64_t probe_ns_ = 0;
  mutable std::vector<int> exited_;
  uint32_t last_ = 0;  // follower: the last sequence number it consumed
};

}  // namespace lfk
