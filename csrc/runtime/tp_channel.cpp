#include "tp_channel.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <chrono>
#include <thread>

namespace lfk {

static constexpr uint32_t kMagic = 0x4c464b54;  // "LFKT"
static constexpr int kMaxFollowers = 8;
static constexpr int kFaultMsg = 240;

struct alignas(64) TPChannel::Hdr {
  uint32_t magic;
  int32_t world;
  int32_t leader_pid;
  uint32_t cap;
  alignas(64) std::atomic<uint32_t> seq;          // commands published (futex word)
  alignas(64) std::atomic<uint32_t> ack[kMaxFollowers];  // last command each rank copied
  std::atomic<int32_t> follower_pid[kMaxFollowers];      // set by attach(): the leader's liveness probe
  // a follower's failure (report_fault): the message first, then the word (release)
  alignas(64) std::atomic<int32_t> fault[kMaxFollowers];
  char fault_msg[kMaxFollowers][kFaultMsg];
  alignas(64) uint32_t len;                        // bytes of the current command
};

// a process that exited - or exited and is not yet reaped (a zombie) - is dead for the channel
static bool pid_alive(int pid) {
  if (pid <= 0) return true;  // not known (yet): nothing to probe
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  if (FILE* f = fopen(path, "r")) {
    char state = 0;
    const int n = fscanf(f, "%*d %*s %c", &state);
    fclose(f);
    if (n == 1 && (state == 'Z' || state == 'X')) return false;
  }
  return true;
}

static_assert(std::atomic<uint32_t>::is_always_lock_free, "futex word must be a plain 32-bit word");

static long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

static std::string shm_name(const std::string& name) { return name.empty() || name[0] != '/' ? "/" + name : name; }

std::unique_ptr<TPChannel> TPChannel::create(const std::string& name, int world, size_t cap) {
  if (world < 2 || world > kMaxFollowers) throw std::runtime_error("tp channel: world must be 2..8");
  std::unique_ptr<TPChannel> c(new TPChannel());
  c->name_ = shm_name(name);
  c->rank_ = 0;
  c->bytes_ = sizeof(Hdr) + cap;
  c->fd_ = shm_open(c->name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (c->fd_ < 0) throw std::runtime_error("tp channel: shm_open(" + c->name_ + ") failed: " + strerror(errno));
  if (ftruncate(c->fd_, (off_t)c->bytes_) != 0) throw std::runtime_error("tp channel: ftruncate failed");
  void* p = mmap(nullptr, c->bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, c->fd_, 0);
  if (p == MAP_FAILED) throw std::runtime_error("tp channel: mmap failed");
  c->h_ = new (p) Hdr();
  c->h_->world = world;
  c->h_->leader_pid = (int32_t)getpid();
  c->h_->cap = (uint32_t)cap;
  c->h_->len = 0;
  c->h_->seq.store(0);
  for (auto& a : c->h_->ack) a.store(0);
  for (auto& p : c->h_->follower_pid) p.store(0);
  for (auto& f : c->h_->fault) f.store(0);
  c->payload_ = static_cast<uint8_t*>(p) + sizeof(Hdr);
  std::atomic_thread_fence(std::memory_order_release);
  c->h_->magic = kMagic;
  return c;
}

std::unique_ptr<TPChannel> TPChannel::attach(const std::string& name, int rank) {
  if (rank < 1 || rank >= kMaxFollowers) throw std::runtime_error("tp channel: bad follower rank");
  std::unique_ptr<TPChannel> c(new TPChannel());
  c->name_ = shm_name(name);
  c->rank_ = rank;
  c->fd_ = shm_open(c->name_.c_str(), O_RDWR, 0600);
  if (c->fd_ < 0) throw std::runtime_error("tp channel: shm_open(" + c->name_ + ") failed: " + strerror(errno));
  struct stat st;
  if (fstat(c->fd_, &st) != 0 || (size_t)st.st_size < sizeof(Hdr)) throw std::runtime_error("tp channel: bad segment");
  c->bytes_ = (size_t)st.st_size;
  void* p = mmap(nullptr, c->bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, c->fd_, 0);
  if (p == MAP_FAILED) throw std::runtime_error("tp channel: mmap failed");
  c->h_ = static_cast<Hdr*>(p);
  std::atomic_thread_fence(std::memory_order_acquire);
  if (c->h_->magic != kMagic || rank >= c->h_->world) throw std::runtime_error("tp channel: segment not initialised");
  c->payload_ = static_cast<uint8_t*>(p) + sizeof(Hdr);
  c->last_ = c->h_->seq.load(std::memory_order_acquire);  // nothing before attach is ours
  c->h_->follower_pid[rank].store((int32_t)getpid(), std::memory_order_relaxed);
  c->h_->ack[rank].store(c->last_, std::memory_order_release);
  return c;
}

TPChannel::~TPChannel() {
  // rank 0 owns the segment; a follower outliving a dead leader removes it too (no /dev/shm leak)
  const bool unlink = !name_.empty() && (rank_ == 0 || (h_ && !leader_alive()));
  if (h_) munmap(h_, bytes_);
  if (fd_ >= 0) close(fd_);
  if (unlink) shm_unlink(name_.c_str());
}

int TPChannel::world() const { return h_->world; }

bool TPChannel::leader_alive() const { return pid_alive(h_->leader_pid); }

void TPChannel::report_fault(const std::string& msg) {
  if (rank_ == 0) return;
  if (h_->fault[rank_].load(std::memory_order_acquire)) return;  // the first failure is the one kept
  const size_t n = std::min(msg.size(), (size_t)kFaultMsg - 1);
  std::memcpy(h_->fault_msg[rank_], msg.data(), n);
  h_->fault_msg[rank_][n] = 0;
  h_->fault[rank_].store(1, std::memory_order_release);
}

std::string TPChannel::fault_report() const {
  std::string out;
  const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  const bool probe = now - probe_ns_ >= 100000000LL;
  if (probe) probe_ns_ = now;
  if ((int)exited_.size() != h_->world) exited_.assign(h_->world, 0);
  for (int r = 1; r < h_->world; ++r) {
    std::string what;
    if (probe && !exited_[r]) exited_[r] = !pid_alive(h_->follower_pid[r].load(std::memory_order_relaxed));
    if (h_->fault[r].load(std::memory_order_acquire)) what = h_->fault_msg[r];
    else if (exited_[r]) what = "exited";
    if (!what.empty()) out += (out.empty() ? "" : "; ") + std::string("rank ") + std::to_string(r) + ": " + what;
  }
  return out;
}

void TPChannel::publish(const TPMsg& m) {
  if (rank_ != 0) throw std::runtime_error("tp channel: only rank 0 publishes");
  if (m.buf.size() > h_->cap) throw std::runtime_error("tp channel: command larger than the mailbox");
  const uint32_t cur = h_->seq.load(std::memory_order_relaxed);
  // every follower must have copied command `cur` before the mailbox is overwritten
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 1; r < h_->world; ++r) {
    int spins = 0;
    while (h_->ack[r].load(std::memory_order_acquire) != cur) {
      if (++spins < 2000) continue;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
      // a crashed follower fails the command at once (every ~50 ms a liveness probe) instead of
      // holding the engine - and the scheduler thread behind it - for the full timeout
      if (spins % 2500 == 0 && !pid_alive(h_->follower_pid[r].load(std::memory_order_relaxed)))
        throw std::runtime_error("tp channel: follower rank " + std::to_string(r) + " exited");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600))
        throw std::runtime_error("tp channel: follower rank " + std::to_string(r) + " stopped consuming commands");
    }
  }
  std::memcpy(payload_, m.buf.data(), m.buf.size());
  h_->len = (uint32_t)m.buf.size();
  h_->seq.store(cur + 1, std::memory_order_release);
  futex(&h_->seq, FUTEX_WAKE, INT32_MAX, nullptr);
}

bool TPChannel::receive(TPMsg& m, int timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  int spins = 0;
  while (true) {
    const uint32_t s = h_->seq.load(std::memory_order_acquire);
    if (s != last_) {
      if (s != last_ + 1) throw std::runtime_error("tp channel: missed a command");
      m.buf.assign(payload_, payload_ + h_->len);
      m.rd = 0;
      last_ = s;
      h_->ack[rank_].store(s, std::memory_order_release);
      return true;
    }
    if (++spins < 4000) continue;  // a decode step's command follows the previous one closely
    const auto now = std::chrono::steady_clock::now();
    if (now >= deadline) return false;
    const auto left = std::chrono::duration_cast<std::chrono::nanoseconds>(deadline - now).count();
    timespec ts{(time_t)(left / 1000000000), (long)(left % 1000000000)};
    futex(&h_->seq, FUTEX_WAIT, s, &ts);  // returns at once if seq already moved
  }
}

}  // namespace lfk
