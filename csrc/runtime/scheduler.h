// Continuous-batching scheduler (native runtime around Engine::slot_begin / batch_step).
//
// The reference serves one generation at a time per pod (reference api.py:50,80-107:
// one consumer task + Semaphore(1); llama-cpp-python's Llama is single-sequence). Batch-1
// decode on MI355X is weight-streaming bound (every token re-reads ~4.6 GB of weights), so
// serving N requests as N independent sequences costs N weight streams; decoding them as
// ONE batch costs one. This scheduler owns a host thread that keeps the engine's KV slots
// busy:
//
//   loop:  retire cancelled requests  ->  admit every queued request that finds a free slot
//          (slots_begin: ONE packed prefill of all their prompts + each first token; the
//          free slot whose resident tokens share the longest prefix with the prompt is
//          chosen and that prefix is not recomputed)
//          ->  one batch_step over every active slot  ->  hand each row its token,
//          finish rows on a stop id / max_new / context end.
//
// Slot 0 is left to the engine's single-sequence path (Engine::generate, used for sampler
// configurations the GPU chain does not cover); the scheduler uses slots [1, n_slots).
// Both paths serialise on the engine's execution guard.
//
// Request threads (Python, GIL released) submit token ids and block in wait() for new
// tokens; detokenisation, stop strings and the OpenAI response shape stay in the facade.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "slots.h"

namespace lfk {

struct SchedPoll {
  std::vector<int> tokens;   // tokens [have, have + n) of the request
  bool done = false;
  std::string finish;        // "stop" | "length" | "cancelled" | "error" once done
  std::string error;
  int n_prompt = 0, n_prefilled = 0;
  double queue_s = 0, prefill_s = 0, decode_s = 0;
};

struct SchedStats {
  long long steps = 0;        // batch_step calls
  long long rows = 0;         // rows decoded over all steps
  long long admitted = 0;
  long long reused_tokens = 0;  // prompt tokens served from a slot's resident KV prefix
  long long joint_admissions = 0;  // admissions that prefilled several prompts in one pass
  long long chunked_admissions = 0;  // prompts prefilled in parts between decode steps
  int active = 0, pending = 0, slots = 0;
};

class BatchScheduler {
 public:
  explicit BatchScheduler(SlotBackend& e);
  ~BatchScheduler();
  BatchScheduler(const BatchScheduler&) = delete;
  BatchScheduler& operator=(const BatchScheduler&) = delete;

  // Queue a request: prompt token ids, at most max_new generated tokens (the context end
  // also ends it), sampling options of the GPU chain, stop token ids. Returns its id.
  int64_t submit(const std::vector<int>& prompt, int max_new, const SamplingOpts& sp,
                 const std::vector<int>& stop_ids);
  // Tokens of request `id` past the first `have`; blocks up to timeout_ms until there is at
  // least one new token or the request is done.
  SchedPoll wait(int64_t id, size_t have, int timeout_ms);
  void cancel(int64_t id);    // cooperative: the row leaves the batch before the next step
  void release(int64_t id);   // forget a finished (or abandoned: cancels it) request
  SchedStats stats();
  void shutdown();            // stop the thread; unfinished requests end "cancelled"

 private:
  struct Req {
    int64_t id = 0;
    std::vector<int> prompt;
    int max_new = 0;
    SamplingOpts sp;
    std::vector<int> stop_ids;
    std::vector<int> tokens;
    int slot = -1;
    int n_prefilled = 0;
    int n_keep = 0;
    int n_done = -1;   // chunked admission: prompt tokens prefilled so far (-1: not prefilling)
    bool cancel = false, done = false;
    std::string finish, error;
    double t_submit = 0, t_start = 0, t_first = 0, t_done = 0;
  };
  void loop();
  void finish(Req& r, const char* reason);
  void push_token(Req& r, int tok);       // append one sampled token; may finish the row
  int pick_slot(const std::vector<int>& prompt, int* lcp);

  SlotBackend& eng_;
  int first_slot_ = 1, n_slots_ = 1;
  bool pipeline_ = false;  // batch_launch / batch_collect (LFK_SCHED_PIPELINE=0: synchronous steps)
  std::mutex mu_;
  std::condition_variable cv_work_, cv_out_;
  std::deque<std::shared_ptr<Req>> pending_;
  std::map<int64_t, std::shared_ptr<Req>> reqs_;
  std::vector<std::shared_ptr<Req>> slot_req_;   // active request per slot (null = free)
  std::vector<std::vector<int>> slot_hist_;      // tokens resident in each slot's KV
  std::vector<long long> slot_used_;             // last admission tick (LRU among equal prefixes)
  long long tick_ = 0;
  int64_t next_id_ = 1;
  bool stop_ = false;
  SchedStats st_;
  std::thread th_;
};

}  // namespace lfk
