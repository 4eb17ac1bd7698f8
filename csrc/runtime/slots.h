// Host-only interface between the continuous-batching scheduler (scheduler.h) and an
// engine that holds several KV slots. The MI355X Engine implements it; tests drive the
// scheduler through a deterministic CPU stand-in (bindings_cpu.cpp) so its admission,
// prefix-reuse and retirement logic is checked without a GPU.
#pragma once
#include <utility>
#include <vector>

namespace lfk {

struct SamplingOpts {
  int top_k = 40;
  float top_p = 0.95f, min_p = 0.05f, temp = 0.8f;
  float repeat_penalty = 1.1f, freq_penalty = 0.f, presence_penalty = 0.f;
  int last_n = 64;
  unsigned long long seed = 0;
  float tfs_z = 1.f, typical_p = 1.f;
  std::vector<std::pair<int, float>> logit_bias;  // distinct tokens, at most kMaxLogitBias
};

class SlotBackend {
 public:
  virtual ~SlotBackend() = default;
  virtual int n_slots() const = 0;
  virtual int max_batch() const = 0;   // rows one batch_step takes
  virtual int n_ctx() const = 0;
  // prefill prompt[n_keep:] into `slot` (its first n_keep positions are reused), set the
  // slot's sampling state, return its first token
  virtual int slot_begin(int slot, const std::vector<int>& prompt, int n_keep, const SamplingOpts& sp) = 0;
  // several admissions at once (slot_begin of each, in order); an engine that can prefill
  // the prompts together (one pass of every weight for all of them) overrides it
  virtual std::vector<int> slots_begin(const std::vector<int>& slots, const std::vector<std::vector<int>>& prompts,
                                       const std::vector<int>& n_keep, const std::vector<SamplingOpts>& sps) {
    std::vector<int> out;
    for (size_t i = 0; i < slots.size(); ++i) out.push_back(slot_begin(slots[i], prompts[i], n_keep[i], sps[i]));
    return out;
  }
  // one decode step of every listed slot at its own position -> each slot's next token
  virtual std::vector<int> batch_step(const std::vector<int>& slots) = 0;
  // Pipelined form (optional): batch_launch queues one step and returns, batch_collect waits
  // for the OLDEST queued step and returns its tokens. Steps run in launch order, each feeding
  // from the tokens its predecessor sampled on the device, so the scheduler can queue step
  // k + 1 before it has handled step k's tokens. At most two steps in flight.
  virtual bool can_pipeline() const { return false; }
  // Chunked admission (optional; prefill_part_tokens() > 0 enables it): slot_begin in parts, so a
  // long prompt arriving while other rows decode does not stall them for its whole prefill.
  // slot_begin_part prefills prompt[n_done, n_done + n) into `slot` (the first call, with
  // n_done == n_keep, also sets the slot's state) and returns the first token once the prompt
  // is complete, -1 before. Decode steps of OTHER slots may run between the parts.
  virtual int prefill_part_tokens() const { return 0; }
  virtual int slot_begin_part(int slot, const std::vector<int>& prompt, int n_keep, int n_done, int n,
                              const SamplingOpts& sp) {
    (void)n_done; (void)n;
    return slot_begin(slot, prompt, n_keep, sp);
  }
  virtual void batch_launch(const std::vector<int>& slots) { (void)slots; }
  virtual std::vector<int> batch_collect() { return {}; }
};

}  // namespace lfk
