// Continuous-batching scheduler: see scheduler.h.
#include "scheduler.h"

#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <stdexcept>

namespace lfk {

static double sched_now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

BatchScheduler::BatchScheduler(SlotBackend& e) : eng_(e) {
  n_slots_ = e.n_slots();
  if (n_slots_ < 2 || e.max_batch() < 1)
    throw std::runtime_error("BatchScheduler: the engine needs n_slots >= 2 (slot 0 stays with generate())");
  // batch_step takes at most max_batch rows: never keep more slots active than that
  n_slots_ = std::min(n_slots_, first_slot_ + e.max_batch());
  slot_req_.resize(n_slots_);
  slot_hist_.resize(n_slots_);
  slot_used_.assign(n_slots_, 0);
  st_.slots = n_slots_ - first_slot_;
  const char* pe = std::getenv("LFK_SCHED_PIPELINE");
  pipeline_ = e.can_pipeline() && !(pe && pe[0] == '0');
  th_ = std::thread([this] { loop(); });
}

BatchScheduler::~BatchScheduler() { shutdown(); }

void BatchScheduler::shutdown() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_ && !th_.joinable()) return;
    stop_ = true;
  }
  cv_work_.notify_all();
  if (th_.joinable()) th_.join();
}

int64_t BatchScheduler::submit(const std::vector<int>& prompt, int max_new, const SamplingOpts& sp,
                               const std::vector<int>& stop_ids) {
  if (prompt.empty()) throw std::runtime_error("empty prompt");
  if ((int)prompt.size() >= eng_.n_ctx()) throw std::runtime_error("prompt exceeds context window");
  auto r = std::make_shared<Req>();
  r->prompt = prompt;
  r->max_new = std::max(1, max_new);
  r->sp = sp;
  r->stop_ids = stop_ids;
  r->t_submit = sched_now();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) throw std::runtime_error("BatchScheduler: shut down");
    r->id = next_id_++;
    reqs_[r->id] = r;
    pending_.push_back(r);
  }
  cv_work_.notify_one();
  return r->id;
}

SchedPoll BatchScheduler::wait(int64_t id, size_t have, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto it = reqs_.find(id);
  if (it == reqs_.end()) throw std::runtime_error("BatchScheduler: unknown request");
  std::shared_ptr<Req> r = it->second;
  cv_out_.wait_for(lk, std::chrono::milliseconds(std::max(0, timeout_ms)),
                   [&] { return r->done || r->tokens.size() > have; });
  SchedPoll p;
  if (r->tokens.size() > have) p.tokens.assign(r->tokens.begin() + have, r->tokens.end());
  p.done = r->done;
  p.finish = r->finish;
  p.error = r->error;
  p.n_prompt = (int)r->prompt.size();
  p.n_prefilled = r->n_prefilled;
  if (r->t_start > 0) p.queue_s = r->t_start - r->t_submit;
  if (r->t_first > 0) p.prefill_s = r->t_first - r->t_start;
  if (r->t_first > 0) p.decode_s = (r->done ? r->t_done : sched_now()) - r->t_first;
  return p;
}

void BatchScheduler::cancel(int64_t id) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = reqs_.find(id);
    if (it == reqs_.end() || it->second->done) return;
    it->second->cancel = true;
  }
  cv_work_.notify_one();
}

void BatchScheduler::release(int64_t id) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = reqs_.find(id);
    if (it == reqs_.end()) return;
    it->second->cancel = true;  // an abandoned active row leaves the batch at the next step
    reqs_.erase(it);
  }
  cv_work_.notify_one();
}

SchedStats BatchScheduler::stats() {
  std::lock_guard<std::mutex> g(mu_);
  SchedStats s = st_;
  s.pending = (int)pending_.size();
  s.active = 0;
  for (int i = first_slot_; i < n_slots_; ++i) s.active += slot_req_[i] != nullptr;
  return s;
}

// caller holds mu_
void BatchScheduler::finish(Req& r, const char* reason) {
  if (r.done) return;
  r.done = true;
  r.finish = reason;
  r.t_done = sched_now();
  if (r.slot >= 0 && slot_req_[r.slot].get() == &r) slot_req_[r.slot] = nullptr;
  cv_out_.notify_all();
}

// caller holds mu_. The KV of the row now holds every token but the newest one, which the
// next batch_step feeds; a row ends on a stop id, max_new, a cancel, or when that next
// step would write past the context.
void BatchScheduler::push_token(Req& r, int tok) {
  r.tokens.push_back(tok);
  if (std::find(r.stop_ids.begin(), r.stop_ids.end(), tok) != r.stop_ids.end()) return finish(r, "stop");
  if ((int)r.tokens.size() >= r.max_new) return finish(r, "length");
  if ((int)(r.prompt.size() + r.tokens.size()) - 1 >= eng_.n_ctx()) return finish(r, "length");
  if (r.cancel) return finish(r, "cancelled");
}

// caller holds mu_: the free slot whose resident tokens share the longest prefix with the
// prompt (least recently admitted among equals, so other conversations' prefixes survive)
int BatchScheduler::pick_slot(const std::vector<int>& prompt, int* lcp) {
  int best = -1, best_lcp = -1;
  for (int s = first_slot_; s < n_slots_; ++s) {
    if (slot_req_[s]) continue;
    const std::vector<int>& h = slot_hist_[s];
    const size_t n = std::min(h.size(), prompt.size());
    size_t k = 0;
    while (k < n && h[k] == prompt[k]) ++k;
    if ((int)k > best_lcp || ((int)k == best_lcp && slot_used_[s] < slot_used_[best])) {
      best = s;
      best_lcp = (int)k;
    }
  }
  *lcp = std::max(0, best_lcp);
  return best;
}

void BatchScheduler::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  std::vector<int> rows;
  std::vector<std::shared_ptr<Req>> row_req;
  struct Flight {
    std::vector<int> rows;
    std::vector<std::shared_ptr<Req>> req;
  };
  std::deque<Flight> flights;  // pipelined steps queued on the engine, oldest first
  std::deque<std::shared_ptr<Req>> prefilling;  // chunked admissions in progress, oldest first
  while (true) {
    cv_work_.wait(lk, [&] {
      if (stop_ || !pending_.empty() || !flights.empty()) return true;
      for (int s = first_slot_; s < n_slots_; ++s)
        if (slot_req_[s]) return true;
      return false;
    });
    if (stop_) break;
    // 1. rows whose request was cancelled / abandoned leave before anything runs
    for (int s = first_slot_; s < n_slots_; ++s)
      if (slot_req_[s] && slot_req_[s]->cancel) finish(*slot_req_[s], "cancelled");
    // 2. admission: queued requests into free slots, prefilled TOGETHER (one packed prefill
    //    pass streams every weight once for all of them) + the first token of each
    {
      std::vector<std::shared_ptr<Req>> adm;
      std::vector<int> a_slot, a_keep;
      const int chunk = eng_.prefill_part_tokens();
      bool decoding = false;
      for (int s = first_slot_; s < n_slots_; ++s) decoding = decoding || (slot_req_[s] && slot_req_[s]->n_done < 0);
      while (!pending_.empty()) {
        std::shared_ptr<Req> r = pending_.front();
        if (r->cancel) {
          pending_.pop_front();
          finish(*r, "cancelled");
          continue;
        }
        int lcp = 0;
        const int slot = pick_slot(r->prompt, &lcp);
        if (slot < 0) break;
        pending_.pop_front();
        r->slot = slot;
        slot_req_[slot] = r;
        slot_used_[slot] = ++tick_;
        r->t_start = sched_now();
        const int keep = std::min(lcp, (int)r->prompt.size() - 1);
        // chunked admission: a prompt longer than one chunk, while rows are decoding, is
        // prefilled in parts between their steps (below) instead of stalling them for all of it
        if (chunk > 0 && decoding && (int)r->prompt.size() - keep > chunk) {
          r->n_keep = keep;
          r->n_done = keep;
          // the parts overwrite the slot's KV from `keep` on: only that prefix of the previous
          // occupant's history stays valid, whether or not this request completes its prefill
          if ((int)slot_hist_[slot].size() > keep) slot_hist_[slot].resize(keep);
          prefilling.push_back(r);
          continue;
        }
        adm.push_back(r);
        a_slot.push_back(slot);
        a_keep.push_back(keep);
      }
      if (!adm.empty()) {
        std::vector<std::vector<int>> prompts;
        std::vector<SamplingOpts> sps;
        for (auto& r : adm) {
          prompts.push_back(r->prompt);
          sps.push_back(r->sp);
        }
        std::string err;
        std::vector<int> toks;
        lk.unlock();
        try {
          toks = adm.size() == 1 ? std::vector<int>{eng_.slot_begin(a_slot[0], prompts[0], a_keep[0], sps[0])}
                                 : eng_.slots_begin(a_slot, prompts, a_keep, sps);
        } catch (const std::exception& e) {
          err = e.what();
        }
        lk.lock();
        const double t = sched_now();
        for (size_t i = 0; i < adm.size(); ++i) {
          Req& r = *adm[i];
          r.t_first = t;
          if (!err.empty()) {
            slot_hist_[a_slot[i]].clear();
            r.error = err;
            finish(r, "error");
            continue;
          }
          ++st_.admitted;
          st_.reused_tokens += a_keep[i];
          r.n_prefilled = (int)r.prompt.size() - a_keep[i];
          slot_hist_[a_slot[i]] = r.prompt;
          push_token(r, toks[i]);
        }
        if (adm.size() > 1) ++st_.joint_admissions;
        cv_out_.notify_all();  // the first tokens reach their waiters now, not after the next step
      }
    }
    // 2b. one part of the oldest chunked admission (a part is one prefill pass; the rows
    //     that decode get their next step right after it)
    if (!prefilling.empty()) {
      std::shared_ptr<Req> r = prefilling.front();
      if (r->cancel || r->done) {
        prefilling.pop_front();
      } else {
        const int n = eng_.prefill_part_tokens();
        const int done = r->n_done;
        const int slot = r->slot, keep = r->n_keep;
        std::vector<int> prompt = r->prompt;
        SamplingOpts sp = r->sp;
        std::string err;
        int tok = -1;
        lk.unlock();
        try {
          tok = eng_.slot_begin_part(slot, prompt, keep, done, n, sp);
        } catch (const std::exception& e) {
          err = e.what();
        }
        lk.lock();
        if (!err.empty()) {
          prefilling.pop_front();
          slot_hist_[slot].clear();
          r->error = err;
          finish(*r, "error");
        } else if (tok < 0) {
          r->n_done = std::min((int)prompt.size(), done + n);
        } else {
          prefilling.pop_front();
          r->n_done = -1;
          r->t_first = sched_now();
          ++st_.admitted;
          ++st_.chunked_admissions;
          st_.reused_tokens += keep;
          r->n_prefilled = (int)prompt.size() - keep;
          slot_hist_[slot] = prompt;
          push_token(*r, tok);
          cv_out_.notify_all();
        }
      }
    }
    // 3. one decode step over every active row. Pipelined (engines that can): the step of
    //    the current rows is queued and, while nothing waits for admission and the rows are
    //    those of the step already in flight, the NEXT step is queued too before the host
    //    handles this one's tokens - the device runs back to back through the host turnaround.
    //    A row that finishes on a step whose successor is already queued just has one extra
    //    token computed and dropped (its request is done; the KV slot is free either way).
    rows.clear();
    row_req.clear();
    for (int s = first_slot_; s < n_slots_; ++s)
      if (slot_req_[s] && slot_req_[s]->n_done < 0) {  // (a slot still prefilling has no row yet)
        rows.push_back(s);
        row_req.push_back(slot_req_[s]);
      }
    if (rows.empty() && flights.empty()) continue;
    std::vector<int> out;
    std::string err;
    Flight cur;
    lk.unlock();
    try {
      if (!pipeline_) {
        out = eng_.batch_step(rows);
        cur.rows = rows;
        cur.req = row_req;
      } else {
        if (flights.empty()) {
          eng_.batch_launch(rows);
          flights.push_back(Flight{rows, row_req});
        }
        // the next step feeds each row's newest token at position prompt + tokens - 1 + 1:
        // only while that stays inside the context (a row finishing on the context end must
        // not get a KV write past n_ctx from a step queued before its end was seen)
        // (queued requests hold the next step back only when one of them could be admitted now:
        // with every slot taken, pipelining stays on through the saturated stretch)
        bool more;
        {
          std::lock_guard<std::mutex> g(mu_);
          bool free_slot = false;
          for (int s = first_slot_; s < n_slots_ && !free_slot; ++s) free_slot = !slot_req_[s];
          more = (pending_.empty() || !free_slot) && !stop_;
          for (size_t b = 0; more && b < row_req.size(); ++b) {
            const Req& r = *row_req[b];
            more = !r.done && !r.cancel && (int)(r.prompt.size() + r.tokens.size()) < eng_.n_ctx();
          }
        }
        if (more && flights.size() == 1 && !rows.empty() && flights.back().rows == rows) {
          eng_.batch_launch(rows);
          flights.push_back(Flight{rows, row_req});
        }
        cur = flights.front();
        flights.pop_front();
        out = eng_.batch_collect();
      }
    } catch (const std::exception& e) {
      err = e.what();
      if (cur.rows.empty()) {
        cur.rows = rows;
        cur.req = row_req;
      }
      // the engine's state after a failed step is unknown: drop every queued step
      for (int k = (int)flights.size(); k > 0; --k) {
        try {
          eng_.batch_collect();
        } catch (...) {
        }
      }
      flights.clear();
    }
    lk.lock();
    ++st_.steps;
    st_.rows += (long long)cur.rows.size();
    for (size_t b = 0; b < cur.rows.size(); ++b) {
      Req& r = *cur.req[b];
      if (!err.empty()) {
        slot_hist_[cur.rows[b]].clear();
        if (!r.done) {
          r.error = err;
          finish(r, "error");
        }
        continue;
      }
      if (r.done) continue;  // finished (or cancelled) after this step was queued: its token is dropped
      slot_hist_[cur.rows[b]].push_back(r.tokens.back());  // the token this step fed is now in the KV
      push_token(r, out[b]);
    }
    cv_out_.notify_all();
  }
  // drain what is still queued before anything else uses the engine
  lk.unlock();
  for (size_t k = 0; k < flights.size(); ++k) {
    try {
      eng_.batch_collect();
    } catch (...) {
    }
  }
  flights.clear();
  lk.lock();
  // shutdown: nothing runs any more
  for (auto& r : pending_) finish(*r, "cancelled");
  pending_.clear();
  for (int s = first_slot_; s < n_slots_; ++s)
    if (slot_req_[s]) finish(*slot_req_[s], "cancelled");
  cv_out_.notify_all();
}

}  // namespace lfk
