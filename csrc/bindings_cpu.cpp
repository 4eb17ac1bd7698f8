// Python bindings of the C++ CPU backend (`llama_fastapi_k8s_gpu_amd.runtime._cpu`).
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bind_scheduler.h"
#include "cpu/cpu_backend.h"
#include "runtime/repack.h"
#include "runtime/tp_channel.h"

#include <chrono>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

namespace py = pybind11;
using namespace lfk;

static CpuSampling parse_sampling(py::dict sp) {
  CpuSampling o;
  if (sp.contains("top_k")) o.top_k = sp["top_k"].cast<int>();
  if (sp.contains("top_p")) o.top_p = sp["top_p"].cast<float>();
  if (sp.contains("min_p")) o.min_p = sp["min_p"].cast<float>();
  if (sp.contains("temperature")) o.temp = sp["temperature"].cast<float>();
  if (sp.contains("repeat_penalty")) o.repeat_penalty = sp["repeat_penalty"].cast<float>();
  if (sp.contains("frequency_penalty")) o.freq_penalty = sp["frequency_penalty"].cast<float>();
  if (sp.contains("presence_penalty")) o.presence_penalty = sp["presence_penalty"].cast<float>();
  if (sp.contains("last_n")) o.last_n = sp["last_n"].cast<int>();
  if (sp.contains("seed")) o.seed = sp["seed"].cast<unsigned long long>();
  return o;
}

// Deterministic stand-in for a multi-slot engine (scheduler tests on the CPU): each slot
// keeps the token sequence its "KV" holds; the next token is a hash of the whole sequence,
// so a request's output depends only on its own tokens (any batching must reproduce a
// sequential run), and slot_begin checks that the reused prefix really is resident.
class FakeSlotEngine : public SlotBackend {
 public:
  FakeSlotEngine(int n_slots, int max_batch, int n_ctx, int vocab, int step_us)
      : n_slots_(n_slots), max_batch_(max_batch), n_ctx_(n_ctx), vocab_(vocab), step_us_(step_us),
        kv_(n_slots), cur_(n_slots, 0) {}
  int n_slots() const override { return n_slots_; }
  int max_batch() const override { return max_batch_; }
  int n_ctx() const override { return n_ctx_; }
  static int next_token(const std::vector<int>& seq, int vocab) {
    unsigned long long h = 1469598103934665603ull;
    for (int t : seq) h = (h ^ (unsigned)t) * 1099511628211ull;
    return (int)(h % (unsigned long long)vocab);
  }
  int slot_begin(int slot, const std::vector<int>& prompt, int n_keep, const SamplingOpts&) override {
    std::lock_guard<std::mutex> g(mu_);
    if (slot < 0 || slot >= n_slots_) throw std::runtime_error("fake: slot out of range");
    std::vector<int>& kv = kv_[slot];
    if (n_keep > (int)kv.size()) throw std::runtime_error("fake: reused prefix is not resident");
    for (int i = 0; i < n_keep; ++i)
      if (kv[i] != prompt[i]) throw std::runtime_error("fake: reused prefix differs");
    kv.assign(prompt.begin(), prompt.end());
    prefilled_ += (long long)prompt.size() - n_keep;
    cur_[slot] = next_token(kv, vocab_);
    return cur_[slot];
  }
  // chunked admission: the prompt enters the slot's KV part by part (a reused prefix first)
  int prefill_part_tokens() const override { return chunk_; }
  int slot_begin_part(int slot, const std::vector<int>& prompt, int n_keep, int n_done, int n,
                      const SamplingOpts&) override {
    std::lock_guard<std::mutex> g(mu_);
    if (slot < 0 || slot >= n_slots_) throw std::runtime_error("fake: slot out of range");
    std::vector<int>& kv = kv_[slot];
    if (n_done == n_keep) {  // first part: the reused prefix must be resident
      if (n_keep > (int)kv.size()) throw std::runtime_error("fake: reused prefix is not resident");
      for (int i = 0; i < n_keep; ++i)
        if (kv[i] != prompt[i]) throw std::runtime_error("fake: reused prefix differs");
      kv.resize(n_keep);
    }
    if ((int)kv.size() != n_done) throw std::runtime_error("fake: prompt part out of order");
    const int end = std::min((int)prompt.size(), n_done + n);
    kv.insert(kv.end(), prompt.begin() + n_done, prompt.begin() + end);
    prefilled_ += end - n_done;
    ++parts_;
    if (end < (int)prompt.size()) return -1;
    cur_[slot] = next_token(kv, vocab_);
    return cur_[slot];
  }
  void set_prefill_chunk(int n) { chunk_ = n; }
  long long parts() { std::lock_guard<std::mutex> g(mu_); return parts_; }
  std::vector<int> batch_step(const std::vector<int>& slots) override {
    if (step_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(step_us_));
    std::lock_guard<std::mutex> g(mu_);
    if ((int)slots.size() > max_batch_) throw std::runtime_error("fake: too many rows");
    std::vector<int> out;
    for (int s : slots) {
      std::vector<int>& kv = kv_[s];
      if ((int)kv.size() >= n_ctx_) throw std::runtime_error("fake: KV write past n_ctx");
      kv.push_back(cur_[s]);
      cur_[s] = next_token(kv, vocab_);
      out.push_back(cur_[s]);
    }
    ++steps_;
    max_rows_ = std::max(max_rows_, (int)slots.size());
    if (fail_at_ > 0 && steps_ == fail_at_) throw std::runtime_error("fake: injected device fault");
    return out;
  }
  // pipelined form (the scheduler's batch_launch / batch_collect path): a launch runs the step
  // at once - its KV effects happen in launch order, as on the device - and queues the tokens
  bool can_pipeline() const override { return pipeline_; }
  void batch_launch(const std::vector<int>& slots) override {
    std::vector<int> out = batch_step(slots);
    std::lock_guard<std::mutex> g(mu_);
    if (queued_.size() >= 2) throw std::runtime_error("fake: two steps already in flight");
    queued_.push_back(std::move(out));
  }
  std::vector<int> batch_collect() override {
    std::lock_guard<std::mutex> g(mu_);
    if (queued_.empty()) throw std::runtime_error("fake: no step in flight");
    std::vector<int> out = std::move(queued_.front());
    queued_.pop_front();
    return out;
  }
  void set_pipeline(bool on) { pipeline_ = on; }
  long long prefilled() { std::lock_guard<std::mutex> g(mu_); return prefilled_; }
  long long steps() { std::lock_guard<std::mutex> g(mu_); return steps_; }
  int max_rows() { std::lock_guard<std::mutex> g(mu_); return max_rows_; }
  void fail_at(long long s) { std::lock_guard<std::mutex> g(mu_); fail_at_ = s; }

 private:
  int n_slots_, max_batch_, n_ctx_, vocab_, step_us_;
  std::mutex mu_;
  std::vector<std::vector<int>> kv_;
  std::vector<int> cur_;
  long long prefilled_ = 0, steps_ = 0, fail_at_ = 0, parts_ = 0;
  int chunk_ = 0;
  int max_rows_ = 0;
  bool pipeline_ = false;
  std::deque<std::vector<int>> queued_;
};

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "C++ CPU backend (OpenMP): GGUF engine for n_gpu_layers = 0";
  py::class_<CpuEngine>(m, "CpuEngine")
      .def(py::init([](const std::string& path, int n_ctx, int n_threads, int n_batch, int tp_rank, int tp_size,
                       int layer_end, bool load_head, const std::vector<float>& tensor_split) {
             CpuOptions o;
             o.n_ctx = n_ctx;
             o.n_threads = n_threads;
             o.n_batch = n_batch;
             o.tp_rank = tp_rank;
             o.tp_size = tp_size;
             o.layer_end = layer_end;
             o.load_head = load_head;
             o.tensor_split = tensor_split;
             py::gil_scoped_release nogil;
             return std::make_unique<CpuEngine>(path, o);
           }),
           py::arg("path"), py::arg("n_ctx") = 512, py::arg("n_threads") = 0, py::arg("n_batch") = 64,
           py::arg("tp_rank") = 0, py::arg("tp_size") = 1, py::arg("layer_end") = -1, py::arg("load_head") = true,
           py::arg("tensor_split") = std::vector<float>{})
      .def("set_comm",
           [](CpuEngine& e, py::object allreduce, py::object allgather) {
             // callbacks get numpy views of the engine's buffers (no copy); they run with the GIL held
             auto ar = [allreduce](float* buf, size_t n) {
               py::gil_scoped_acquire g;
               py::array_t<float> a({(py::ssize_t)n}, {(py::ssize_t)sizeof(float)}, buf, py::none());
               allreduce(a);
             };
             auto ag = [allgather](const float* loc, float* all, size_t n) {
               py::gil_scoped_acquire g;
               py::array_t<float> a({(py::ssize_t)n}, {(py::ssize_t)sizeof(float)}, const_cast<float*>(loc),
                                    py::none());
               py::array_t<float> out = allgather(a).cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
               std::memcpy(all, out.data(), sizeof(float) * out.size());
             };
             e.set_comm(ar, ag);
           })
      .def("eval_hidden",
           [](CpuEngine& e, const std::vector<int>& tokens, int pos0) {
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.eval_hidden(tokens, pos0);
             }
             py::array_t<float> a({(py::ssize_t)tokens.size(), (py::ssize_t)(v.size() / tokens.size())});
             std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(float));
             return a;
           })
      .def("kv_state_bytes", &CpuEngine::kv_state_bytes)
      .def("kv_save",
           [](CpuEngine& e, int n) {
             py::array_t<uint8_t> a((py::ssize_t)e.kv_state_bytes(n));
             e.kv_transfer(a.mutable_data(), n, false);
             return a;
           })
      .def("kv_load",
           [](CpuEngine& e, py::array_t<uint8_t, py::array::c_style> a, int n) {
             if ((size_t)a.size() != e.kv_state_bytes(n)) throw std::runtime_error("kv_load: size mismatch");
             e.kv_transfer(const_cast<uint8_t*>(a.data()), n, true);
           })
      .def_property_readonly("layer_end", &CpuEngine::layer_end)
      .def_property_readonly("n_embd", &CpuEngine::n_embd)
      .def_property_readonly("tp_rank", &CpuEngine::tp_rank)
      .def_property_readonly("tp_size", &CpuEngine::tp_size)
      .def("generate",
           [](CpuEngine& e, const std::vector<int>& prompt, int n_keep, int max_new, py::dict sp,
              const std::vector<int>& stop, py::object poll, py::object on_token) {
             CpuSampling o = parse_sampling(sp);
             std::function<bool()> pf;
             std::function<void(int)> tf;
             if (!poll.is_none()) pf = [poll]() { py::gil_scoped_acquire g; return poll().cast<bool>(); };
             if (!on_token.is_none()) tf = [on_token](int t) { py::gil_scoped_acquire g; on_token(t); };
             CpuGenOut r;
             {
               py::gil_scoped_release nogil;
               r = e.generate(prompt, n_keep, max_new, o, stop, pf, tf);
             }
             py::dict d;
             d["tokens"] = r.tokens;
             d["finish"] = r.finish;
             d["n_evaluated"] = r.n_evaluated;
             d["n_prefilled"] = r.n_prefilled;
             d["prefill_s"] = r.prefill_s;
             d["decode_s"] = r.decode_s;
             return d;
           },
           py::arg("prompt"), py::arg("n_keep"), py::arg("max_new"), py::arg("sampling"), py::arg("stop_ids"),
           py::arg("poll") = py::none(), py::arg("on_token") = py::none())
      .def("eval_logits",
           [](CpuEngine& e, const std::vector<int>& tokens, int pos0) {
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.eval_logits(tokens, pos0);
             }
             return py::array_t<float>(v.size(), v.data());
           })
      .def_property_readonly("n_vocab", &CpuEngine::n_vocab)
      .def_property_readonly("n_layer", &CpuEngine::n_layer)
      .def_property_readonly("n_ctx", &CpuEngine::n_ctx);

  m.def("sample", [](py::array_t<float, py::array::c_style> logits, const std::vector<int>& window, py::dict sp,
                     int step) {
    std::vector<float> l(logits.data(), logits.data() + logits.size());
    return cpu_sample(l, window, parse_sampling(sp), step);
  });
  m.def("uniform", &splitmix_uniform);

  py::class_<FakeSlotEngine>(m, "FakeSlotEngine")
      .def(py::init<int, int, int, int, int>(), py::arg("n_slots"), py::arg("max_batch"), py::arg("n_ctx"),
           py::arg("vocab") = 1000, py::arg("step_us") = 0)
      .def_static("next_token", &FakeSlotEngine::next_token)
      .def_property_readonly("prefilled", &FakeSlotEngine::prefilled)
      .def_property_readonly("steps", &FakeSlotEngine::steps)
      .def_property_readonly("max_rows", &FakeSlotEngine::max_rows)
      .def("fail_at", &FakeSlotEngine::fail_at)
      .def("set_pipeline", &FakeSlotEngine::set_pipeline)
      .def("set_prefill_chunk", &FakeSlotEngine::set_prefill_chunk)
      .def_property_readonly("parts", &FakeSlotEngine::parts);
  bind_scheduler<FakeSlotEngine>(m);

  // the tensor-parallel control channel (runtime/tp_channel.h), for host-side tests of its
  // ordering / acknowledgement / leader-liveness semantics across processes
  py::class_<TPChannel>(m, "TPChannel")
      .def_static("create", [](const std::string& name, int world, size_t cap) {
        return TPChannel::create(name, world, cap);
      })
      .def_static("attach", [](const std::string& name, int rank) { return TPChannel::attach(name, rank); })
      .def("publish", [](TPChannel& c, py::bytes b) {
        TPMsg m;
        const std::string v(b);
        m.buf.assign(v.begin(), v.end());
        py::gil_scoped_release nogil;
        c.publish(m);
      })
      .def("receive", [](TPChannel& c, int timeout_ms) -> py::object {
        TPMsg m;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = c.receive(m, timeout_ms);
        }
        if (!ok) return py::none();
        return py::bytes(reinterpret_cast<const char*>(m.buf.data()), m.buf.size());
      })
      .def("leader_alive", &TPChannel::leader_alive)
      .def_property_readonly("world", &TPChannel::world);
}
