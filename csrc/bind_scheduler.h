// pybind11 surface of the continuous-batching scheduler, shared by the _hip module (over
// the MI355X Engine) and the _cpu module (over a deterministic stand-in used by the tests).
// Types are module-local: each extension registers its own copy.
#pragma once
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime/scheduler.h"

namespace lfk {

inline SamplingOpts sampling_opts_from(pybind11::dict sp) {
  namespace py = pybind11;
  SamplingOpts o;
  o.top_k = sp.contains("top_k") ? sp["top_k"].cast<int>() : 40;
  o.top_p = sp.contains("top_p") ? sp["top_p"].cast<float>() : 0.95f;
  o.min_p = sp.contains("min_p") ? sp["min_p"].cast<float>() : 0.05f;
  o.temp = sp.contains("temperature") ? sp["temperature"].cast<float>() : 0.8f;
  o.repeat_penalty = sp.contains("repeat_penalty") ? sp["repeat_penalty"].cast<float>() : 1.1f;
  o.freq_penalty = sp.contains("frequency_penalty") ? sp["frequency_penalty"].cast<float>() : 0.f;
  o.presence_penalty = sp.contains("presence_penalty") ? sp["presence_penalty"].cast<float>() : 0.f;
  o.last_n = sp.contains("last_n") ? sp["last_n"].cast<int>() : 64;
  o.seed = sp.contains("seed") ? sp["seed"].cast<unsigned long long>() : 0ull;
  o.tfs_z = sp.contains("tfs_z") ? sp["tfs_z"].cast<float>() : 1.f;
  o.typical_p = sp.contains("typical_p") ? sp["typical_p"].cast<float>() : 1.f;
  if (sp.contains("logit_bias"))
    for (auto kv : sp["logit_bias"].cast<py::dict>())
      o.logit_bias.emplace_back(kv.first.cast<int>(), kv.second.cast<float>());
  return o;
}

// Backend: the pybind-registered class of the slot engine the scheduler is built over.
template <class Backend>
void bind_scheduler(pybind11::module_& m) {
  namespace py = pybind11;
  py::class_<BatchScheduler>(m, "BatchScheduler", py::module_local())
      .def(py::init([](Backend& e) { return std::make_unique<BatchScheduler>(e); }), py::arg("engine"),
           py::keep_alive<1, 2>())
      .def("submit",
           [](BatchScheduler& b, const std::vector<int>& prompt, int max_new, py::dict sp,
              const std::vector<int>& stop_ids) {
             const SamplingOpts o = sampling_opts_from(sp);
             py::gil_scoped_release nogil;
             return b.submit(prompt, max_new, o, stop_ids);
           },
           py::arg("prompt"), py::arg("max_new"), py::arg("sampling"), py::arg("stop_ids"))
      .def("wait",
           [](BatchScheduler& b, int64_t id, size_t have, int timeout_ms) {
             SchedPoll p;
             {
               py::gil_scoped_release nogil;
               p = b.wait(id, have, timeout_ms);
             }
             py::dict d;
             d["tokens"] = p.tokens;
             d["done"] = p.done;
             d["finish"] = p.finish;
             d["error"] = p.error;
             d["n_prompt"] = p.n_prompt;
             d["n_prefilled"] = p.n_prefilled;
             d["queue_s"] = p.queue_s;
             d["prefill_s"] = p.prefill_s;
             d["decode_s"] = p.decode_s;
             return d;
           },
           py::arg("id"), py::arg("have") = 0, py::arg("timeout_ms") = 50)
      .def("cancel", &BatchScheduler::cancel)
      .def("release", &BatchScheduler::release)
      .def("stats",
           [](BatchScheduler& b) {
             const SchedStats s = b.stats();
             py::dict d;
             d["steps"] = s.steps;
             d["rows"] = s.rows;
             d["admitted"] = s.admitted;
             d["reused_tokens"] = s.reused_tokens;
             d["joint_admissions"] = s.joint_admissions;
             d["chunked_admissions"] = s.chunked_admissions;
             d["active"] = s.active;
             d["pending"] = s.pending;
             d["slots"] = s.slots;
             return d;
           })
      .def("shutdown", [](BatchScheduler& b) {
        py::gil_scoped_release nogil;
        b.shutdown();
      });
}

}  // namespace lfk
