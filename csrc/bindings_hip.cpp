// Python bindings of the MI355X runtime (`llama_fastapi_k8s_gpu_amd.runtime._hip`).
//
// Two surfaces:
//   * Engine      - the serving engine (load, generate, test hooks); the GIL is
//                   released for the whole generation loop and re-acquired only
//                   for the optional per-token callback / cancel poll.
//   * kernel hooks - thin wrappers taking raw device pointers (torch
//                   `data_ptr()`) and a stream handle, used by the numerics tests
//                   that compare each kernel with a PyTorch fp32 reference.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>

#include "bind_scheduler.h"
#include "kernels/kernels.h"
#include "runtime/engine.h"
#include "runtime/repack.h"

namespace py = pybind11;
using namespace lfk;

template <class T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void hip_ok(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static SamplingOpts sampling_opts(py::dict sp) { return sampling_opts_from(sp); }

PYBIND11_MODULE(_hip, m) {
  m.doc() = "MI355X (gfx950) runtime: GGUF engine + HIP kernels";

  py::class_<Engine>(m, "Engine")
      .def(py::init([](const std::string& path, int n_ctx, int n_batch, int device, bool use_graph, int tp_rank,
                       int tp_size, py::bytes nccl_id, int layer_begin, const std::vector<float>& tensor_split,
                       int n_slots, const std::string& comm, int layer_end, const std::string& test_fault) {
             EngineOptions o;
             o.test_fault = test_fault;
             o.layer_begin = layer_begin;
             o.layer_end = layer_end;
             o.n_slots = n_slots;
             o.n_ctx = n_ctx;
             o.n_batch = n_batch;
             o.device = device;
             o.use_graph = use_graph;
             o.tp_rank = tp_rank;
             o.tp_size = tp_size;
             o.nccl_id = std::string(nccl_id);
             o.tensor_split = tensor_split;
             o.comm = comm;
             py::gil_scoped_release nogil;
             return std::make_unique<Engine>(path, o);
           }),
           py::arg("path"), py::arg("n_ctx") = 1024, py::arg("n_batch") = 512, py::arg("device") = 0,
           py::arg("use_graph") = true, py::arg("tp_rank") = 0, py::arg("tp_size") = 1,
           py::arg("nccl_id") = py::bytes(""), py::arg("layer_begin") = 0,
           py::arg("tensor_split") = std::vector<float>{}, py::arg("n_slots") = 1, py::arg("comm") = "auto",
           py::arg("layer_end") = -1, py::arg("test_fault") = "")
      .def(
          "generate",
          [](Engine& e, const std::vector<int>& prompt, int n_keep, int max_new, py::dict sp,
             const std::vector<int>& stop_ids, py::object poll, py::object on_token) {
            const SamplingOpts o = sampling_opts(sp);
            std::function<bool()> pf;
            std::function<void(int)> tf;
            if (!poll.is_none()) pf = [poll]() { py::gil_scoped_acquire g; return poll().cast<bool>(); };
            if (!on_token.is_none()) tf = [on_token](int t) { py::gil_scoped_acquire g; on_token(t); };
            GenOut r;
            {
              py::gil_scoped_release nogil;
              r = e.generate(prompt, n_keep, max_new, o, stop_ids, pf, tf);
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
           [](Engine& e, const std::vector<int>& tokens, int pos0) {
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.eval_logits(tokens, pos0);
             }
             return py::array_t<float>(v.size(), v.data());
           })
      .def("eval_hidden",
           [](Engine& e, py::array_t<float, py::array::c_style | py::array::forcecast> x, int pos0) {
             if (x.ndim() != 2 || x.shape(1) != e.hparams().n_embd)
               throw std::runtime_error("eval_hidden: x must be [T, n_embd]");
             std::vector<float> v;
             const int T = (int)x.shape(0);
             const float* ptr = x.data();
             {
               py::gil_scoped_release nogil;
               v = e.eval_hidden(ptr, T, pos0);
             }
             return py::array_t<float>(v.size(), v.data());
           })
      .def_property_readonly("layer_begin", &Engine::layer_begin)
      .def_property_readonly("layer_end", &Engine::layer_end)
      .def_property_readonly("has_head", &Engine::has_head)
      .def("eval_stage",
           [](Engine& e, py::object x, std::vector<int> tokens, int pos0, bool to_host) {
             std::vector<float> v;
             int T = (int)tokens.size();
             if (!x.is_none()) {
               auto a = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(x);
               if (!a || a.ndim() != 2 || a.shape(1) != e.hparams().n_embd)
                 throw std::runtime_error("eval_stage: x must be [T, n_embd]");
               T = (int)a.shape(0);
               const float* ptr = a.data();
               py::gil_scoped_release nogil;
               v = e.eval_stage(ptr, nullptr, T, pos0, to_host);
             } else {
               py::gil_scoped_release nogil;
               v = e.eval_stage(nullptr, tokens.data(), T, pos0, to_host);
             }
             const bool hidden = !e.has_head() && to_host;
             py::array_t<float> out(v.size(), v.data());
             if (hidden) out.resize({(py::ssize_t)T, (py::ssize_t)e.hparams().n_embd});
             return out;
           },
           py::arg("x"), py::arg("tokens") = std::vector<int>{}, py::arg("pos0") = 0, py::arg("to_host") = true)
      .def("eval_stage_peer",
           [](Engine& e, const Engine& prev, int T, int pos0) {
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.eval_stage_peer(prev, T, pos0);
             }
             return py::array_t<float>(v.size(), v.data());
           })
      .def("decode_logits",
           [](Engine& e, int token, int pos) {
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.decode_logits(token, pos);
             }
             return py::array_t<float>(v.size(), v.data());
           })
      .def_property_readonly("n_slots", &Engine::n_slots)
      .def_property_readonly("max_batch", &Engine::max_batch)
      .def_property_readonly("batch_gemv", &Engine::batch_gemv)
      .def_property_readonly("prefill_t16", &Engine::prefill_t16)
      .def("slot_begin",
           [](Engine& e, int slot, const std::vector<int>& prompt, int n_keep, py::dict sp) {
             const SamplingOpts o = sampling_opts(sp);
             py::gil_scoped_release nogil;
             return e.slot_begin(slot, prompt, n_keep, o);
           })
      .def("slot_begin_part",
           [](Engine& e, int slot, const std::vector<int>& prompt, int n_keep, int n_done, int n, py::dict sp) {
             const SamplingOpts o = sampling_opts(sp);
             py::gil_scoped_release nogil;
             return e.slot_begin_part(slot, prompt, n_keep, n_done, n, o);
           })
      .def_property_readonly("prefill_part_tokens", &Engine::prefill_part_tokens)
      .def("slots_begin",
           [](Engine& e, const std::vector<int>& slots, const std::vector<std::vector<int>>& prompts,
              const std::vector<int>& n_keep, py::list sps) {
             std::vector<SamplingOpts> o;
             for (auto h : sps) o.push_back(sampling_opts(h.cast<py::dict>()));
             py::gil_scoped_release nogil;
             return e.slots_begin(slots, prompts, n_keep, o);
           })
      .def("batch_step",
           [](Engine& e, const std::vector<int>& slots) {
             py::gil_scoped_release nogil;
             return e.batch_step(slots);
           })
      .def("batch_launch",
           [](Engine& e, const std::vector<int>& slots) {
             py::gil_scoped_release nogil;
             e.batch_launch(slots);
           })
      .def("batch_collect",
           [](Engine& e) {
             py::gil_scoped_release nogil;
             return e.batch_collect();
           })
      .def_property_readonly("can_pipeline", &Engine::can_pipeline)
      .def("batch_logits",
           [](Engine& e, int B) {
             std::vector<float> v = e.batch_logits(B);
             py::array_t<float> a({(py::ssize_t)B, (py::ssize_t)(v.size() / B)});
             std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(float));
             return a;
           })
      .def("step_clk", [](Engine& e) {
        std::vector<long long> v;
        {
          py::gil_scoped_release nogil;
          v = e.step_clk();
        }
        py::array_t<long long> out({(py::ssize_t)5, (py::ssize_t)Engine::kStepClkBlocks, (py::ssize_t)16});
        std::copy(v.begin(), v.end(), out.mutable_data());
        return out;
      })
      .def("step_clk_zero", &Engine::step_clk_zero)
      .def("kv_state_bytes", &Engine::kv_state_bytes)
      .def("kv_save",
           [](Engine& e, int n) {
             py::array_t<uint8_t> a((py::ssize_t)e.kv_state_bytes(n));
             void* p = a.mutable_data();
             {
               py::gil_scoped_release nogil;
               e.kv_transfer(p, n, false);
             }
             return a;
           })
      .def("kv_load",
           [](Engine& e, py::array_t<uint8_t, py::array::c_style> a, int n) {
             if ((size_t)a.size() != e.kv_state_bytes(n)) throw std::runtime_error("kv_load: size mismatch");
             void* p = const_cast<uint8_t*>(a.data());
             py::gil_scoped_release nogil;
             e.kv_transfer(p, n, true);
           })
      .def("kv_transfer_ptr",  // device (or pinned host) buffer of kv_state_bytes(n) bytes
           [](Engine& e, uintptr_t buf, int n, bool load) {
             py::gil_scoped_release nogil;
             e.kv_transfer(reinterpret_cast<void*>(buf), n, load);
           })
      .def("bench_decode",
           [](Engine& e, int n, int pos0) {
             double ms = 0;
             py::gil_scoped_release nogil;
             e.bench_decode(n, pos0, &ms);
             return ms;
           })
      .def("comm_info", [](Engine& e) {
        py::dict d;
        for (auto& kv : e.comm_info()) d[py::str(kv.first)] = kv.second;
        return d;
      })
      .def_property_readonly("device_bytes", &Engine::device_bytes)
      .def_property_readonly("healthy", &Engine::healthy)
      .def("p2p_handle", [](Engine& e) { return py::bytes(e.p2p_handle()); })
      .def("p2p_open", [](Engine& e, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (const auto& h : hs) v.push_back(std::string(h));
        e.p2p_open(v);
      })
      .def_property_readonly("p2p_ready", &Engine::p2p_ready)
      .def("tp_ctl_create", &Engine::tp_ctl_create)
      .def("tp_ctl_attach", &Engine::tp_ctl_attach)
      .def_property_readonly("tp_ctl_open", &Engine::tp_ctl_open)
      .def("follow", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.follow();
      })
      .def("tp_stop", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.tp_stop();
      })
      .def_property_readonly("last_error", &Engine::last_error)
      .def_property_readonly("n_ctx", &Engine::n_ctx)
      .def_property_readonly("tp_rank", &Engine::tp_rank)
      .def_property_readonly("tp_size", &Engine::tp_size)
      .def_property_readonly("hparams", [](const Engine& e) {
        const HParams& h = e.hparams();
        py::dict d;
        d["n_vocab"] = h.n_vocab; d["n_embd"] = h.n_embd; d["n_layer"] = h.n_layer; d["n_head"] = h.n_head;
        d["n_head_kv"] = h.n_head_kv; d["head_dim"] = h.head_dim; d["n_ff"] = h.n_ff;
        d["n_expert"] = h.n_expert; d["n_expert_used"] = h.n_expert_used;
        d["rope_base"] = h.rope_base; d["rms_eps"] = h.rms_eps;
        return d;
      });

  bind_scheduler<Engine>(m);

  m.def("nccl_unique_id", []() {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    return n;
  });

  // ------------------------------------------------------------------ kernel hooks (tests)
  m.def("repack", [](int type, py::array_t<uint8_t, py::array::c_style> src, size_t K_src, size_t r0, size_t R,
                     size_t c0, size_t K, size_t R_dst, int G, int off) {
    py::array_t<uint8_t> dst(qbytes(type, R_dst, K));
    std::memset(dst.mutable_data(), 0, dst.size());
    repack_planar(type, src.data(), K_src, r0, R, c0, K, dst.mutable_data(), R_dst, G, off);
    return dst;
  });
  m.def("qbytes", [](int type, size_t R, size_t K) { return qbytes(type, R, K); });

  m.def("gemv", [](uintptr_t w, int type, int rows, int K, uintptr_t x, uintptr_t norm, float eps, uintptr_t out,
                   int n_out, int epi, uintptr_t stream, int n_slots, uintptr_t ids, size_t expert_stride,
                   int slot_stride, uintptr_t resid, int debug, uintptr_t dbg_clk) {
    GemvArgs a;
    a.debug = debug;
    a.dbg_clk = P<long long>(dbg_clk);
    a.w = make_qmat(P<void>(w), type, rows, K, expert_stride);
    a.x = P<float>(x); a.norm_w = P<float>(norm); a.eps = eps; a.out = P<float>(out); a.n_out = n_out;
    a.n_slots = n_slots; a.expert_ids = P<int>(ids); a.out_slot_stride = slot_stride; a.resid = P<float>(resid);
    gemv(a, epi, S(stream));
    hip_ok("gemv");
  }, py::arg("w"), py::arg("type"), py::arg("rows"), py::arg("K"), py::arg("x"), py::arg("norm"), py::arg("eps"),
     py::arg("out"), py::arg("n_out"), py::arg("epi"), py::arg("stream"), py::arg("n_slots") = 1,
     py::arg("ids") = 0, py::arg("expert_stride") = 0, py::arg("slot_stride") = 0, py::arg("resid") = 0,
     py::arg("debug") = 0, py::arg("dbg_clk") = 0);

  // the row-parallel decode GEMV with its epilogue all-reduce (GemvArgs::tp_*) for ONE rank of a
  // group whose regions the caller laid out (tests/test_tp_epilogue_gpu.py: a single process
  // pre-writes the peers' granules and fault words, so any world size runs on one GPU)
  m.def("gemv_tp", [](uintptr_t w, int type, int rows, int K, uintptr_t x, uintptr_t out, int n_out, uintptr_t resid,
                      const std::vector<uintptr_t>& data, const std::vector<uintptr_t>& fault, int rank, int stride,
                      int off, uintptr_t epochs, uintptr_t err, uintptr_t stream) {
    const int W = (int)data.size();
    if (W < 1 || W > kP2PMaxRanks || (int)fault.size() != W || rank < 0 || rank >= W || stride < n_out + off)
      throw std::runtime_error("gemv_tp: bad group layout");
    GemvArgs a;
    a.w = make_qmat(P<void>(w), type, rows, K, 0);
    a.x = P<float>(x); a.out = P<float>(out); a.n_out = n_out; a.resid = P<float>(resid);
    for (int p = 0; p < W; ++p) {
      a.tp_peers.data[p] = P<float>(data[p]);
      a.tp_peers.fault[p] = P<int>(fault[p]);
    }
    a.tp_world = W; a.tp_rank = rank; a.tp_stride = stride; a.tp_off = off;
    a.tp_epochs = P<int>(epochs); a.tp_err = P<int>(err);
    gemv(a, EPI_STORE, S(stream));
    hip_ok("gemv_tp");
  });

  m.def("bprep", [](uintptr_t x, int ldx, bool swiglu, uintptr_t norm, float eps, int K, int B, uintptr_t xh, int ldh,
                    uintptr_t stream, uintptr_t zero, int zero_n, int swiglu_group) {
    BPrepArgs a;
    a.swiglu_group = swiglu_group;
    a.x = P<float>(x); a.ldx = ldx; a.swiglu = swiglu; a.norm_w = P<float>(norm); a.eps = eps; a.K = K; a.B = B;
    a.xh = P<__half>(xh); a.ldh = ldh; a.zero = P<float>(zero); a.zero_n = zero_n;
    bprep(a, S(stream));
    hip_ok("bprep");
  }, py::arg("x"), py::arg("ldx"), py::arg("swiglu"), py::arg("norm"), py::arg("eps"), py::arg("K"), py::arg("B"),
     py::arg("xh"), py::arg("ldh"), py::arg("stream"), py::arg("zero") = 0, py::arg("zero_n") = 0,
     py::arg("swiglu_group") = 32);
  m.def("bmm", [](uintptr_t w, int type, int rows, int K, uintptr_t xh, int ldh, uintptr_t out, int ldo, int B,
                  uintptr_t stream, int debug, uintptr_t h_out, int ldh_out, uintptr_t xf, int ldxf,
                  uintptr_t norm, float eps, bool store_out, uintptr_t dbg_clk) {
    BmmArgs a;
    a.debug = debug;
    a.dbg_clk = P<long long>(dbg_clk);
    a.w = make_qmat(P<void>(w), type, rows, K);
    a.xh = P<__half>(xh); a.ldh = ldh; a.out = P<float>(out); a.ldo = ldo; a.n_out = rows; a.B = B;
    if (h_out) {  // SwiGLU epilogue (gate/up rows in 32-row groups)
      a.swiglu_epi = true; a.h_out = P<__half>(h_out); a.ldh_out = ldh_out;
    }
    if (xf) {     // RMSNorm folded into the staging (fp32 rows xf, weights norm)
      a.xf = P<float>(xf); a.ldxf = ldxf; a.norm_w = P<float>(norm); a.eps = eps;
    }
    a.store_out = store_out;
    bmm(a, S(stream));
    hip_ok("bmm");
  }, py::arg("w"), py::arg("type"), py::arg("rows"), py::arg("K"), py::arg("xh"), py::arg("ldh"), py::arg("out"),
     py::arg("ldo"), py::arg("B"), py::arg("stream"), py::arg("debug") = 0, py::arg("h_out") = 0,
     py::arg("ldh_out") = 0, py::arg("xf") = 0, py::arg("ldxf") = 0, py::arg("norm") = 0, py::arg("eps") = 1e-5f,
     py::arg("store_out") = false, py::arg("dbg_clk") = 0);
  // the gate/up + down chain in one launch (tests/test_kernels_gpu.py::test_bmm_ffn_chain_*): gate/up
  // rows in the SwiGLU tile16 copy (wg, 2F x K), down (wd, K x F) over the f16 SwiGLU output hout
  // [B][F]; out [B][K] accumulates; cnt >= 64 ints, zeroed by the caller
  m.def("chain_layout", []() { return std::make_tuple(kChainStride, kChainXcds, kChainInts); });
  m.def("bmm_ffn_chain", [](uintptr_t wg, int tg, int F, int K, uintptr_t xh, uintptr_t xf, uintptr_t norm, float eps,
                            uintptr_t wd, int td, uintptr_t hout, uintptr_t out, int B, uintptr_t cnt,
                            uintptr_t stream) {
    BmmArgs gu, dn;
    gu.w = make_qmat(P<void>(wg), tg, 2 * F, K);
    gu.xh = P<__half>(xh); gu.ldh = K; gu.n_out = 2 * F; gu.B = B;
    gu.swiglu_epi = true; gu.h_out = P<__half>(hout); gu.ldh_out = F;
    if (xf) {
      gu.xf = P<float>(xf); gu.ldxf = K; gu.norm_w = P<float>(norm); gu.eps = eps;
    }
    dn.w = make_qmat(P<void>(wd), td, K, F);
    dn.xh = P<__half>(hout); dn.ldh = F; dn.out = P<float>(out); dn.ldo = K; dn.n_out = K; dn.B = B;
    if (!bmm_ffn_chain_supported(gu, dn)) throw std::runtime_error("bmm_ffn_chain: unsupported shapes");
    bmm_ffn_chain(gu, dn, P<int>(cnt), nullptr, S(stream));
    hip_ok("bmm_ffn_chain");
  }, py::arg("wg"), py::arg("tg"), py::arg("F"), py::arg("K"), py::arg("xh"), py::arg("xf"), py::arg("norm"),
     py::arg("eps"), py::arg("wd"), py::arg("td"), py::arg("hout"), py::arg("out"), py::arg("B"), py::arg("cnt"),
     py::arg("stream"));
  // Wo -> gate/up -> down in one launch (tests/test_kernels_gpu.py::test_bmm_wo_ffn_chain_*): Wo adds
  // W_o . xa into the residual rows `resid`, the gate/up stages norm(resid), the down adds into resid
  m.def("bmm_wo_ffn_chain", [](uintptr_t wo, int to, int Kwo, uintptr_t xa, uintptr_t wg, int tg, int F, int K,
                               uintptr_t norm, float eps, uintptr_t wd, int td, uintptr_t xh, uintptr_t hout,
                               uintptr_t resid, int B, uintptr_t cnt, uintptr_t stream) {
    BmmArgs o, gu, dn;
    o.w = make_qmat(P<void>(wo), to, K, Kwo);
    o.xh = P<__half>(xa); o.ldh = Kwo; o.out = P<float>(resid); o.ldo = K; o.n_out = K; o.B = B;
    gu.w = make_qmat(P<void>(wg), tg, 2 * F, K);
    gu.xh = P<__half>(xh); gu.ldh = K; gu.n_out = 2 * F; gu.B = B;
    gu.swiglu_epi = true; gu.h_out = P<__half>(hout); gu.ldh_out = F;
    gu.xf = P<float>(resid); gu.ldxf = K; gu.norm_w = P<float>(norm); gu.eps = eps;
    dn.w = make_qmat(P<void>(wd), td, K, F);
    dn.xh = P<__half>(hout); dn.ldh = F; dn.out = P<float>(resid); dn.ldo = K; dn.n_out = K; dn.B = B;
    if (!bmm_wo_ffn_chain_supported(o, gu, dn)) throw std::runtime_error("bmm_wo_ffn_chain: unsupported shapes");
    bmm_wo_ffn_chain(o, gu, dn, P<int>(cnt), nullptr, S(stream));
    hip_ok("bmm_wo_ffn_chain");
  }, py::arg("wo"), py::arg("to"), py::arg("Kwo"), py::arg("xa"), py::arg("wg"), py::arg("tg"), py::arg("F"),
     py::arg("K"), py::arg("norm"), py::arg("eps"), py::arg("wd"), py::arg("td"), py::arg("xh"), py::arg("hout"),
     py::arg("resid"), py::arg("B"), py::arg("cnt"), py::arg("stream"));
  m.def("bmm_norm_fits", &bmm_norm_fits);
  m.def("bmm_supported", &bmm_supported);
  m.def("t16_bytes", &t16_bytes);
  m.def("t16_repack", [](uintptr_t w, int type, int rows, int K, uintptr_t dst, uintptr_t stream, bool swiglu) {
    t16_repack(make_qmat(P<void>(w), type, rows, K), P<uint8_t>(dst), S(stream), swiglu);
    hip_ok("t16_repack");
  }, py::arg("w"), py::arg("type"), py::arg("rows"), py::arg("K"), py::arg("dst"), py::arg("stream"),
     py::arg("swiglu") = false);

  py::class_<P2PComm>(m, "P2PComm")
      .def(py::init<int, int, int, int, bool>(), py::arg("rank"), py::arg("world"), py::arg("max_n"), py::arg("device"),
           py::arg("uncached") = true)
      .def("handle", [](const P2PComm& c) { return py::bytes(c.handle()); })
      .def("open", [](P2PComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (const auto& h : hs) v.push_back(std::string(h));
        c.open(v);
      })
      .def("allreduce", [](P2PComm& c, uintptr_t src, uintptr_t dst, int n, uintptr_t stream) {
        c.allreduce(P<float>(src), P<float>(dst), n, S(stream));
        hip_ok("p2p_allreduce");
      })
      .def("allreduce_add", [](P2PComm& c, uintptr_t src, uintptr_t dst, int n, uintptr_t stream) {
        c.allreduce_add(P<float>(src), P<float>(dst), n, S(stream));
        hip_ok("p2p_allreduce_add");
      })
      .def("allgather", [](P2PComm& c, uintptr_t src, uintptr_t dst, int n, uintptr_t stream) {
        c.allgather(P<float>(src), P<float>(dst), n, S(stream));
        hip_ok("p2p_allgather");
      })
      .def("error", &P2PComm::error)
      .def_property_readonly("uncached", &P2PComm::uncached)
      .def("mappings", &P2PComm::mappings)
      .def("reset_error", &P2PComm::reset_error);

  m.def("gemv_qkv", [](uintptr_t wq, int tq, uintptr_t wk, int tk, uintptr_t wv, int tv, int nq, int nkv, int K,
                       uintptr_t x, uintptr_t norm, float eps, uintptr_t q_out, uintptr_t kc, uintptr_t vc, int n_ctx,
                       int hd, uintptr_t pos, uintptr_t rope, uintptr_t stream) {
    QkvArgs a;
    a.wq = make_qmat(P<void>(wq), tq, nq, K);
    a.wk = make_qmat(P<void>(wk), tk, nkv, K);
    a.wv = make_qmat(P<void>(wv), tv, nkv, K);
    a.x = P<float>(x); a.norm_w = P<float>(norm); a.eps = eps; a.q_out = P<float>(q_out);
    a.k_cache = P<__half>(kc); a.v_cache = P<__half>(vc); a.n_ctx = n_ctx; a.head_dim = hd;
    a.pos = P<int>(pos); a.rope = P<float2>(rope);
    gemv_qkv(a, S(stream));
    hip_ok("gemv_qkv");
  });

  m.def("moe_down", [](uintptr_t w, int type, int rows, int K, size_t expert_stride, uintptr_t h, uintptr_t ids,
                       uintptr_t ew, int n_slots, uintptr_t out, uintptr_t stream) {
    MoeDownArgs a;
    a.w = make_qmat(P<void>(w), type, rows, K, expert_stride);
    a.h = P<float>(h); a.expert_ids = P<int>(ids); a.expert_w = P<float>(ew); a.n_slots = n_slots;
    a.out = P<float>(out);
    gemv_moe_down(a, S(stream));
    hip_ok("moe_down");
  });
  m.def("moe_route", [](uintptr_t logits, int E, int k, uintptr_t ids, uintptr_t w, uintptr_t stream) {
    moe_route(P<float>(logits), E, k, P<int>(ids), P<float>(w), S(stream));
    hip_ok("moe_route");
  });

  m.def("gemm", [](uintptr_t w, int type, int rows, int K, uintptr_t x, int T, uintptr_t out, uintptr_t out_bf16,
                   int ldo, int epi, uintptr_t stream, uintptr_t resid) {
    GemmArgs a;
    a.w = make_qmat(P<void>(w), type, rows, K);
    a.x = P<__hip_bfloat16>(x); a.T = T; a.out = P<float>(out); a.out_bf16 = P<__hip_bfloat16>(out_bf16);
    a.ldo = ldo; a.resid = P<float>(resid);
    gemm_dq(a, epi, S(stream));
    hip_ok("gemm");
  }, py::arg("w"), py::arg("type"), py::arg("rows"), py::arg("K"), py::arg("x"), py::arg("T"), py::arg("out"),
     py::arg("out_bf16"), py::arg("ldo"), py::arg("epi"), py::arg("stream"), py::arg("resid") = 0);

  m.def("moe_router_rows", [](uintptr_t x, int ldx, int B, uintptr_t nw, float eps, uintptr_t W, int d, int E, int k,
                              uintptr_t wd, int ld, uintptr_t stream) {
    moe_router_rows(P<float>(x), ldx, B, P<float>(nw), eps, P<float>(W), d, E, k, P<float>(wd), ld, S(stream));
    hip_ok("moe_router_rows");
  }, py::arg("x"), py::arg("ldx"), py::arg("B"), py::arg("nw"), py::arg("eps"), py::arg("W"), py::arg("d"),
     py::arg("E"), py::arg("k"), py::arg("wd"), py::arg("ld"), py::arg("stream"));

  // layer split (split_mode=layer): the whole generation over a chain of stage engines, natively
  m.def("chain_generate",
        [](std::vector<Engine*> stages, const std::vector<int>& prompt, int n_keep, int max_new, py::dict sp,
           const std::vector<int>& stop_ids, py::object poll, py::object on_token) {
          const SamplingOpts o = sampling_opts(sp);
          std::function<bool()> pf;
          std::function<void(int)> tf;
          if (!poll.is_none()) pf = [poll]() { py::gil_scoped_acquire g; return poll().cast<bool>(); };
          if (!on_token.is_none()) tf = [on_token](int t) { py::gil_scoped_acquire g; on_token(t); };
          GenOut r;
          {
            py::gil_scoped_release nogil;
            r = Engine::chain_generate(stages, prompt, n_keep, max_new, o, stop_ids, pf, tf);
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
        py::arg("stages"), py::arg("prompt"), py::arg("n_keep"), py::arg("max_new"), py::arg("sampling"),
        py::arg("stop_ids"), py::arg("poll") = py::none(), py::arg("on_token") = py::none());

  m.def("gemm_t16", [](uintptr_t w, int type, int rows, int K, uintptr_t x, int T, uintptr_t out, int ldo,
                       uintptr_t out_h, int ldh, int epi, uintptr_t stream, uintptr_t resid, int cfg,
                       std::vector<std::pair<uintptr_t, int>> wseg) {
    GemmT16Args a;
    a.w = make_qmat(P<void>(w), type, rows, K);
    a.x = P<__half>(x); a.T = T; a.out = P<float>(out); a.ldo = ldo; a.resid = P<float>(resid);
    a.out_h = P<__half>(out_h); a.ldh = ldh; a.cfg = cfg;
    if (!wseg.empty()) {  // stacked matrices: (tile16 base, rows) per segment, the first = w
      if (wseg.size() > 3) throw std::runtime_error("gemm_t16: at most 3 segments");
      a.nwseg = (int)wseg.size();
      for (int i = 0; i < a.nwseg; ++i) {
        a.wseg_base[i] = P<uint8_t>(wseg[i].first);
        a.wseg_tiles[i] = wseg[i].second / 16;
      }
    }
    gemm_t16(a, epi, S(stream));
    hip_ok("gemm_t16");
  }, py::arg("w"), py::arg("type"), py::arg("rows"), py::arg("K"), py::arg("x"), py::arg("T"), py::arg("out"),
     py::arg("ldo"), py::arg("out_h"), py::arg("ldh"), py::arg("epi"), py::arg("stream"), py::arg("resid") = 0,
     py::arg("cfg") = 0, py::arg("wseg") = std::vector<std::pair<uintptr_t, int>>{});

  m.def("attn_decode", [](uintptr_t q, uintptr_t kc, uintptr_t vc, uintptr_t pos, int n_ctx, int n_head, int n_kv,
                          int hd, float scale, uintptr_t part, uintptr_t out, uintptr_t stream, uintptr_t counters,
                          int debug_stop, uintptr_t dbg_clk, int batch, uintptr_t slots, size_t slot_stride,
                          uintptr_t out_h, uintptr_t qkv_raw, size_t qkv_ld, size_t k_off, size_t v_off, uintptr_t ss,
                          float inv_k, float eps, uintptr_t rope_freq) {
    AttnDecodeArgs a;
    a.rope_freq = P<float>(rope_freq);
    a.qkv_raw = P<float>(qkv_raw); a.qkv_ld = qkv_ld; a.k_off = k_off; a.v_off = v_off;
    a.ss = P<float>(ss); a.inv_k = inv_k; a.eps = eps;
    if (batch > 0) {  // rows b: query q + b*n_head*hd, slot slots[b], position pos[b], own workspaces
      a.batch = batch; a.slots = P<int>(slots); a.slot_stride = slot_stride;
      a.q_stride = (size_t)n_head * hd; a.out_stride = (size_t)n_head * hd;
      a.part_stride = attn_decode_workspace_floats(n_ctx, n_head, hd);
      a.out_h = P<__half>(out_h); a.out_h_stride = (size_t)n_head * hd;
    }
    a.debug_stop = debug_stop;
    a.dbg_clk = P<long long>(dbg_clk);
    a.counters = P<int>(counters);
    a.q = P<float>(q); a.k_cache = P<__half>(kc); a.v_cache = P<__half>(vc); a.pos = P<int>(pos);
    a.n_ctx = n_ctx; a.n_head = n_head; a.n_kv_head = n_kv; a.head_dim = hd; a.scale = scale;
    a.part = P<float>(part); a.out = P<float>(out);
    attn_decode(a, S(stream));
    hip_ok("attn_decode");
  }, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("pos"), py::arg("n_ctx"), py::arg("n_head"), py::arg("n_kv"),
     py::arg("hd"), py::arg("scale"), py::arg("part"), py::arg("out"), py::arg("stream"), py::arg("counters"),
     py::arg("debug_stop") = 0, py::arg("dbg_clk") = 0, py::arg("batch") = 0, py::arg("slots") = 0,
     py::arg("slot_stride") = 0, py::arg("out_h") = 0, py::arg("qkv_raw") = 0, py::arg("qkv_ld") = 0,
     py::arg("k_off") = 0, py::arg("v_off") = 0, py::arg("ss") = 0, py::arg("inv_k") = 0.f, py::arg("eps") = 1e-5f,
     py::arg("rope_freq") = 0);
  // split-K Q|K|V (BmmArgs::qkv_sk) over tile16 copies: RoPE'd partial sums added into out [B][ldo]
  // (Q at 0, K at nq, V at nq + nkv), the rows' sums of squares into ss_out [B]
  m.def("bmm_qkv_sk", [](uintptr_t wq, int tq, int nq, uintptr_t wk, int tk, uintptr_t wv, int tv, int nkv, int K,
                         uintptr_t xf, int ldxf, uintptr_t norm, float eps, int B, uintptr_t out, int ldo,
                         uintptr_t ss_out, uintptr_t pos, uintptr_t rope, int head_dim, int n_ctx, uintptr_t stream,
                         uintptr_t zero, int zero_n, uintptr_t dbg_clk) {
    BmmArgs a;
    a.w = make_qmat(P<void>(wq), tq, nq, K); a.n_out = nq; a.out = P<float>(out); a.ldo = ldo; a.B = B;
    a.nseg = 3;
    a.seg_base[1] = P<uint8_t>(wk); a.seg_rows[1] = nkv; a.seg_out[1] = P<float>(out) + nq;
    a.seg_base[2] = P<uint8_t>(wv); a.seg_rows[2] = nkv; a.seg_out[2] = P<float>(out) + nq + nkv;
    a.seg_split = tk != tq ? 1 : tv != tq ? 2 : 3;
    a.type2 = tk != tq ? tk : tv != tq ? tv : 0;
    a.qkv_sk = true;
    a.qkv.pos = P<int>(pos); a.qkv.rope = P<float2>(rope); a.qkv.head_dim = head_dim; a.qkv.n_ctx = n_ctx;
    a.xf = P<float>(xf); a.ldxf = ldxf; a.norm_w = P<float>(norm); a.eps = eps; a.ss_out = P<float>(ss_out);
    a.zero = P<float>(zero); a.zero_n = zero_n;
    a.dbg_clk = P<long long>(dbg_clk);
    bmm(a, S(stream));
    hip_ok("bmm_qkv_sk");
  }, py::arg("wq"), py::arg("tq"), py::arg("nq"), py::arg("wk"), py::arg("tk"), py::arg("wv"), py::arg("tv"),
     py::arg("nkv"), py::arg("K"), py::arg("xf"), py::arg("ldxf"), py::arg("norm"), py::arg("eps"), py::arg("B"),
     py::arg("out"), py::arg("ldo"), py::arg("ss_out"), py::arg("pos"), py::arg("rope"), py::arg("head_dim"),
     py::arg("n_ctx"), py::arg("stream"), py::arg("zero") = 0, py::arg("zero_n") = 0, py::arg("dbg_clk") = 0);
  m.def("bmm_qkv_sk_supported", &bmm_qkv_sk_supported);
  m.def("bmm_qkv_sk_defers_rope", &bmm_qkv_sk_defers_rope);
  m.def("attn_decode_workspace_floats", &attn_decode_workspace_floats);
  m.def("attn_prefill", [](uintptr_t q, uintptr_t kc, uintptr_t vc, int T, int pos0, int n_ctx, int n_head, int n_kv,
                           int hd, float scale, uintptr_t out, uintptr_t stream, bool out_bf16, bool out_h) {
    AttnPrefillArgs a;
    a.q = P<float>(q); a.k_cache = P<__half>(kc); a.v_cache = P<__half>(vc); a.T = T; a.pos0 = pos0;
    a.n_ctx = n_ctx; a.n_head = n_head; a.n_kv_head = n_kv; a.head_dim = hd; a.scale = scale;
    if (out_h) a.out_h = P<__half>(out);
    else if (out_bf16) a.out_bf16 = P<__hip_bfloat16>(out);
    else a.out = P<float>(out);
    a.out_stride = n_head * hd;
    attn_prefill(a, S(stream));
    hip_ok("attn_prefill");
  }, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("T"), py::arg("pos0"), py::arg("n_ctx"), py::arg("n_head"),
     py::arg("n_kv"), py::arg("hd"), py::arg("scale"), py::arg("out"), py::arg("stream"), py::arg("out_bf16") = false,
     py::arg("out_h") = false);
  m.def("embed", [](uintptr_t w, int type, int V, int d, uintptr_t tokens, int T, uintptr_t x, uintptr_t stream) {
    embed_rows(make_qmat(P<void>(w), type, V, d), P<int>(tokens), T, P<float>(x), S(stream));
    hip_ok("embed");
  });
  m.def("rmsnorm_bf16", [](uintptr_t x, uintptr_t w, float eps, int T, int d, uintptr_t y, uintptr_t stream,
                           bool f16sw) {
    rmsnorm_bf16(P<float>(x), P<float>(w), eps, T, d, P<__hip_bfloat16>(y), S(stream), nullptr, 0, f16sw);
    hip_ok("rmsnorm_bf16");
  }, py::arg("x"), py::arg("w"), py::arg("eps"), py::arg("T"), py::arg("d"), py::arg("y"), py::arg("stream"),
     py::arg("f16sw") = false);
  m.def("launch_probe", [](int threads, int blocks, size_t lds, int iters, uintptr_t out, uintptr_t stream) {
    launch_probe(threads, blocks, lds, iters, P<float>(out), S(stream));
  });
  m.def("clock_probe", [](uintptr_t out, int iters, uintptr_t stream) {
    clock_probe(P<long long>(out), iters, S(stream));
    hip_ok("clock_probe");
  });
  m.def("sampler_blocks", &sampler_blocks);
  m.def("sampler_cand_words", &sampler_cand_words);
  // stage 1 over logits[0, V) whose global ids start at vocab_off (slices over [0, V_span)),
  // then - if cand_all is given - stage 2 over `world` gathered blocks, else over this one
  m.def("sample", [](uintptr_t logits, int V, uintptr_t params, uintptr_t ring, uintptr_t state, uintptr_t cand,
                     uintptr_t out_tokens, int out_cap, int advance, uintptr_t stream, uintptr_t dbg_clk,
                     int vocab_off, int V_glob, int V_span, uintptr_t cand_all, int world, int stage) {
    SamplerArgs a;
    a.dbg_clk = P<long long>(dbg_clk);
    a.logits = P<float>(logits); a.V = V; a.p = P<SamplerParamsDev>(params); a.ring = P<int>(ring);
    a.state = P<int>(state); a.cand = P<unsigned>(cand); a.out_tokens = P<int>(out_tokens);
    a.out_cap = out_cap; a.advance_pos = advance;
    a.vocab_off = vocab_off; a.V_glob = V_glob; a.V_span = V_span;
    a.cand_all = P<const unsigned>(cand_all); a.world = world;
    if (stage & 1) sample_stage1(a, S(stream));
    if (stage & 2) sample_stage2(a, S(stream));
    hip_ok("sample");
  }, py::arg("logits"), py::arg("V"), py::arg("params"), py::arg("ring"), py::arg("state"), py::arg("cand"),
     py::arg("out_tokens"), py::arg("out_cap"), py::arg("advance"), py::arg("stream"), py::arg("dbg_clk") = 0,
     py::arg("vocab_off") = 0, py::arg("V_glob") = 0, py::arg("V_span") = 0, py::arg("cand_all") = 0,
     py::arg("world") = 1, py::arg("stage") = 3);
  m.def("sampler_params_bytes", [](int top_k, float top_p, float min_p, float temp, float rp, float fp, float pp,
                                   int last_n, unsigned long long seed, int greedy, float tfs_z, float typical_p,
                                   py::dict logit_bias) {
    SamplerParamsDev p;
    p.top_k = top_k; p.top_p = top_p; p.min_p = min_p; p.temp = temp; p.repeat_penalty = rp;
    p.freq_penalty = fp; p.presence_penalty = pp; p.last_n = last_n; p.seed = seed; p.greedy = greedy;
    p.tfs_z = tfs_z; p.typical_p = typical_p;
    for (auto kv : logit_bias) {
      if (p.n_bias == kMaxLogitBias) throw std::runtime_error("at most 64 logit_bias entries");
      p.bias_tok[p.n_bias] = kv.first.cast<int>();
      p.bias_val[p.n_bias++] = kv.second.cast<float>();
    }
    return py::bytes(reinterpret_cast<const char*>(&p), sizeof(p));
  }, py::arg("top_k"), py::arg("top_p"), py::arg("min_p"), py::arg("temp"), py::arg("rp"), py::arg("fp"),
     py::arg("pp"), py::arg("last_n"), py::arg("seed"), py::arg("greedy"), py::arg("tfs_z") = 1.f,
     py::arg("typical_p") = 1.f, py::arg("logit_bias") = py::dict());
  m.def("fill_random", [](uintptr_t base, int type, size_t rows, size_t K, float std, unsigned long long seed,
                          uintptr_t stream) {
    fill_random_planar(P<uint8_t>(base), type, rows, K, std, seed, S(stream));
    hip_ok("fill_random");
  });
}
