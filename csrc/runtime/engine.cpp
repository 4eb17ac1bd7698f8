#include "engine.h"

#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "repack.h"
#include "shard.h"

namespace lfk {

#define HIPCHK(x) check((x), #x)

// roctx ranges (visible with rocprofv3 --marker-trace): prefill chunks, decode loop
struct RoctxRange {
  explicit RoctxRange(const char* m) { roctxRangePushA(m); }
  ~RoctxRange() { roctxRangePop(); }
};

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

HParams read_hparams(const GGUFFile& f) {
  HParams h;
  std::string arch = f.get_str("general.architecture", "llama");
  if (arch != "llama" && arch != "mistral" && arch != "mixtral")
    throw std::runtime_error("unsupported architecture " + arch);
  auto gi = [&](const char* k, int64_t d) { return (int)f.get_int(arch + "." + k, d); };
  h.n_embd = gi("embedding_length", 0);
  h.n_layer = gi("block_count", 0);
  h.n_head = gi("attention.head_count", 0);
  h.n_head_kv = gi("attention.head_count_kv", h.n_head);
  h.head_dim = gi("rope.dimension_count", h.n_head ? h.n_embd / h.n_head : 0);
  h.n_ff = gi("feed_forward_length", 0);
  h.n_expert = gi("expert_count", 0);
  h.n_expert_used = gi("expert_used_count", 0);
  h.n_ctx_train = gi("context_length", 2048);
  h.rope_base = (float)f.get_float(arch + ".rope.freq_base", 10000.0);
  h.rms_eps = (float)f.get_float(arch + ".attention.layer_norm_rms_epsilon", 1e-5);
  const GGUFTensor* emb = f.find("token_embd.weight");
  if (!emb) throw std::runtime_error("missing token_embd.weight");
  h.n_vocab = (int)emb->ne[1];
  return h;
}

void Engine::check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    healthy_ = false;
    last_error_ = std::string(what) + ": " + hipGetErrorString(e);
    throw std::runtime_error(last_error_);
  }
}

static void ncclchk(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

void* Engine::dalloc(size_t bytes) {
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, bytes < 16 ? 16 : bytes));
  allocs_.push_back(p);
  dev_bytes_ += bytes;
  return p;
}

uint8_t* Engine::stage_acquire(size_t bytes) {
  const int i = stage_.cur;
  if (!upload_stream_) {
    HIPCHK(hipStreamCreateWithFlags(&upload_stream_, hipStreamNonBlocking));
    for (auto& e : stage_.done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  HIPCHK(hipEventSynchronize(stage_.done[i]));   // its previous copy has left the buffer
  if (stage_.cap[i] < bytes) {
    if (stage_.buf[i]) HIPCHK(hipHostFree(stage_.buf[i]));
    stage_.buf[i] = nullptr;
    const size_t cap = (bytes + (4u << 20) - 1) & ~(size_t)((4u << 20) - 1);
    HIPCHK(hipHostMalloc((void**)&stage_.buf[i], cap, hipHostMallocDefault));
    stage_.cap[i] = cap;
  }
  return stage_.buf[i];
}

void Engine::stage_commit(void* dev, size_t bytes) {
  const int i = stage_.cur;
  HIPCHK(hipMemcpyAsync(dev, stage_.buf[i], bytes, hipMemcpyHostToDevice, upload_stream_));
  HIPCHK(hipEventRecord(stage_.done[i], upload_stream_));
  stage_.cur ^= 1;
}

void Engine::stage_release() {
  if (!upload_stream_) return;
  HIPCHK(hipStreamSynchronize(upload_stream_));
  for (int i = 0; i < 2; ++i) {
    if (stage_.buf[i]) HIPCHK(hipHostFree(stage_.buf[i]));
    stage_.buf[i] = nullptr;
    stage_.cap[i] = 0;
    if (stage_.done[i]) HIPCHK(hipEventDestroy(stage_.done[i]));
    stage_.done[i] = nullptr;
  }
  HIPCHK(hipStreamDestroy(upload_stream_));
  upload_stream_ = nullptr;
}

Engine::Engine(const std::string& path, const EngineOptions& opts) : opt_(opts) {
  HIPCHK(hipSetDevice(opt_.device));
  HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  for (auto& e : step_ev_) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  GGUFFile f(path);
  hp_ = read_hparams(f);
  const int tp = opt_.tp_size, r = opt_.tp_rank;
  const ShardPlan sp =
      make_shard_plan(hp_.n_head, hp_.n_head_kv, hp_.head_dim, hp_.n_ff, hp_.n_vocab, tp, r, opt_.tensor_split);
  q0_ = sp.q_row0();
  kv0_ = sp.kv_row0();
  f0_ = sp.f0();
  nh_l_ = sp.nh_l;
  nkv_l_ = sp.nkv_l;
  nq_ = sp.nq;
  nkvd_ = sp.nkvd;
  F_l_ = sp.F_l;
  // fault-injection test hook (EngineOptions::test_fault; never set in production), parsed once
  if (!opt_.test_fault.empty()) {
    int rk = -1, n = -1;
    char kind[8] = {0};
    const int got = std::sscanf(opt_.test_fault.c_str(), "%d:%d:%7s", &rk, &n, kind);
    if (got < 2) throw std::runtime_error("test_fault: expected <rank>:<n>[:dev|:shard]");
    std::fprintf(stderr, "[lfk] WARNING: fault-injection test hook active on rank %d: %s\n", r,
                 opt_.test_fault.c_str());
    if (rk == r && tp > 1) {
      if (got == 3 && std::strcmp(kind, "shard") == 0) {
        f0_ = (f0_ + (size_t)F_l_) % (size_t)hp_.n_ff;
      } else if (n > 0) {
        fault_after_ = n;
        fault_dev_ = got == 3 && std::strcmp(kind, "dev") == 0;
      }
    }
  }
  V_l_ = sp.V_l;
  V_pad_ = sp.V_pad;
  V_real_l_ = std::max(0, std::min(V_l_, hp_.n_vocab - r * V_l_));
  if (opt_.comm != "auto" && opt_.comm != "ipc" && opt_.comm != "rccl")
    throw std::runtime_error("comm must be auto, ipc or rccl");
  if (opt_.layer_begin < 0 || opt_.layer_begin > hp_.n_layer) throw std::runtime_error("bad layer_begin");
  if (opt_.layer_begin > 0 && tp > 1) throw std::runtime_error("partial offload cannot be combined with split_mode=row");
  if (opt_.n_ctx <= 0) opt_.n_ctx = hp_.n_ctx_train;
  if (opt_.n_slots < 1) throw std::runtime_error("n_slots must be >= 1");
  layer_end_ = opt_.layer_end < 0 ? hp_.n_layer : opt_.layer_end;
  if (layer_end_ <= opt_.layer_begin || layer_end_ > hp_.n_layer) throw std::runtime_error("bad layer_end");
  if (layer_end_ < hp_.n_layer && tp > 1) throw std::runtime_error("a layer split cannot be combined with split_mode=row");
  if (opt_.n_slots > 1 && (opt_.layer_begin > 0 || layer_end_ < hp_.n_layer))
    throw std::runtime_error("KV slots (batched decode) need the GPU to hold every layer");
  // comm=rccl at tp_size 1: the tensor-parallel code paths over a ONE-rank RCCL communicator
  // (every collective a copy) - how a one-GPU box runs the RCCL branch inside captured graphs
  tp_on_ = tp > 1 || opt_.comm == "rccl";
  if (tp_on_ && opt_.comm != "ipc") {
    if (opt_.nccl_id.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad nccl id");
    ncclUniqueId id;
    std::memcpy(&id, opt_.nccl_id.data(), sizeof(id));
    ncclComm_t c;
    ncclchk(ncclCommInitRank(&c, tp, id, r), "ncclCommInitRank");
    comm_ = c;
  }
  load(f);
  stage_release();   // every weight is on the device before anything reads it
  alloc_buffers();
  build_rope();
  setup_batch_mfma();
  HIPCHK(hipStreamSynchronize(stream_));
}

Engine::~Engine() {
  try {
    if (leader() && tp_ctl_ && !tp_stopped_) tp_stop();
  } catch (...) {
  }
  if (graph_exec_) hipGraphExecDestroy(graph_exec_);
  if (graph_exec2_) hipGraphExecDestroy(graph_exec2_);
  for (hipGraphExec_t g : chain_graph_)
    if (g) hipGraphExecDestroy(g);
  if (chain_ev_) hipEventDestroy(chain_ev_);
  for (size_t i = 1; i < sgraph_.size(); ++i)
    if (sgraph_[i]) hipGraphExecDestroy(sgraph_[i]);
  for (size_t i = 1; i < sgraph2_.size(); ++i)
    if (sgraph2_[i]) hipGraphExecDestroy(sgraph2_[i]);
  for (hipGraphExec_t g : bgraph_)
    if (g) hipGraphExecDestroy(g);
  for (hipGraphExec_t g : bgraph2_)
    if (g) hipGraphExecDestroy(g);
  if (graph_) hipGraphDestroy(graph_);
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
  for (void* p : allocs_) hipFree(p);
  try {
    stage_release();
  } catch (...) {
  }
  if (h_ring_) hipHostFree(h_ring_);
  if (h_tokens_) hipHostFree(h_tokens_);
  if (h_bslots_) hipHostFree(h_bslots_);
  if (h_btok_) hipHostFree(h_btok_);
  for (int i = 0; i < 2; ++i) {
    if (h_btok2_[i]) hipHostFree(h_btok2_[i]);
    if (bev_[i]) hipEventDestroy(bev_[i]);
  }
  if (h_rmeta_) hipHostFree(h_rmeta_);
  if (wo_err_h_) hipHostFree(wo_err_h_);
  if (chain_err_h_) hipHostFree(chain_err_h_);
  for (auto& e : step_ev_) if (e) hipEventDestroy(e);
  if (stream_) hipStreamDestroy(stream_);
}

// ------------------------------------------------------------------------ loading
QMat Engine::upload_matrix(const GGUFFile& f, const std::string& name, size_t r0, size_t R, size_t c0, size_t K,
                           int n_expert) {
  const GGUFTensor* t = f.find(name);
  if (!t) throw std::runtime_error("missing tensor " + name);
  const size_t K_src = (size_t)t->ne[0];
  const size_t R_src = (size_t)t->ne[1];
  const int E = n_expert > 0 ? n_expert : 1;
  const size_t one = qbytes(t->type, R, K);
  const TypeInfo ti = type_info(t->type);
  const size_t src_expert = R_src * (K_src / ti.block) * ti.bytes;
  f.prefetch(*t);
  uint8_t* host = stage_acquire(one * E);
  for (int e = 0; e < E; ++e) {
    const size_t rows_avail = r0 < R_src ? std::min(R, R_src - r0) : 0;
    if (rows_avail < R) std::memset(host + one * e, 0, one);
    repack_planar(t->type, f.data(*t) + src_expert * e, K_src, r0, rows_avail, c0, K, host + one * e, R, 0, 0);
  }
  void* d = dalloc(one * E);
  stage_commit(d, one * E);
  return make_qmat(d, t->type, (int)R, (int)K, n_expert > 0 ? one : 0);
}

QMat Engine::upload_gate_up(const GGUFFile& f, const std::string& gate, const std::string& up, size_t f0, size_t F,
                            int n_expert) {
  const GGUFTensor* tg = f.find(gate);
  const GGUFTensor* tu = f.find(up);
  if (!tg || !tu) throw std::runtime_error("missing " + gate + " / " + up);
  if (tg->type != tu->type) throw std::runtime_error("gate/up projections must share a quant type");
  if (F % 32) throw std::runtime_error("n_ff per rank must be a multiple of 32");
  const size_t K = (size_t)tg->ne[0];
  const int E = n_expert > 0 ? n_expert : 1;
  const size_t one = qbytes(tg->type, 2 * F, K);
  const TypeInfo ti = type_info(tg->type);
  const size_t src_expert = (size_t)tg->ne[1] * (K / ti.block) * ti.bytes;
  f.prefetch(*tg);
  f.prefetch(*tu);
  uint8_t* host = stage_acquire(one * E);
  for (int e = 0; e < E; ++e) {
    repack_planar(tg->type, f.data(*tg) + src_expert * e, K, f0, F, 0, K, host + one * e, 2 * F, 32, 0);
    repack_planar(tu->type, f.data(*tu) + src_expert * e, K, f0, F, 0, K, host + one * e, 2 * F, 32, 32);
  }
  void* d = dalloc(one * E);
  stage_commit(d, one * E);
  return make_qmat(d, tg->type, (int)(2 * F), (int)K, n_expert > 0 ? one : 0);
}

float* Engine::upload_f32(const GGUFFile& f, const std::string& name) {
  const GGUFTensor* t = f.find(name);
  if (!t) throw std::runtime_error("missing tensor " + name);
  if (t->type != T_F32) throw std::runtime_error(name + ": expected F32");
  float* d = static_cast<float*>(dalloc(t->nbytes));
  std::memcpy(stage_acquire(t->nbytes), f.data(*t), t->nbytes);
  stage_commit(d, t->nbytes);
  return d;
}

void Engine::load(const GGUFFile& f) {
  const int r = opt_.tp_rank;
  const int d = hp_.n_embd, hd = hp_.head_dim;
  // only the stage that starts at layer 0 gathers embeddings (a hybrid / layer-split stage past
  // it takes hidden states in)
  if (opt_.layer_begin == 0) tok_embd_ = upload_matrix(f, "token_embd.weight", 0, hp_.n_vocab, 0, d);
  if (has_head()) {  // (a layer-split stage before the last holds no head)
    out_norm_ = upload_f32(f, "output_norm.weight");
    const std::string out_name = f.find("output.weight") ? "output.weight" : "token_embd.weight";
    output_ = upload_matrix(f, out_name, (size_t)r * V_l_, V_l_, 0, d);
  }
  layers_.resize(hp_.n_layer);
  for (int l = opt_.layer_begin; l < layer_end_; ++l) {
    const std::string p = "blk." + std::to_string(l) + ".";
    Layer& L = layers_[l];
    L.attn_norm = upload_f32(f, p + "attn_norm.weight");
    L.ffn_norm = upload_f32(f, p + "ffn_norm.weight");
    L.wq = upload_matrix(f, p + "attn_q.weight", q0_, nq_, 0, d);
    L.wk = upload_matrix(f, p + "attn_k.weight", kv0_, nkvd_, 0, d);
    L.wv = upload_matrix(f, p + "attn_v.weight", kv0_, nkvd_, 0, d);
    L.wo = upload_matrix(f, p + "attn_output.weight", 0, d, q0_, nq_);
    if (hp_.n_expert > 0) {
      L.router = upload_matrix(f, p + "ffn_gate_inp.weight", 0, hp_.n_expert, 0, d);
      L.gu_exps = upload_gate_up(f, p + "ffn_gate_exps.weight", p + "ffn_up_exps.weight", f0_, F_l_,
                                 hp_.n_expert);
      L.down_exps = upload_matrix(f, p + "ffn_down_exps.weight", 0, d, f0_, F_l_, hp_.n_expert);
    } else {
      L.w_gu = upload_gate_up(f, p + "ffn_gate.weight", p + "ffn_up.weight", f0_, F_l_);
      L.w_down = upload_matrix(f, p + "ffn_down.weight", 0, d, f0_, F_l_);
    }
    (void)hd;
  }
}

void Engine::alloc_buffers() {
  // activation rows: n_batch for prompt chunks; a batching engine on one GPU packs a joint admission
  // (slots_begin) into chunks of up to kJointRows rows - six ~390-token prompts in ONE pass over the
  // weights instead of five n_batch chunks, at the GEMMs' large-T efficiency (the activations of
  // 4096 rows are ~0.55 GB at the 8B, ~1.1 GB at the 70B)
  nb_cap_ = opt_.n_batch;
  long long joint = kJointRows;
  if (const char* e = std::getenv("LFK_JOINT_ROWS")) joint = std::atoll(e);  // A/B, tests (0: n_batch chunks)
  if (opt_.n_slots > 1 && opt_.tp_size == 1)
    nb_cap_ = std::max(nb_cap_, (int)std::min<long long>(joint, (long long)opt_.n_slots * opt_.n_ctx));
  const int B = nb_cap_, d = hp_.n_embd, hd = hp_.head_dim;
  const int E = std::max(hp_.n_expert, 1), KU = std::max(hp_.n_expert_used, 1);
  x_ = (float*)dalloc(sizeof(float) * B * d);
  tmp_ = (float*)dalloc(sizeof(float) * B * d);
  xb_ = (__hip_bfloat16*)dalloc(2ull * B * d);
  qkv_ = (float*)dalloc(sizeof(float) * B * (nq_ + 2 * nkvd_));
  q_ = (float*)dalloc(sizeof(float) * B * nq_);
  attn_ = (float*)dalloc(sizeof(float) * B * nq_);
  attnb_ = (__hip_bfloat16*)dalloc(2ull * B * nq_);
  h_ = (__hip_bfloat16*)dalloc(2ull * B * F_l_);
  hf_ = (float*)dalloc(sizeof(float) * KU * F_l_);
  logits_ = (float*)dalloc(sizeof(float) * V_pad_);
  logits_l_ = (float*)dalloc(sizeof(float) * V_l_);
  HIPCHK(hipMemset(logits_l_, 0, sizeof(float) * V_l_));
  // KV of this engine's layers only (a layer-split / hybrid stage holds its range's part)
  const size_t kv = (size_t)(layer_end_ - opt_.layer_begin) * nkv_l_ * opt_.n_ctx * hd;
  const int NS = opt_.n_slots;
  slot_stride_ = kv;
  kc_ = (__half*)dalloc(kv * 2 * NS);
  vc_ = (__half*)dalloc(kv * 2 * NS);
  HIPCHK(hipMemset(kc_, 0, kv * 2 * NS));
  HIPCHK(hipMemset(vc_, 0, kv * 2 * NS));
  rope_ = (float2*)dalloc(sizeof(float2) * opt_.n_ctx * (hd / 2));
  rope_freq_ = (float*)dalloc(sizeof(float) * (hd / 2));
  attn_part_ = (float*)dalloc(sizeof(float) * attn_decode_workspace_floats(opt_.n_ctx, nh_l_, hd));
  attn_cnt_ = (int*)dalloc(sizeof(int) * 64);
  HIPCHK(hipMemset(attn_cnt_, 0, sizeof(int) * 64));
  if (const char* e = std::getenv("LFK_ATTN_TOUCH")) attn_touch_ = e[0] != '0';  // A/B (test_engine_gpu)
  // single-row decode: attention + Wo in one launch (attn_wo1); per-layer done counters, zeroed
  // by every decode step's embedding launch
  if (const char* e = std::getenv("LFK_WO_FUSE")) wo_fuse_ = e[0] != '0';  // A/B
  if (const char* e = std::getenv("LFK_MOE_ROUTE_FUSE")) moe_route_fuse_ = e[0] != '0';  // A/B (test_engine_gpu)
  if (const char* e = std::getenv("LFK_TP_EPILOGUE")) tp_epi_ = e[0] != '0';  // A/B: the separate collective kernel
  if (const char* e = std::getenv("LFK_PIECES_ATTN")) pieces_attn_ = e[0] != '0';  // A/B: one launch per piece
  if (wo_fuse_ && nkv_l_ <= 64) {
    HIPCHK(hipHostMalloc((void**)&wo_err_h_, sizeof(int), hipHostMallocMapped));
    *wo_err_h_ = 0;
    HIPCHK(hipHostGetDevicePointer((void**)&wo_err_, wo_err_h_, 0));
    dec_done_ = (int*)dalloc(sizeof(int) * 64 * hp_.n_layer);
    HIPCHK(hipMemset(dec_done_, 0, sizeof(int) * 64 * hp_.n_layer));
  } else {
    wo_fuse_ = false;
  }
  const int tp = opt_.tp_size;
  cand_words_ = sampler_cand_words(V_l_);
  cand_ = (unsigned*)dalloc(sizeof(unsigned) * cand_words_);
  if (tp_on_) cand_all_ = (unsigned*)dalloc(sizeof(unsigned) * cand_words_ * tp);
  state_ = (int*)dalloc(sizeof(int) * S_NSTATE * NS);
  ring_ = (int*)dalloc(sizeof(int) * 64 * NS);
  out_tokens_ = (int*)dalloc(sizeof(int) * 64);
  tokens_ = (int*)dalloc(sizeof(int) * B);
  sparams_ = (SamplerParamsDev*)dalloc(sizeof(SamplerParamsDev) * NS);
  router_logits_ = (float*)dalloc(sizeof(float) * B * E);
  moe_ids_ = (int*)dalloc(sizeof(int) * KU);
  moe_w_ = (float*)dalloc(sizeof(float) * KU);
  if (hp_.n_expert > 0) {
    const size_t R = (size_t)B * KU;
    moe_sel_ = (int*)dalloc(sizeof(int) * R);
    moe_selw_ = (float*)dalloc(sizeof(float) * R);
    moe_off_ = (int*)dalloc(sizeof(int) * (E + 1));
    moe_tok_ = (int*)dalloc(sizeof(int) * R);
    moe_gw_ = (float*)dalloc(sizeof(float) * R);
    moe_pos_ = (int*)dalloc(sizeof(int) * R);
    moe_xg_ = (__hip_bfloat16*)dalloc(2 * R * d);
    moe_hg_ = (__hip_bfloat16*)dalloc(2 * R * F_l_);
    moe_yg_ = (float*)dalloc(sizeof(float) * R * d);
  }
  HIPCHK(hipMemset(state_, 0, sizeof(int) * S_NSTATE * NS));
  HIPCHK(hipMemset(ring_, 0, sizeof(int) * 64 * NS));
  if (NS > 1) {
    bmax_ = std::min(NS, opt_.n_batch);
    bslots_ = (int*)dalloc(sizeof(int) * bmax_);
    bpos_ = (int*)dalloc(sizeof(int) * bmax_);
    btok_ = (int*)dalloc(sizeof(int) * bmax_);
    btok_out_ = (int*)dalloc(sizeof(int) * bmax_);
    logits_b_ = (float*)dalloc(sizeof(float) * bmax_ * V_pad_);
    cand_b_ = (unsigned*)dalloc(sizeof(unsigned) * bmax_ * cand_words_);
    if (tp_on_) cand_all_b_ = (unsigned*)dalloc(sizeof(unsigned) * bmax_ * cand_words_ * tp);
    attn_part_b_ = (float*)dalloc(sizeof(float) * bmax_ * attn_decode_workspace_floats(opt_.n_ctx, nh_l_, hd));
    attn_cnt_b_ = (int*)dalloc(sizeof(int) * 64 * bmax_);
    HIPCHK(hipMemset(attn_cnt_b_, 0, sizeof(int) * 64 * bmax_));
    gu_b_ = (float*)dalloc(sizeof(float) * bmax_ * 2 * F_l_);
    if (tp_on_) {  // the batched row-parallel partials (zero between launches: P2PArgs::accumulate)
      tmp_b_ = (float*)dalloc(sizeof(float) * bmax_ * d);
      HIPCHK(hipMemset(tmp_b_, 0, sizeof(float) * bmax_ * d));
    }
    HIPCHK(hipHostMalloc((void**)&h_bslots_, sizeof(int) * bmax_, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&h_btok_, sizeof(int) * bmax_, hipHostMallocDefault));
    for (int i = 0; i < 2; ++i) {
      HIPCHK(hipHostMalloc((void**)&h_btok2_[i], sizeof(int) * bmax_, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(h_btok2_[i], 0, sizeof(int) * bmax_);
      HIPCHK(hipHostGetDevicePointer((void**)&btok_dev_[i], h_btok2_[i], 0));
      HIPCHK(hipEventCreateWithFlags(&bev_[i], hipEventDisableTiming));
    }
    rpos_ = (int*)dalloc(sizeof(int) * B);
    rslots_ = (int*)dalloc(sizeof(int) * B);
    HIPCHK(hipHostMalloc((void**)&h_rmeta_, sizeof(int) * 3 * B, hipHostMallocDefault));
  }
  HIPCHK(hipMemset(out_tokens_, 0, sizeof(int) * 64));
  // P2P messages: a decode step's hidden rows and the sampler's candidate blocks; in "ipc"
  // mode (no RCCL) also prefill chunks and the test hooks' logit gathers
  {
    size_t m = (size_t)std::max(bmax_, 1) * std::max<size_t>((size_t)d, cand_words_);
    if (opt_.comm == "ipc")
      m = std::max({m, (size_t)B * d, (size_t)std::max(bmax_, 1) * V_pad_});
    if (m > (size_t)INT32_MAX / 4) throw std::runtime_error("p2p message bound too large");
    p2p_max_n_ = (int)m;
  }
  HIPCHK(hipHostMalloc((void**)&h_ring_, sizeof(int) * 64, hipHostMallocDefault));
  HIPCHK(hipHostMalloc((void**)&h_tokens_, sizeof(int) * B, hipHostMallocDefault));
}

void Engine::setup_batch_mfma() {
  bg_ = bg_ffn_ = false;
  if (!bmax_ || opt_.layer_begin > 0 || !has_head()) return;
  auto ok = [&](const QMat& m) { return m.base && bmm_supported(m.type, m.K); };
  auto kfit = [](int K) { return K % 128 == 0 && K <= 32768; };  // bprep's row shapes
  bool att = ok(output_) && kfit(hp_.n_embd) && kfit(nq_) && (V_pad_ % 4) == 0 && ((nq_ + 2 * nkvd_) % 4) == 0;
  bool ffn = hp_.n_expert == 0 && kfit(F_l_) && (2 * F_l_) % 64 == 0;
  for (int l = 0; l < hp_.n_layer; ++l) {
    const Layer& L = layers_[l];
    att = att && ok(L.wq) && ok(L.wk) && ok(L.wv) && ok(L.wo);
    ffn = ffn && ok(L.w_gu) && ok(L.w_down);
  }
  bool moe = hp_.n_expert > 0 && moe_router_fused_ok(layers_[0].router.type, hp_.n_expert, hp_.n_embd) &&
             F_l_ % 256 == 0 && (2 * F_l_) % 64 == 0 && kfit(hp_.n_embd);
  for (int l = 0; moe && l < hp_.n_layer; ++l) {
    const Layer& L = layers_[l];
    moe = moe_router_fused_ok(L.router.type, hp_.n_expert, hp_.n_embd) && ok(L.gu_exps) && ok(L.down_exps);
  }
  bg_ = att;
  bg_ffn_ = att && ffn;
  moe_b_ = att && moe;
  const char* sk = std::getenv("LFK_QKV_SK");
  qkv_sk_ = !(sk && sk[0] == '0');
  if (const char* sc = std::getenv("LFK_STEP_CLK")) {
    step_clk_layer_ = std::atoi(sc);
    step_clk_ = (long long*)dalloc(sizeof(long long) * 5 * kStepClkBlocks * 16);
    HIPCHK(hipMemsetAsync(step_clk_, 0, sizeof(long long) * 5 * kStepClkBlocks * 16, stream_));
  }
  if (!bg_) return;
  if (const char* e = std::getenv("LFK_FFN_CHAIN")) ffn_chain_ = std::max(0, std::min(2, std::atoi(e)));  // A/B
  if (ffn_chain_) {
    chain_cnt_ = (int*)dalloc(sizeof(int) * kChainInts * hp_.n_layer);
    HIPCHK(hipMemsetAsync(chain_cnt_, 0, sizeof(int) * kChainInts * hp_.n_layer, stream_));
    HIPCHK(hipHostMalloc((void**)&chain_err_h_, sizeof(int), hipHostMallocMapped));
    *chain_err_h_ = 0;
    HIPCHK(hipHostGetDevicePointer((void**)&chain_err_, chain_err_h_, 0));
  }
  const int E = std::max(1, hp_.n_expert);
  xh_b_ = (__half*)dalloc(2ull * bmax_ * std::max({hp_.n_embd, nq_, F_l_}));
  {
    const size_t n = qkv_b_zero_n();  // + ss_b_ [16]
    qkv_b_ = (float*)dalloc(sizeof(float) * n);
    HIPCHK(hipMemsetAsync(qkv_b_, 0, sizeof(float) * n, stream_));
    ss_b_ = qkv_b_ + (size_t)bmax_ * (nq_ + 2 * nkvd_);
  }
  hh_b_ = (__half*)dalloc(2ull * bmax_ * std::max(1, F_l_) * (moe_b_ ? E : 1));
  if (moe_b_) ew_b_ = (float*)dalloc(sizeof(float) * bmax_ * E);
  // the batched path reads its own copy of the weights, laid out per 16-row tile (bmm.hip)
  auto tile = [&](const QMat& m, bool swiglu = false) {
    QMat t = m;
    uint8_t* dst = (uint8_t*)dalloc(t16_bytes(m.type, m.rows, m.K));
    t16_repack(m, dst, stream_, swiglu);
    t.base = dst;
    return t;
  };
  t_output_ = tile(output_);
  for (int l = 0; l < hp_.n_layer; ++l) {
    Layer& L = layers_[l];
    L.t_wq = tile(L.wq); L.t_wk = tile(L.wk); L.t_wv = tile(L.wv); L.t_wo = tile(L.wo);
    if (bg_ffn_) { L.t_gu = tile(L.w_gu, /*swiglu=*/true); L.t_down = tile(L.w_down); }
    if (moe_b_) {
      // gate/up: the experts' SwiGLU tile16 copies back to back (expert e = tiles [e T, (e+1) T))
      const size_t gu1 = t16_bytes(L.gu_exps.type, L.gu_exps.rows, L.gu_exps.K);
      uint8_t* gdst = (uint8_t*)dalloc(gu1 * E);
      // down: every 16-row tile's 256-k steps run expert 0's F_l, then expert 1's, ... (K = E F_l):
      // each expert's copy goes through `tmp` and is strided into its step range of every tile
      const int dsteps = L.down_exps.K / 256, dtiles = (L.down_exps.rows + 15) / 16;
      const size_t dn1 = t16_bytes(L.down_exps.type, L.down_exps.rows, L.down_exps.K);
      const size_t run = dn1 / dtiles;  // one tile's steps of one expert
      uint8_t* ddst = (uint8_t*)dalloc(dn1 * E);
      // one expert's copy, strided into place, then freed (the P2P receive region checks that it
      // is a whole allocation of its own, runtime/p2p.cpp, so a reuse of this block cannot alias it)
      uint8_t* tmp = nullptr;
      HIPCHK(hipMalloc((void**)&tmp, dn1));
      for (int e = 0; e < E; ++e) {
        QMat g = L.gu_exps;
        g.base += L.gu_exps.expert_stride * e;
        g.expert_stride = 0;
        t16_repack(g, gdst + gu1 * e, stream_, /*swiglu=*/true);
        QMat dm = L.down_exps;
        dm.base += L.down_exps.expert_stride * e;
        dm.expert_stride = 0;
        t16_repack(dm, tmp, stream_);
        HIPCHK(hipMemcpy2DAsync(ddst + run * e, run * E, tmp, run, run, dtiles, hipMemcpyDeviceToDevice, stream_));
      }
      HIPCHK(hipStreamSynchronize(stream_));
      HIPCHK(hipFree(tmp));
      L.t_gu = L.gu_exps;
      L.t_gu.base = gdst; L.t_gu.rows = L.gu_exps.rows * E; L.t_gu.expert_stride = 0;
      L.t_down = L.down_exps;
      L.t_down.base = ddst; L.t_down.K = dsteps * 256 * E; L.t_down.expert_stride = 0;
    }
  }
  HIPCHK(hipStreamSynchronize(stream_));
  // dense models: prompt chunks on the same tile16 copies (gemm_t16: the dequantisation spread
  // over 128 tokens per fragment, f16 activations - measured against gemm_dq in profiles/)
  // (MoE: the experts run on the stacked SwiGLU copy and the K-concatenated down copy)
  const char* pt = std::getenv("LFK_PREFILL_T16");
  bool t16 = (hp_.n_expert > 0 ? moe_b_ : bg_ffn_) && !(pt && pt[0] == '0');
  for (int l = 0; t16 && l < hp_.n_layer; ++l) {
    const Layer& L = layers_[l];
    for (const QMat* m : {&L.t_wq, &L.t_wk, &L.t_wv, &L.t_wo, &L.t_gu, &L.t_down}) t16 = t16 && m->base && m->rows % 16 == 0;
    if (hp_.n_expert > 0) t16 = t16 && L.down_exps.K % 256 == 0 && L.gu_exps.rows % 16 == 0;
  }
  prefill_t16_ = t16;
}

std::vector<long long> Engine::step_clk() {
  std::vector<long long> h((size_t)5 * kStepClkBlocks * 16, 0);
  if (step_clk_) {
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(h.data(), step_clk_, sizeof(long long) * h.size(), hipMemcpyDeviceToHost));
  }
  return h;
}

void Engine::step_clk_zero() {
  if (!step_clk_) return;
  HIPCHK(hipStreamSynchronize(stream_));
  HIPCHK(hipMemset(step_clk_, 0, sizeof(long long) * 5 * kStepClkBlocks * 16));
}

std::string Engine::group_fault() const {
  if (!leader() || !tp_ctl_ || tp_stopped_) return "";
  return tp_ctl_->fault_report();
}

void Engine::check_device_err() {
  // the bounded in-kernel waits: the P2P all-reduce's (TP) and the batched Wo's (a host-mapped
  // word: no copy); a blocking read of an error word nothing else writes cost every step a copy.
  // Under TP a timed-out wait on ANY rank stores that rank's code into every rank's region, and a
  // follower's host failure lands in the control channel: either poisons the group here
  int e = 0;
  std::string group;
  // (the P2P fault words through their host-mapped mirror: no blocking copy per step)
  if (p2p_ && p2p_->ready()) group = p2p_->fault_report(/*fresh=*/false);
  if (group.empty()) group = group_fault();
  if (!group.empty()) {
    healthy_ = false;
    last_error_ = "tensor-parallel group fault: " + group;
    throw std::runtime_error(last_error_);
  }
  if (wo_err_h_ && __atomic_load_n(wo_err_h_, __ATOMIC_ACQUIRE)) e = 200;  // the batched Wo's wait
  if (!e && chain_err_h_ && __atomic_load_n(chain_err_h_, __ATOMIC_ACQUIRE)) e = 201;  // the FFN chain's
  if (e != 0) {
    healthy_ = false;
    last_error_ = "in-kernel hand-off wait timed out (code " + std::to_string(e) + ")";
    throw std::runtime_error(last_error_);
  }
}

void Engine::build_rope() {
  const int hd = hp_.head_dim, n = opt_.n_ctx;
  // one angle for every path: the fp32 product pos * freq (as the batched attention's deferred
  // RoPE forms it on the device, and as llama.cpp does), its cos / sin taken exactly - so a key
  // is rotated the same whether a prefill, a single-row decode or a batched step wrote it (a
  // double-precision angle drifted from the fp32 one by up to pos * 2^-24 rad)
  std::vector<float> f(hd / 2);
  for (int i = 0; i < hd / 2; ++i) f[i] = (float)std::pow((double)hp_.rope_base, -2.0 * i / hd);
  std::vector<float2> t((size_t)n * (hd / 2));
  for (int p = 0; p < n; ++p)
    for (int i = 0; i < hd / 2; ++i) {
      const float a = (float)p * f[i];
      t[(size_t)p * (hd / 2) + i] = make_float2((float)std::cos((double)a), (float)std::sin((double)a));
    }
  HIPCHK(hipMemcpy(rope_, t.data(), t.size() * sizeof(float2), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(rope_freq_, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice));
}

// ------------------------------------------------------------------------ schedule
std::string Engine::p2p_handle() {
  if (opt_.tp_size < 2) throw std::runtime_error("p2p: tensor parallelism is off");
  if (opt_.comm == "rccl") throw std::runtime_error("p2p: comm=rccl has no P2P path");
  // (+ the fused area of d granules: the decode GEMVs' epilogue all-reduce, tp_epilogue())
  if (!p2p_) p2p_ = std::make_unique<P2PComm>(opt_.tp_rank, opt_.tp_size, p2p_max_n_, opt_.device, true, hp_.n_embd);
  return p2p_->handle();
}

void Engine::p2p_open(const std::vector<std::string>& handles) {
  if (!p2p_) throw std::runtime_error("p2p: call p2p_handle() first");
  if (graph_exec_) throw std::runtime_error("p2p: open the peers before the first decode step");
  p2p_->open(handles);
}

// Decode-sized messages (a step's hidden rows, the sampler's candidate blocks) take the
// one-shot P2P path when the peers are open; prefill-sized ones (T x d) go to RCCL's
// ring/tree algorithms - or, with comm=ipc (no RCCL), to the P2P kernel as well.
// Decode GEMVs under TP: the row-parallel all-reduce in the epilogue (GemvArgs::tp_*) when the
// P2P regions carry the fused area (one launch per projection instead of two, no tmp_ copy)
bool Engine::tp_epilogue(GemvArgs& g) const {
  if (!tp_epi_ || !p2p_ || !p2p_->ready() || p2p_->fused_n() < hp_.n_embd || g.n_out > p2p_->fused_n()) return false;
  // more than two ranks on ONE GPU (the eight-rank rehearsal): a waiting epilogue needs every
  // peer's GEMV resident at once, and eight single-queue processes are not reliably co-scheduled
  // (runs of 15 s to > 170 s, r4) - the separate collective kernel's short waits are
  if (p2p_->shared_device() && p2p_->world() > 2) return false;
  // ... and two ranks on ONE GPU at the 70B width: the 2-rank 70B rehearsal's epilogue waits timed
  // out (a rank's spinning waves and its peer's grids did not co-schedule; profiles/README.md,
  // round 6), while the collective kernel's path ran it to the end. One process per GPU - every
  // real deployment - has no co-scheduling requirement and keeps the epilogue.
  if (p2p_->shared_device() && hp_.n_embd > 4096) return false;
  g.tp_peers = p2p_->peers();
  g.tp_world = p2p_->world(); g.tp_rank = p2p_->rank();
  g.tp_stride = p2p_->stride(); g.tp_off = p2p_->fused_offset();
  g.tp_epochs = p2p_->fused_epochs(); g.tp_err = p2p_->err_word();
  // ranks sharing this GPU (the one-GPU rehearsal): each rank's grid a 1/world share of the
  // resident blocks, or one rank's waiting epilogue waves could hold every CU its peers need
  if (p2p_->shared_device()) g.grid_div = p2p_->world();
  return true;
}

std::vector<std::pair<std::string, std::string>> Engine::comm_info() const {
  std::vector<std::pair<std::string, std::string>> o;
  auto put = [&](const char* k, const std::string& v) { o.emplace_back(k, v); };
  put("tp_size", std::to_string(opt_.tp_size));
  put("comm", opt_.comm);
  int nccl_ranks = 0;
  if (comm_ && ncclCommCount(static_cast<ncclComm_t>(comm_), &nccl_ranks) != ncclSuccess) nccl_ranks = -1;
  put("rccl_comm_ranks", std::to_string(nccl_ranks));
  const bool p2p = p2p_ && p2p_->ready();
  put("p2p_ready", p2p ? "1" : "0");
  if (p2p) {
    put("p2p_shared_device", p2p_->shared_device() ? "1" : "0");
    put("p2p_uncached_region", p2p_->uncached() ? "1" : "0");
    put("p2p_max_floats", std::to_string(p2p_->max_n()));
  }
  GemvArgs probe;
  probe.n_out = hp_.n_embd;
  const bool epi = tp_on_ && tp_epilogue(probe);
  const std::string coll = p2p ? "p2p one-shot collective kernel" : comm_ ? "rccl all-reduce" : "none";
  put("decode_row_parallel_allreduce", !tp_on_ ? "none (tp=1)" : epi ? "gemv epilogue granules (no collective launch)" : coll);
  const size_t brow = (size_t)std::max(bmax_, 1) * hp_.n_embd;
  put("batched_row_parallel_allreduce",
      !tp_on_ ? "none (tp=1)"
      : p2p && brow <= (size_t)p2p_->max_n() ? "p2p one-shot collective kernel (accumulating: no copy / fill nodes)"
      : comm_ ? "rccl all-reduce" : "none");
  const size_t pre = (size_t)opt_.n_batch * hp_.n_embd;
  put("prefill_allreduce",
      !tp_on_ ? "none (tp=1)" : p2p && pre <= (size_t)p2p_->max_n() ? "p2p one-shot collective kernel" : comm_ ? "rccl all-reduce" : "none");
  put("sampler_candidate_gather", !tp_on_ ? "none (tp=1)" : p2p ? "p2p all-gather" : comm_ ? "rccl all-gather" : "none");
  return o;
}

void Engine::allreduce_into(const float* send, float* recv, size_t n, hipStream_t s) {
  if (p2p_ && p2p_->ready() && n <= (size_t)p2p_->max_n()) {
    p2p_->allreduce(send, recv, (int)n, s);
    return;
  }
  if (!comm_) throw std::runtime_error("all-reduce of " + std::to_string(n) + " floats: no RCCL communicator and " +
                                       (p2p_ready() ? "the message exceeds the P2P slot" : "P2P peers not open"));
  ncclchk(ncclAllReduce(send, recv, n, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm_), s), "ncclAllReduce");
}

void Engine::allgather_into(const float* send, float* recv, size_t n, hipStream_t s) {
  if (p2p_ && p2p_->ready() && n <= (size_t)p2p_->max_n()) {
    p2p_->allgather(send, recv, (int)n, s);
    return;
  }
  if (!comm_) throw std::runtime_error("all-gather of " + std::to_string(n) + " floats: no RCCL communicator and " +
                                       (p2p_ready() ? "the message exceeds the P2P slot" : "P2P peers not open"));
  ncclchk(ncclAllGather(send, recv, n, ncclFloat32, static_cast<ncclComm_t>(comm_), s), "ncclAllGather");
}

void Engine::enqueue_sample(const float* logits, int rows, size_t ld, int slot, int advance_pos, hipStream_t s) {
  const bool batched = rows > 0;
  SamplerArgs sa;
  sa.logits = const_cast<float*>(logits);
  sa.V = V_real_l_;
  sa.vocab_off = opt_.tp_rank * V_l_;
  sa.V_glob = hp_.n_vocab;
  sa.V_span = V_l_;
  sa.advance_pos = advance_pos;
  if (batched) {
    sa.p = sparams_; sa.ring = ring_; sa.state = state_;
    sa.batch = rows; sa.slots = bslots_; sa.logits_ld = ld; sa.batch_out = btok_out_; sa.batch_out_host = sample_host_;
    sa.cand = cand_b_;
  } else {
    sa.p = sparams_ + slot; sa.ring = ring_ + 64 * slot; sa.state = state_ + (size_t)S_NSTATE * slot;
    sa.cand = cand_;
    if (slot == 0) {
      sa.out_tokens = out_tokens_; sa.out_cap = 64;
    }
  }
  sample_stage1(sa, s);
  if (tp_on_) {
    const size_t words = cand_words_ * (batched ? rows : 1);
    unsigned* all = batched ? cand_all_b_ : cand_all_;
    allgather_into(reinterpret_cast<const float*>(sa.cand), reinterpret_cast<float*>(all), words, s);
    sa.cand_all = all;
    sa.world = opt_.tp_size;
  }
  sample_stage2(sa, s);
}

void Engine::enqueue_layer_decode(int l, hipStream_t s) {
  const Layer& L = layers_[l];
  const int d = hp_.n_embd, hd = hp_.head_dim;
  const bool tp = tp_on_;
  const size_t kv_layer = (size_t)nkv_l_ * opt_.n_ctx * hd;
  int* st = state_ + (size_t)S_NSTATE * dslot_;
  QkvArgs qa;
  qa.wq = L.wq; qa.wk = L.wk; qa.wv = L.wv;
  qa.x = x_; qa.norm_w = L.attn_norm; qa.eps = hp_.rms_eps;
  qa.q_out = q_;
  qa.k_cache = kc_ + slot_stride_ * dslot_ + kv_layer * (l - opt_.layer_begin);
  qa.v_cache = vc_ + slot_stride_ * dslot_ + kv_layer * (l - opt_.layer_begin);
  qa.n_ctx = opt_.n_ctx; qa.head_dim = hd;
  qa.pos = st + S_POS;
  qa.rope = rope_;
  gemv_qkv(qa, s);

  AttnDecodeArgs aa;
  aa.q = q_; aa.k_cache = qa.k_cache; aa.v_cache = qa.v_cache; aa.pos = st + S_POS;
  aa.n_ctx = opt_.n_ctx; aa.n_head = nh_l_; aa.n_kv_head = nkv_l_; aa.head_dim = hd;
  aa.scale = 1.f / std::sqrt((float)hd);
  aa.part = attn_part_; aa.counters = attn_cnt_; aa.out = attn_;
  GemvArgs o;
  o.w = L.wo; o.x = attn_; o.n_out = d;
  const bool tpe = tp && tp_epilogue(o);  // the all-reduce in the GEMV epilogue (no collective launch)
  // attention + Wo in one launch: Wo's weights stream while the attention runs
  bool fused = false;
  if (!tp && wo_fuse_) {
    aa.done = dec_done_ + 64 * l;
    o.out = x_;
    o.wait = aa.done; o.wait_cnt = nkv_l_; o.wait_n = 1; o.wait_err = wo_err_;
    fused = attn_wo1(aa, o, s);
    if (!fused) {
      aa.done = nullptr;
      o.wait = nullptr; o.wait_cnt = 0; o.wait_n = 0; o.wait_err = nullptr;
    }
  }
  if (!fused) {
    if (attn_touch_ && nkv_l_ < 63) {  // this layer's Wo into the memory-side cache under the attention
      aa.pf_sink = attn_cnt_ + 63;
      aa.pf[0] = L.wo.base;
      aa.pf_bytes[0] = qmat_bytes(L.wo);
    }
    attn_decode(aa, s);
  }

  if (fused) {
  } else if (!tp) {
    o.out = x_;
    gemv(o, EPI_ADD, s);
  } else if (tpe) {
    o.out = x_; o.resid = x_;  // x += sum over ranks of the partial rows
    gemv(o, EPI_STORE, s);
  } else {
    o.out = tmp_;
    o.resid = opt_.tp_rank == 0 ? x_ : nullptr;
    gemv(o, EPI_STORE, s);
    allreduce_into(tmp_, x_, d, s);
  }

  if (hp_.n_expert > 0) {
    // the router inside the gate/up GEMV's blocks (each block routes the token itself, block 0
    // writes the picks for the down projection): one launch and one dependent boundary less
    const bool route_in_gu = moe_route_fuse_ && moe_router_fused_ok(L.router.type, hp_.n_expert, d) &&
                             hp_.n_expert <= 8 && d == 4096;
    if (route_in_gu) {
      // (routing happens in the gate/up launch below)
    } else if (moe_router_fused_ok(L.router.type, hp_.n_expert, d)) {  // one launch: norm + f32 router + top-k
      moe_router_fused(x_, L.ffn_norm, hp_.rms_eps, reinterpret_cast<const float*>(L.router.base), d, hp_.n_expert,
                       hp_.n_expert_used, router_logits_, moe_ids_, moe_w_, s);
    } else {
      GemvArgs ra;
      ra.w = L.router; ra.x = x_; ra.norm_w = L.ffn_norm; ra.eps = hp_.rms_eps;
      ra.out = router_logits_; ra.n_out = hp_.n_expert;
      gemv(ra, EPI_STORE, s);
      moe_route(router_logits_, hp_.n_expert, hp_.n_expert_used, moe_ids_, moe_w_, s);
    }
    GemvArgs g;
    g.w = L.gu_exps; g.x = x_; g.norm_w = L.ffn_norm; g.eps = hp_.rms_eps;
    g.out = hf_; g.n_out = F_l_; g.n_slots = hp_.n_expert_used; g.expert_ids = moe_ids_; g.out_slot_stride = F_l_;
    if (route_in_gu) {
      g.route_w = reinterpret_cast<const float*>(L.router.base);
      g.route_E = hp_.n_expert; g.route_k = hp_.n_expert_used;
      g.route_ids = moe_ids_; g.route_wts = moe_w_; g.route_logits = router_logits_;
    }
    gemv(g, EPI_SWIGLU, s);
    MoeDownArgs md;
    md.w = L.down_exps; md.h = hf_; md.expert_ids = moe_ids_; md.expert_w = moe_w_; md.n_slots = hp_.n_expert_used;
    if (!tp) {
      md.out = x_;
      gemv_moe_down(md, s);
    } else {
      if (opt_.tp_rank == 0) HIPCHK(hipMemcpyAsync(tmp_, x_, sizeof(float) * d, hipMemcpyDeviceToDevice, s));
      else HIPCHK(hipMemsetAsync(tmp_, 0, sizeof(float) * d, s));
      md.out = tmp_;
      gemv_moe_down(md, s);
      allreduce_into(tmp_, x_, d, s);
    }
  } else {
    GemvArgs g;
    g.w = L.w_gu; g.x = x_; g.norm_w = L.ffn_norm; g.eps = hp_.rms_eps;
    g.out = hf_; g.n_out = F_l_;
    gemv(g, EPI_SWIGLU, s);
    GemvArgs dn;
    dn.w = L.w_down; dn.x = hf_; dn.n_out = d;
    if (!tp) {
      dn.out = x_;
      gemv(dn, EPI_ADD, s);
    } else if (tp_epilogue(dn)) {
      dn.out = x_; dn.resid = x_;
      gemv(dn, EPI_STORE, s);
    } else {
      dn.out = tmp_;
      dn.resid = opt_.tp_rank == 0 ? x_ : nullptr;
      gemv(dn, EPI_STORE, s);
      allreduce_into(tmp_, x_, d, s);
    }
  }
}

void Engine::enqueue_head(const float* xrow, int advance_pos, hipStream_t s, int slot) {
  GemvArgs h;
  h.w = output_; h.x = xrow; h.norm_w = out_norm_; h.eps = hp_.rms_eps;
  h.n_out = V_real_l_;
  h.out = tp_on_ ? logits_l_ : logits_;
  if (h.n_out > 0) gemv(h, EPI_STORE, s);
  // vocabulary-parallel sampling: stage 1 on this rank's shard, all-gather of the candidate
  // blocks (a few KB), identical stage 2 on every rank (no logit all-gather)
  enqueue_sample(h.out, 0, 0, slot, advance_pos, s);
  if (slot == 0) HIPCHK(hipMemcpyAsync(h_ring_, out_tokens_, sizeof(int) * 64, hipMemcpyDeviceToHost, s));
}

void Engine::enqueue_decode(hipStream_t s) {
  // (the embedding launch also zeroes the layers' attention -> Wo done counters)
  if (!tok_embd_.base) throw std::runtime_error("decode: this stage starts past layer 0 (hidden states in)");
  embed_rows(tok_embd_, state_ + (size_t)S_NSTATE * dslot_ + S_TOKEN, 1, x_, s, dec_done_, 64 * hp_.n_layer);
  for (int l = opt_.layer_begin; l < layer_end_; ++l) enqueue_layer_decode(l, s);
  enqueue_head(x_, 1, s, dslot_);
}

void Engine::enqueue_prefill(int T, int pos0, hipStream_t s, bool embed) {
  if (embed && !tok_embd_.base) throw std::runtime_error("prefill: this stage starts past layer 0 (hidden states in)");
  if (embed) embed_rows(tok_embd_, tokens_, T, x_, s);
  for (int l = opt_.layer_begin; l < layer_end_; ++l) enqueue_rows_layer(l, T, pos0, false, s);
}

void Engine::enqueue_rows_layer(int l, int T, int pos0, bool batched, hipStream_t s) {
  const int d = hp_.n_embd, hd = hp_.head_dim;
  const bool tp = tp_on_;
  const size_t kv_layer = (size_t)nkv_l_ * opt_.n_ctx * hd;
  const int ncol = nq_ + 2 * nkvd_;
  {
    const Layer& L = layers_[l];
    // prompt chunks on the tile16 copies: f16 activations in bmm's k order (same 2-byte buffers)
    const bool t16 = prefill_t16_ && !batched;
    __half* const xh16 = reinterpret_cast<__half*>(xb_);
    __half* const attnh16 = reinterpret_cast<__half*>(attnb_);
    // (+ zero the q|k|v rows for gemm_dq's split-K partials; the tile16 GEMM splits its stacked
    // Q|K|V only on tiny grids and then zeroes what it splits itself - a 4096-row admission's
    // zeroing pass was 57 MB per layer)
    rmsnorm_bf16(x_, L.attn_norm, hp_.rms_eps, T, d, xb_, s, t16 ? nullptr : qkv_, t16 ? 0 : ncol, t16);
    if (t16) {
      GemmT16Args g;
      g.x = xh16; g.T = T; g.ldo = ncol; g.out_zeroed = false;
      // Q|K|V stacked into one launch per run of equal weight type (their outputs are adjacent
      // columns of qkv_): one grid of 384 blocks at d = 4096 instead of three narrow ones
      const QMat* m[3] = {&L.t_wq, &L.t_wk, &L.t_wv};
      float* o[3] = {qkv_, qkv_ + nq_, qkv_ + nq_ + nkvd_};
      for (int i = 0; i < 3;) {
        int j = i + 1;
        while (j < 3 && m[j]->type == m[i]->type && m[j]->K == m[i]->K) ++j;
        g.w = *m[i]; g.out = o[i];
        g.nwseg = j - i;
        g.wseg_tiles[0] = m[i]->rows / 16;
        for (int k = 1; k < g.nwseg; ++k) {
          g.wseg_base[k] = m[i + k]->base;
          g.wseg_tiles[k] = m[i + k]->rows / 16;
          g.w.rows += m[i + k]->rows;
        }
        gemm_t16(g, GEMM_STORE, s);
        i = j;
      }
    } else {
      GemmArgs g;
      g.x = xb_; g.T = T; g.ldo = ncol; g.out_zeroed = true;
      g.w = L.wq; g.out = qkv_; gemm_dq(g, GEMM_STORE, s);
      g.w = L.wk; g.out = qkv_ + nq_; gemm_dq(g, GEMM_STORE, s);
      g.w = L.wv; g.out = qkv_ + nq_ + nkvd_; gemm_dq(g, GEMM_STORE, s);
    }
    if (!batched && segs_) {  // packed prompts: per-row slot / position, attention per piece
      __half* kcl = kc_ + kv_layer * (l - opt_.layer_begin);  // slot 0's layer l; + slot * slot_stride_
      __half* vcl = vc_ + kv_layer * (l - opt_.layer_begin);
      rope_kv_prefill(qkv_, T, 0, nq_, nkvd_, hd, opt_.n_ctx, rope_, q_, kcl, vcl, s, rpos_, rslots_, slot_stride_);
      // every piece in one launch (up to 16 per launch; grid z = pieces): the pieces of a joint
      // admission ran one launch each, ~100 blocks apiece on a 256-CU chip
      const std::vector<PrefillSeg>& sg = *segs_;
      const int G = nh_l_ / std::max(1, nkv_l_);
      const bool mfma = (G & (G - 1)) == 0 && G <= 16;
      for (size_t i0 = 0; i0 < sg.size();) {
        AttnPrefillArgs pa;
        pa.q = q_; pa.k_cache = kcl; pa.v_cache = vcl; pa.n_ctx = opt_.n_ctx;
        pa.n_head = nh_l_; pa.n_kv_head = nkv_l_; pa.head_dim = hd; pa.scale = 1.f / std::sqrt((float)hd);
        if (t16) pa.out_h = attnh16;
        else pa.out_bf16 = attnb_;
        pa.out_stride = nq_;
        if (mfma && pieces_attn_) {
          pa.slot_stride = slot_stride_;
          const size_t i1 = std::min(sg.size(), i0 + AttnPrefillArgs::kMaxPieces);
          for (size_t i = i0; i < i1; ++i) {
            const int k = (int)(i - i0);
            pa.pc_row[k] = sg[i].row; pa.pc_n[k] = sg[i].n; pa.pc_pos[k] = sg[i].pos; pa.pc_slot[k] = sg[i].slot;
          }
          pa.n_pieces = (int)(i1 - i0);
          attn_prefill(pa, s);
          i0 = i1;
          continue;
        }
        const PrefillSeg& g = sg[i0++];
        pa.q = q_ + (size_t)g.row * nq_;
        pa.k_cache = kcl + slot_stride_ * g.slot; pa.v_cache = vcl + slot_stride_ * g.slot;
        pa.T = g.n; pa.pos0 = g.pos;
        if (t16) pa.out_h = attnh16 + (size_t)g.row * nq_;
        else pa.out_bf16 = attnb_ + (size_t)g.row * nq_;
        attn_prefill(pa, s);
      }
    } else if (!batched) {
      __half* kcl = kc_ + slot_stride_ * kv_slot_ + kv_layer * (l - opt_.layer_begin);
      __half* vcl = vc_ + slot_stride_ * kv_slot_ + kv_layer * (l - opt_.layer_begin);
      rope_kv_prefill(qkv_, T, pos0, nq_, nkvd_, hd, opt_.n_ctx, rope_, q_, kcl, vcl, s);
      AttnPrefillArgs pa;
      pa.q = q_; pa.k_cache = kcl; pa.v_cache = vcl; pa.T = T; pa.pos0 = pos0; pa.n_ctx = opt_.n_ctx;
      pa.n_head = nh_l_; pa.n_kv_head = nkv_l_; pa.head_dim = hd; pa.scale = 1.f / std::sqrt((float)hd);
      if (t16) pa.out_h = attnh16;  // straight into the Wo GEMM's input (f16 / bf16)
      else pa.out_bf16 = attnb_;
      pa.out_stride = nq_;
      attn_prefill(pa, s);
    } else {  // T decode rows, each of its own KV slot and position
      __half* kcl = kc_ + kv_layer * (l - opt_.layer_begin);  // slot 0's layer l; the kernels add slot * slot_stride_
      __half* vcl = vc_ + kv_layer * (l - opt_.layer_begin);
      rope_kv_prefill(qkv_, T, 0, nq_, nkvd_, hd, opt_.n_ctx, rope_, q_, kcl, vcl, s, bpos_, bslots_, slot_stride_);
      AttnDecodeArgs aa;
      aa.q = q_; aa.k_cache = kcl; aa.v_cache = vcl; aa.pos = bpos_;
      aa.n_ctx = opt_.n_ctx; aa.n_head = nh_l_; aa.n_kv_head = nkv_l_; aa.head_dim = hd;
      aa.scale = 1.f / std::sqrt((float)hd);
      aa.part = attn_part_b_; aa.counters = attn_cnt_b_; aa.out = attn_;
      aa.batch = T; aa.slots = bslots_; aa.slot_stride = slot_stride_;
      aa.q_stride = nq_; aa.out_stride = nq_;
      aa.part_stride = attn_decode_workspace_floats(opt_.n_ctx, nh_l_, hd);
      attn_decode(aa, s);
      to_bf16(attn_, T * nq_, attnb_, s);
    }
    if (t16) {
      GemmT16Args o;
      o.w = L.t_wo; o.x = attnh16; o.T = T; o.ldo = d;
      if (!tp) {
        o.out = x_;
        gemm_t16(o, GEMM_ADD, s);
      } else {
        o.out = tmp_;
        o.resid = opt_.tp_rank == 0 ? x_ : nullptr;
        gemm_t16(o, GEMM_STORE, s);
        allreduce_into(tmp_, x_, (size_t)T * d, s);
      }
    } else {
      GemmArgs o;
      o.w = L.wo; o.x = attnb_; o.T = T; o.ldo = d;
      if (!tp) {
        o.out = x_;
        gemm_dq(o, GEMM_ADD, s);
      } else {
        o.out = tmp_;
        o.resid = opt_.tp_rank == 0 ? x_ : nullptr;
        gemm_dq(o, GEMM_STORE, s);
        allreduce_into(tmp_, x_, (size_t)T * d, s);
      }
    }
  }
  enqueue_rows_ffn(l, T, s, prefill_t16_ && !batched);
}

// The FFN half of a layer over T rows (prompt chunk or batched decode rows): RMSNorm ->
// gate/up (or MoE routing + grouped experts) -> down, residual into x_.
void Engine::enqueue_rows_ffn(int l, int T, hipStream_t s, bool t16) {
  const Layer& L = layers_[l];
  const int d = hp_.n_embd;
  const bool tp = tp_on_;
  // MoE: the router GEMM reads the bf16 norm; the experts' f16 norm is written after it
  rmsnorm_bf16(x_, L.ffn_norm, hp_.rms_eps, T, d, xb_, s, nullptr, 0, t16 && hp_.n_expert == 0);
  if (t16 && hp_.n_expert == 0) {
    GemmT16Args gu;
    gu.w = L.t_gu; gu.x = reinterpret_cast<const __half*>(xb_); gu.T = T;
    gu.out_h = reinterpret_cast<__half*>(h_); gu.ldh = F_l_;
    gemm_t16(gu, GEMM_SWIGLU, s);
    GemmT16Args dn;
    dn.w = L.t_down; dn.x = reinterpret_cast<const __half*>(h_); dn.T = T; dn.ldo = d;
    if (!tp) {
      dn.out = x_;
      gemm_t16(dn, GEMM_ADD, s);
    } else {
      dn.out = tmp_;
      dn.resid = opt_.tp_rank == 0 ? x_ : nullptr;
      gemm_t16(dn, GEMM_STORE, s);
      allreduce_into(tmp_, x_, (size_t)T * d, s);
    }
    return;
  }
  if (hp_.n_expert > 0) {
    const int E = hp_.n_expert;
    GemmArgs ra;
    ra.w = L.router; ra.x = xb_; ra.T = T; ra.out = router_logits_; ra.ldo = E;
    gemm_dq(ra, GEMM_STORE, s);
    const int KU = hp_.n_expert_used;
    // device-side routing -> per-expert row lists; gather the routed rows once
    moe_route_group(router_logits_, T, E, KU, moe_sel_, moe_selw_, moe_off_, moe_tok_, moe_gw_, moe_pos_, s);
    if (t16) rmsnorm_bf16(x_, L.ffn_norm, hp_.rms_eps, T, d, xb_, s, nullptr, 0, true);  // after the router read xb_
    gather_rows_bf16(xb_, moe_tok_, T * KU, d, moe_xg_, s);  // 2-byte rows: bf16 or f16 alike
    if (tp) {
      if (opt_.tp_rank == 0) HIPCHK(hipMemcpyAsync(tmp_, x_, sizeof(float) * T * d, hipMemcpyDeviceToDevice, s));
      else HIPCHK(hipMemsetAsync(tmp_, 0, sizeof(float) * T * d, s));
    }
    float* acc = tp ? tmp_ : x_;
    // split-K partials of the grouped down GEMMs meet by atomic add: zero the gathered output
    HIPCHK(hipMemsetAsync(moe_yg_, 0, sizeof(float) * (size_t)T * KU * d, s));
    const int hint = std::max(1, T * KU / E);
    for (int e = 0; t16 && e < E; ++e) {  // the tile16 expert copies (stacked gate/up, K-concatenated down)
      GemmT16Args gu;
      gu.w = L.gu_exps; gu.w.expert_stride = 0;
      gu.w.base = L.t_gu.base + t16_bytes(L.gu_exps.type, L.gu_exps.rows, L.gu_exps.K) * e;
      gu.x = reinterpret_cast<const __half*>(moe_xg_); gu.T = T;
      gu.out_h = reinterpret_cast<__half*>(moe_hg_); gu.ldh = F_l_;
      gu.seg_dev = moe_off_ + e; gu.rows_hint = hint;
      gemm_t16(gu, GEMM_SWIGLU, s);
      GemmT16Args dn;
      dn.w = L.down_exps; dn.w.expert_stride = 0; dn.w.base = L.t_down.base;
      dn.tile_stride = t16_bytes(L.down_exps.type, 16, L.t_down.K);  // one tile over all experts' K
      dn.step0 = e * (L.down_exps.K / 256);
      dn.x = reinterpret_cast<const __half*>(moe_hg_); dn.T = T; dn.ldo = d; dn.out = moe_yg_; dn.out_zeroed = true;
      dn.seg_dev = moe_off_ + e; dn.rows_hint = hint;
      gemm_t16(dn, GEMM_STORE, s);
    }
    for (int e = 0; !t16 && e < E; ++e) {  // each expert multiplies only its rows (count/offset read on the device)
      GemmArgs gu;
      gu.w = L.gu_exps; gu.w.base += L.gu_exps.expert_stride * e;
      gu.x = moe_xg_; gu.T = T; gu.out_bf16 = moe_hg_; gu.seg_dev = moe_off_ + e; gu.rows_hint = hint;
      gemm_dq(gu, GEMM_SWIGLU, s);
      GemmArgs dn;
      dn.w = L.down_exps; dn.w.base += L.down_exps.expert_stride * e;
      dn.x = moe_hg_; dn.T = T; dn.ldo = d; dn.out = moe_yg_; dn.seg_dev = moe_off_ + e; dn.rows_hint = hint;
      gemm_dq(dn, GEMM_STORE, s);
    }
    moe_scatter_add(acc, moe_yg_, moe_pos_, moe_gw_, T, KU, d, s);
    if (tp) allreduce_into(tmp_, x_, (size_t)T * d, s);
  } else {
    GemmArgs gu;
    gu.w = L.w_gu; gu.x = xb_; gu.T = T; gu.out_bf16 = h_;
    gemm_dq(gu, GEMM_SWIGLU, s);
    GemmArgs dn;
    dn.w = L.w_down; dn.x = h_; dn.T = T; dn.ldo = d;
    if (!tp) {
      dn.out = x_;
      gemm_dq(dn, GEMM_ADD, s);
    } else {
      dn.out = tmp_;
      dn.resid = opt_.tp_rank == 0 ? x_ : nullptr;
      gemm_dq(dn, GEMM_STORE, s);
      allreduce_into(tmp_, x_, (size_t)T * d, s);
    }
  }
}

// (two instantiations of every one-row graph: pipelined one-row steps alternate them as the
// batched ones do - an instance relaunched while its previous launch is still queued can be held
// back until that launch completes; launch_par_ picks the flight's instance)
void Engine::launch_step(int slot) {
  dslot_ = slot;
  if (opt_.use_graph) {
    if (slot == 0) {
      if (!graph_exec_) {
        HIPCHK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
        enqueue_decode(stream_);
        HIPCHK(hipStreamEndCapture(stream_, &graph_));
        HIPCHK(hipGraphInstantiate(&graph_exec_, graph_, nullptr, nullptr, 0));
        HIPCHK(hipGraphInstantiate(&graph_exec2_, graph_, nullptr, nullptr, 0));
      }
      HIPCHK(hipGraphLaunch(launch_par_ ? graph_exec2_ : graph_exec_, stream_));
    } else {
      if ((int)sgraph_.size() <= slot) {
        sgraph_.resize(slot + 1, nullptr);
        sgraph2_.resize(slot + 1, nullptr);
      }
      if (!sgraph_[slot]) {
        hipGraph_t g = nullptr;
        HIPCHK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
        enqueue_decode(stream_);
        HIPCHK(hipStreamEndCapture(stream_, &g));
        hipError_t e = hipGraphInstantiate(&sgraph_[slot], g, nullptr, nullptr, 0);
        if (e == hipSuccess) e = hipGraphInstantiate(&sgraph2_[slot], g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        HIPCHK(e);
      }
      HIPCHK(hipGraphLaunch(launch_par_ ? sgraph2_[slot] : sgraph_[slot], stream_));
    }
  } else {
    enqueue_decode(stream_);
  }
  dslot_ = 0;
}

// ------------------------------------------------------------------------ generation
SamplerParamsDev Engine::make_sparams(const SamplingOpts& sp) const {
  if (sp.top_k < 0 || sp.top_k > 64) throw std::runtime_error("GPU sampler: top_k must be in [0, 64]");
  SamplerParamsDev p;
  p.greedy = sp.temp <= 0.f ? 1 : 0;
  p.top_k = p.greedy ? 1 : (sp.top_k == 0 ? 64 : sp.top_k);
  p.top_p = sp.top_p; p.min_p = sp.min_p; p.temp = sp.temp;
  p.repeat_penalty = sp.repeat_penalty; p.freq_penalty = sp.freq_penalty; p.presence_penalty = sp.presence_penalty;
  p.last_n = std::min(sp.last_n, 64);
  p.seed = sp.seed;
  p.tfs_z = sp.tfs_z; p.typical_p = sp.typical_p;
  if ((int)sp.logit_bias.size() > kMaxLogitBias) throw std::runtime_error("GPU sampler: at most 64 logit_bias entries");
  for (const auto& [t, b] : sp.logit_bias) {
    if (t < 0 || t >= hp_.n_vocab) continue;  // out-of-vocabulary entries are ignored (as upstream)
    for (int j = 0; j < p.n_bias; ++j)
      if (p.bias_tok[j] == t) throw std::runtime_error("GPU sampler: duplicate logit_bias token");
    p.bias_tok[p.n_bias] = t;
    p.bias_val[p.n_bias++] = b;
  }
  return p;
}

// Sampling params, penalty ring (prompt tail) and counters of one slot's request.
void Engine::begin_slot_state(int slot, const std::vector<int>& prompt, const SamplingOpts& sp) {
  const SamplerParamsDev p = make_sparams(sp);
  const int n_prompt = (int)prompt.size();
  int hstate[S_NSTATE] = {0};
  int hring[64] = {0};
  const int rl = std::min(n_prompt, 64);
  for (int i = 0; i < rl; ++i) hring[i] = prompt[n_prompt - rl + i];
  hstate[S_TOKEN] = prompt.back();
  hstate[S_POS] = n_prompt;  // position the first generated token will occupy
  hstate[S_RING_LEN] = rl;
  hstate[S_RING_HEAD] = rl & 63;
  HIPCHK(hipMemcpyAsync(sparams_ + slot, &p, sizeof(p), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemcpyAsync(ring_ + 64 * slot, hring, sizeof(hring), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemcpyAsync(state_ + (size_t)S_NSTATE * slot, hstate, sizeof(hstate), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipStreamSynchronize(stream_));  // the host arrays are on this stack frame
}

// bmm over B rows: groups of kBmmMaxRows columns (one more weight stream per group)
void Engine::bmm_rows(const QMat& w, const __half* xh, int ldh, float* out, int ldo, int n_out, int B,
                      hipStream_t s, long long* dbg) {
  for (int b0 = 0; b0 < B; b0 += kBmmMaxRows) {
    BmmArgs a;
    a.dbg_clk = b0 == 0 ? dbg : nullptr;
    a.w = w; a.xh = xh + (size_t)b0 * ldh; a.ldh = ldh;
    a.out = out + (size_t)b0 * ldo; a.ldo = ldo; a.n_out = n_out;
    a.B = std::min(kBmmMaxRows, B - b0);
    bmm(a, s);
  }
}

// the down projection (split-K into the residual); with the split-K Q|K|V (`zero_qkv`) its blocks
// also re-zero qkv_b_ / ss_b_ for the next layer (the attention, their only reader, has finished)
void Engine::down_rows(const QMat& w, const __half* xh, int ldh, float* out, int B, hipStream_t s, bool zero_qkv,
                       long long* dbg) {
  const int d = hp_.n_embd;
  BmmArgs a;
  a.w = w; a.xh = xh; a.ldh = ldh; a.out = out; a.ldo = d; a.n_out = d; a.B = B; a.dbg_clk = dbg;
  if (zero_qkv) {
    a.zero = qkv_b_; a.zero_n = (int)qkv_b_zero_n();
  }
  bmm(a, s);
}

void Engine::bprep_rows(const float* x, int ldx, bool swiglu, const float* norm_w, int K, int B, float* zero,
                        int zero_n, hipStream_t s, int swiglu_group) {
  BPrepArgs p;
  p.swiglu_group = swiglu_group;
  p.x = x; p.ldx = ldx; p.swiglu = swiglu; p.norm_w = norm_w; p.eps = hp_.rms_eps;
  p.K = K; p.B = B; p.xh = xh_b_; p.ldh = K; p.zero = zero; p.zero_n = zero_n;
  bprep(p, s);
}

// One layer of batch_step on the MFMA batched projections (bmm.hip). Every projection input
// is prepared once (bprep: norm / SwiGLU, f16) and that launch also zeroes the split-K output
// of the projection it feeds (qkv_, gu_b_); Wo and down accumulate into the residual x_.
void Engine::enqueue_batch_layer(int l, int B, hipStream_t s) {
  const Layer& L = layers_[l];
  const int d = hp_.n_embd, hd = hp_.head_dim, ncol = nq_ + 2 * nkvd_;
  // row-parallel Wo / down under TP: accumulate this rank's partial into tmp_ (holding the
  // residual on rank 0, zeros elsewhere), then all-reduce into x_
  // P2P path: the partials go to tmp_b_, which the accumulating all-reduce (x_ += sum) leaves zeroed
  // for the next projection - no copy / fill node per collective. RCCL fallback: the residual seeds
  // rank 0's tmp_, zeros the others', and the all-reduce stores the sum into x_.
  const bool tp = tp_on_;
  const bool tp_acc = tp && tmp_b_ && p2p_ && p2p_->ready() && (size_t)B * d <= (size_t)p2p_->max_n();
  float* acc = tp_acc ? tmp_b_ : tp ? tmp_ : x_;
  auto tp_begin = [&]() {
    if (!tp || tp_acc) return;
    if (opt_.tp_rank == 0) HIPCHK(hipMemcpyAsync(tmp_, x_, sizeof(float) * B * d, hipMemcpyDeviceToDevice, s));
    else HIPCHK(hipMemsetAsync(tmp_, 0, sizeof(float) * B * d, s));
  };
  auto tp_end = [&]() {
    if (tp_acc) p2p_->allreduce_add(tmp_b_, x_, B * d, s);
    else if (tp) allreduce_into(tmp_, x_, (size_t)B * d, s);
  };
  const size_t kv_layer = (size_t)nkv_l_ * opt_.n_ctx * hd;
  __half* kcl = kc_ + kv_layer * (l - opt_.layer_begin);  // slot 0's layer l; the kernels add slot * slot_stride_
  __half* vcl = vc_ + kv_layer * (l - opt_.layer_begin);
  // RoPE + KV append in the Q|K|V epilogue when the whole K fits one LDS-staged part
  const bool fused = B <= kBmmMaxRows && bmm_qkv_fits(d, B);
  // attention / FFN RMSNorm folded into the one-part projections' x staging (no prep launch)
  const bool fnorm = fused && bmm_norm_fits(d, B);
  // Q|K|V split over K (the default at B <= 8): RoPE'd partial sums into qkv_b_, normalised and
  // appended to the caches by the attention
  const bool sk = qkv_sk_ && bmm_qkv_sk_supported(L.t_wq.type, L.t_wk.type, L.t_wv.type, d, B);
  // FFN paths without the down projection's zero side job: a memset node re-zeroes qkv_b_ / ss_b_
  auto zero_qkv = [&]() {
    if (sk) HIPCHK(hipMemsetAsync(qkv_b_, 0, sizeof(float) * qkv_b_zero_n(), s));
  };
  if (sk) {
    BmmArgs a;
    a.w = L.t_wq; a.n_out = L.t_wq.rows; a.out = qkv_b_; a.ldo = ncol; a.B = B;
    a.nseg = 3;
    a.seg_base[1] = L.t_wk.base; a.seg_rows[1] = L.t_wk.rows; a.seg_out[1] = qkv_b_ + nq_;
    a.seg_base[2] = L.t_wv.base; a.seg_rows[2] = L.t_wv.rows; a.seg_out[2] = qkv_b_ + nq_ + nkvd_;
    const int tq = L.t_wq.type, tk = L.t_wk.type, tv = L.t_wv.type;
    a.seg_split = tk != tq ? 1 : tv != tq ? 2 : 3;
    a.type2 = tk != tq ? tk : tv != tq ? tv : 0;
    a.qkv_sk = true;
    a.qkv.pos = bpos_; a.qkv.rope = rope_; a.qkv.head_dim = hd; a.qkv.n_ctx = opt_.n_ctx;
    a.xf = x_; a.ldxf = d; a.norm_w = L.attn_norm; a.eps = hp_.rms_eps; a.ss_out = ss_b_;
    a.dbg_clk = clk_of(l, 0);
    bmm(a, s);
  } else {
    if (!fnorm) bprep_rows(x_, d, false, L.attn_norm, d, B, fused ? nullptr : qkv_, fused ? 0 : B * ncol, s);
    // Q|K|V: one launch per run of equal weight type (Q4_K_M: one, or Q|K + V on bumped layers;
    // a side-stream graph branch for the V run measured no gain)
    const QMat* m[3] = {&L.t_wq, &L.t_wk, &L.t_wv};
    float* o[3] = {qkv_, qkv_ + nq_, qkv_ + nq_ + nkvd_};
    std::vector<BmmArgs> rl;
    for (int i = 0; i < 3;) {
      int j = i + 1;
      while (j < 3 && m[j]->type == m[i]->type) ++j;
      for (int b0 = 0; b0 < B; b0 += kBmmMaxRows) {
        BmmArgs a;
        a.w = *m[i]; a.xh = xh_b_ + (size_t)b0 * d; a.ldh = d;
        a.out = o[i] + (size_t)b0 * ncol; a.ldo = ncol; a.n_out = m[i]->rows;
        a.B = std::min(kBmmMaxRows, B - b0);
        a.nseg = j - i;
        for (int k = 1; k < a.nseg; ++k) {
          a.seg_base[k] = m[i + k]->base; a.seg_rows[k] = m[i + k]->rows; a.seg_out[k] = o[i + k] + (size_t)b0 * ncol;
        }
        if (fnorm) {
          a.xf = x_ + (size_t)b0 * d; a.ldxf = d; a.norm_w = L.attn_norm; a.eps = hp_.rms_eps;
        }
        if (rl.empty() && b0 == 0) a.dbg_clk = clk_of(l, 0);
        if (fused) {
          a.qkv_epi = true;
          for (int k = 0; k < a.nseg; ++k) a.qkv.kind[k] = i + k;
          a.qkv.q_out = q_ + (size_t)b0 * nq_; a.qkv.q_ld = nq_;
          a.qkv.k_cache = kcl; a.qkv.v_cache = vcl; a.qkv.slot_stride = slot_stride_;
          a.qkv.n_ctx = opt_.n_ctx; a.qkv.head_dim = hd;
          a.qkv.pos = bpos_ + b0; a.qkv.slots = bslots_ + b0; a.qkv.rope = rope_;
        }
        rl.push_back(a);
      }
      i = j;
    }
    // bumped layers (Q|K Q4_K + V Q6_K): both runs in one launch
    if (!(rl.size() == 2 && B <= kBmmMaxRows && bmm_qkv2(rl[0], rl[1], s)))
      for (const BmmArgs& a : rl) bmm(a, s);
    if (!fused)
      rope_kv_prefill(qkv_, B, 0, nq_, nkvd_, hd, opt_.n_ctx, rope_, q_, kcl, vcl, s, bpos_, bslots_, slot_stride_);
  }
  AttnDecodeArgs aa;
  aa.q = q_; aa.k_cache = kcl; aa.v_cache = vcl; aa.pos = bpos_;
  aa.n_ctx = opt_.n_ctx; aa.n_head = nh_l_; aa.n_kv_head = nkv_l_; aa.head_dim = hd;
  aa.scale = 1.f / std::sqrt((float)hd);
  aa.part = attn_part_b_; aa.counters = attn_cnt_b_; aa.out = attn_;
  aa.batch = B; aa.slots = bslots_; aa.slot_stride = slot_stride_;
  aa.q_stride = nq_; aa.out_stride = nq_;
  aa.part_stride = attn_decode_workspace_floats(opt_.n_ctx, nh_l_, hd);
  aa.out_h = xh_b_; aa.out_h_stride = nq_;   // the Wo input, already in bmm's f16 layout
  aa.out = nullptr;                          // (nothing reads an f32 copy of it)
  if (sk) {
    aa.qkv_raw = qkv_b_; aa.qkv_ld = ncol; aa.k_off = nq_; aa.v_off = nq_ + nkvd_;
    aa.ss = ss_b_; aa.inv_k = 1.f / (float)d; aa.eps = hp_.rms_eps;
    if (bmm_qkv_sk_defers_rope()) aa.rope_freq = rope_freq_;
  }
  aa.dbg_clk = clk_of(l, 1);
  // (the batched Wo stays its own launch: in one launch with the attention - Wo planes streaming
  // their weights meanwhile and starting on done counters - the B = 6 step measured 2.42 vs 2.34
  // ms, r4: the in-launch hand-off costs what the boundary did and the weight stream slowed the
  // attention's K / V loads)
  attn_decode(aa, s);
  // dense FFN on the SwiGLU epilogue path: its gate/up and down (and, ffn_chain_ 2, Wo before them)
  BmmArgs wo, gu, dn;
  wo.w = L.t_wo; wo.xh = xh_b_; wo.ldh = nq_; wo.out = acc; wo.ldo = d; wo.n_out = d; wo.B = B;
  wo.dbg_clk = clk_of(l, 2);
  const bool dense_ffn = !(moe_b_ && fused) && bg_ffn_ && fused;
  if (dense_ffn) {
    if (fnorm) {
      gu.xf = x_; gu.ldxf = d; gu.norm_w = L.ffn_norm; gu.eps = hp_.rms_eps;
    }
    gu.w = L.t_gu; gu.xh = xh_b_; gu.ldh = d;
    gu.out = nullptr; gu.ldo = 0; gu.n_out = 2 * F_l_; gu.B = B;
    gu.swiglu_epi = true; gu.h_out = hh_b_; gu.ldh_out = F_l_;
    gu.dbg_clk = clk_of(l, 3);
    dn.w = L.t_down; dn.xh = hh_b_; dn.ldh = F_l_; dn.out = acc; dn.ldo = d; dn.n_out = d; dn.B = B;
    dn.dbg_clk = clk_of(l, 4);
    if (sk) {  // (the down projection re-zeroes the split-K Q|K|V rows for the next layer)
      dn.zero = qkv_b_; dn.zero_n = (int)qkv_b_zero_n();
    }
    // Wo, gate/up and down in ONE launch: the gate/up blocks start on the CUs the Wo frees and issue
    // their weights while the last Wo partials land (bmm_wo_ffn_chain)
    if (ffn_chain_ >= 2 && !tp && fnorm && B <= kBmmMaxRows && bmm_wo_ffn_chain_supported(wo, gu, dn)) {
      bmm_wo_ffn_chain(wo, gu, dn, chain_cnt_ + kChainInts * l, chain_err_, s);
      return;
    }
  }
  tp_begin();
  if (B <= kBmmMaxRows) bmm(wo, s);
  else bmm_rows(L.t_wo, xh_b_, nq_, acc, d, d, B, s, clk_of(l, 2));
  tp_end();
  if (moe_b_ && fused) {
    // MoE: dense per-row expert weights (f32 router on the normed rows), then every expert's
    // SwiGLU rows in ONE gate/up launch (epilogue scaled by the row's weight for that expert,
    // 0 when unrouted) and ONE down launch over the K-concatenated experts (parts of unrouted
    // experts skipped): two weight streams per layer instead of a GEMM pair per expert
    const int E = hp_.n_expert;
    moe_router_rows(x_, d, B, L.ffn_norm, hp_.rms_eps, reinterpret_cast<const float*>(L.router.base), d, E,
                    hp_.n_expert_used, ew_b_, E, s);
    BmmArgs a;
    if (fnorm) {
      a.xf = x_; a.ldxf = d; a.norm_w = L.ffn_norm; a.eps = hp_.rms_eps;
    } else {
      bprep_rows(x_, d, false, L.ffn_norm, d, B, nullptr, 0, s);
    }
    a.w = L.t_gu; a.xh = xh_b_; a.ldh = d;
    a.out = nullptr; a.ldo = 0; a.n_out = L.t_gu.rows; a.B = B;
    a.swiglu_epi = true; a.h_out = hh_b_; a.ldh_out = E * F_l_;
    a.ew = ew_b_; a.ew_ld = E; a.tiles_per_expert = 2 * F_l_ / 16;
    bmm(a, s);
    tp_begin();
    BmmArgs dn;
    dn.w = L.t_down; dn.xh = hh_b_; dn.ldh = E * F_l_;
    dn.out = acc; dn.ldo = d; dn.n_out = d; dn.B = B;
    dn.ew = ew_b_; dn.ew_ld = E; dn.steps_per_expert = F_l_ / 256;
    if (sk) {  // (the wave-owned down re-zeroes the split-K Q|K|V rows as a side job)
      dn.zero = qkv_b_; dn.zero_n = (int)qkv_b_zero_n();
    }
    bmm(dn, s);
    tp_end();
    return;
  }
  if (dense_ffn) {
    // SwiGLU in the gate/up epilogue: one K part, silu(gate) * up straight to the down
    // projection's f16 input (hh_b_; xh_b_ is still being read by other blocks)
    if (!fnorm) bprep_rows(x_, d, false, L.ffn_norm, d, B, nullptr, 0, s);
    // gate/up and down in ONE launch, the down blocks waiting per K part on the gate/up tiles
    // they read (bmm_ffn_chain): the down weight stream starts under the gate/up's last tiles
    // instead of after a kernel boundary
    // (under TP with more than two ranks on ONE GPU - the eight-rank rehearsal - the chain's down
    // blocks, waiting on their gate/up, and the peers' spinning collectives can hold each other's
    // CUs: a 2 s chain timeout in r5; the same rule as tp_epilogue's)
    const bool tp_chain = tp_acc && !(p2p_->shared_device() && p2p_->world() > 2);
    if (ffn_chain_ >= 1 && (!tp || tp_chain) && bmm_ffn_chain_supported(gu, dn)) {
      bmm_ffn_chain(gu, dn, chain_cnt_ + kChainInts * l, chain_err_, s);
      tp_end();
      return;
    }
    bmm(gu, s);
    tp_begin();
    bmm(dn, s);
    tp_end();
    return;
  }
  if (bg_ffn_) {
    bprep_rows(x_, d, false, L.ffn_norm, d, B, gu_b_, B * 2 * F_l_, s);
    bmm_rows(L.t_gu, xh_b_, d, gu_b_, 2 * F_l_, 2 * F_l_, B, s);
    bprep_rows(gu_b_, 2 * F_l_, true, nullptr, F_l_, B, nullptr, 0, s, /*swiglu_group=*/8);  // t_gu: SwiGLU copy
    tp_begin();
    down_rows(L.t_down, xh_b_, F_l_, acc, B, s, sk);
    tp_end();
    return;
  }
  // MoE (or unsupported FFN types): the grouped-GEMM FFN of the prompt path over the B rows
  enqueue_rows_ffn(l, B, s);
  zero_qkv();
}

// The device work of one batch step over B rows (slots / positions / tokens are read from
// device memory, so one captured graph per B serves every step).
void Engine::enqueue_batch_step(int B, hipStream_t s) {
  const int d = hp_.n_embd;
  // (its launch also zeroes the FFN chain counters of every layer)
  batch_gather_embed(bslots_, B, state_, btok_, bpos_, tok_embd_, x_, s, chain_cnt_,
                     chain_cnt_ ? kChainInts / kChainStride * hp_.n_layer : 0, kChainStride);
  if (bg_) {
    for (int l = 0; l < hp_.n_layer; ++l) enqueue_batch_layer(l, B, s);
    // the head stores its logits (one K part, plain stores: no zeroed rows to add into); the
    // store-only epilogue runs on the wave-owned kernel, which takes at most 8 rows per launch
    bprep_rows(x_, d, false, out_norm_, d, B, nullptr, 0, s);
    constexpr int kHeadRows = 8;
    for (int b0 = 0; b0 < B; b0 += kHeadRows) {
      BmmArgs h;
      h.w = t_output_; h.xh = xh_b_ + (size_t)b0 * d; h.ldh = d;
      h.out = logits_b_ + (size_t)b0 * V_pad_; h.ldo = V_pad_; h.n_out = V_l_;
      h.B = std::min(kHeadRows, B - b0);
      h.store_out = true;
      bmm(h, s);
    }
  } else {
    for (int l = 0; l < hp_.n_layer; ++l) enqueue_rows_layer(l, B, 0, true, s);
    rmsnorm_bf16(x_, out_norm_, hp_.rms_eps, B, d, xb_, s);
    GemmArgs h;
    h.w = output_; h.x = xb_; h.T = B; h.out = logits_b_; h.ldo = V_pad_;
    gemm_dq(h, GEMM_STORE, s);
  }
  enqueue_sample(logits_b_, B, V_pad_, 0, 1, s);
}



// ------------------------------------------------------------------------ tensor-parallel control
// Commands rank 0 publishes before enqueueing the matching device work (tp_channel.h).
enum TPOp : int32_t {
  TPO_STOP = 1,
  TPO_SLOT_STATE,   // generate(): slot, prompt, sampling
  TPO_PREFILL,      // generate(): slot, pos, head?, tokens of one chunk
  TPO_DECODE_STEP,  // generate(): one graph-replayed decode step
  TPO_SYNC,         // generate(): end of the request
  TPO_SLOT_BEGIN,   // slot_begin()
  TPO_BATCH_STEP,   // batch_step()
  TPO_EVAL_LOGITS,  // eval_logits()
  TPO_DECODE_LOGITS,
  TPO_BATCH_LOGITS,
  TPO_BENCH_DECODE,
  TPO_SLOTS_BEGIN,  // slots_begin(): n, slots, n_keep, then n x (prompt, sampling)
  TPO_BATCH_LAUNCH,   // batch_launch(): slots (pipelined steps: queued, not waited for)
  TPO_BATCH_COLLECT,  // batch_collect(): the oldest step in flight
};

static void put_sp(TPMsg& m, const SamplingOpts& sp) {
  m.put(sp.top_k); m.put(sp.top_p); m.put(sp.min_p); m.put(sp.temp);
  m.put(sp.repeat_penalty); m.put(sp.freq_penalty); m.put(sp.presence_penalty);
  m.put(sp.last_n); m.put(sp.seed); m.put(sp.tfs_z); m.put(sp.typical_p);
  m.put_vec(sp.logit_bias);
}

static SamplingOpts get_sp(TPMsg& m) {
  SamplingOpts sp;
  sp.top_k = m.get<int>(); sp.top_p = m.get<float>(); sp.min_p = m.get<float>(); sp.temp = m.get<float>();
  sp.repeat_penalty = m.get<float>(); sp.freq_penalty = m.get<float>(); sp.presence_penalty = m.get<float>();
  sp.last_n = m.get<int>(); sp.seed = m.get<unsigned long long>(); sp.tfs_z = m.get<float>();
  sp.typical_p = m.get<float>();
  sp.logit_bias = m.get_vec<std::pair<int, float>>();
  return sp;
}

void Engine::mirror(const TPMsg& m) {
  if (opt_.tp_size < 2) return;
  if (opt_.tp_rank != 0) throw std::runtime_error("tensor parallelism: follower ranks only run follow()");
  if (!tp_ctl_) throw std::runtime_error("tensor parallelism: the control channel is not open (tp_ctl_create)");
  if (tp_stopped_) throw std::runtime_error("tensor parallelism: the group was stopped");
  // a poisoned group (a rank's wait timed out, a follower failed or exited) runs no further step:
  // its ranks' states have diverged, so every later result would be computed from stale data
  if (!healthy_) throw std::runtime_error("tensor parallelism: the group is poisoned (" + last_error_ + ")");
  const std::string f = group_fault();
  if (!f.empty()) {
    healthy_ = false;
    last_error_ = "tensor-parallel group fault: " + f;
    throw std::runtime_error(last_error_);
  }
  tp_ctl_->publish(m);
}

void Engine::tp_ctl_create(const std::string& name) {
  if (opt_.tp_size < 2 || opt_.tp_rank != 0) throw std::runtime_error("tp_ctl_create: rank 0 of a TP group only");
  // largest command: a prefill chunk / a whole prompt plus sampling options - or one of those
  // per KV slot (a joint admission, slots_begin)
  const size_t one = 256 + sizeof(int) * (size_t)std::max(opt_.n_ctx, opt_.n_batch) + 16 * kMaxLogitBias;
  const size_t cap = 4096 + one * (size_t)std::max(1, bmax_);
  tp_ctl_ = TPChannel::create(name, opt_.tp_size, cap);
}

void Engine::tp_ctl_attach(const std::string& name) {
  if (opt_.tp_size < 2 || opt_.tp_rank == 0) throw std::runtime_error("tp_ctl_attach: follower ranks only");
  tp_ctl_ = TPChannel::attach(name, opt_.tp_rank);
  // (the fault-injection hook, EngineOptions::test_fault, was parsed by the constructor)
}

void Engine::tp_stop() {
  if (!leader() || !tp_ctl_ || tp_stopped_) return;
  ExecGuard guard(this);
  TPMsg m;
  m.put<int32_t>(TPO_STOP);
  tp_ctl_->publish(m);
  tp_stopped_ = true;
}

// Follower ranks: replay rank 0's commands until TPO_STOP. A failing command marks this
// rank unhealthy and publishes the failure (channel word + every rank's region fault word), so
// rank 0 fails the request in flight and refuses further steps; the loop goes on, so a later
// STOP still ends it.
void Engine::follow() {
  if (!tp_ctl_ || opt_.tp_rank == 0) throw std::runtime_error("follow: attach a follower rank first");
  TPMsg m;
  while (true) {
    if (!tp_ctl_->receive(m, 1000)) {
      if (!tp_ctl_->leader_alive()) throw std::runtime_error("follow: rank 0 exited without stopping the group");
      continue;
    }
    const int32_t op = m.get<int32_t>();
    ExecGuard guard(this);
    if (op == TPO_STOP) {
      HIPCHK(hipStreamSynchronize(stream_));
      return;
    }
    try {
      if (fault_after_ > 0 && --fault_after_ == 0) {
        if (!fault_dev_) throw std::runtime_error("injected follower fault (test hook)");
        if (p2p_ && p2p_->ready()) p2p_->raise_fault(300 + opt_.tp_rank);  // as a timed-out epilogue wait
      }
      switch (op) {
        case TPO_SLOT_STATE: {
          const int slot = m.get<int>();
          const std::vector<int> prompt = m.get_vec<int>();
          begin_slot_state(slot, prompt, get_sp(m));
          break;
        }
        case TPO_PREFILL: {
          const int slot = m.get<int>(), pos = m.get<int>(), head = m.get<int>();
          const std::vector<int> toks = m.get_vec<int>();
          prefill_chunk(slot, toks.data(), (int)toks.size(), pos, head != 0);
          break;
        }
        case TPO_DECODE_STEP: launch_step(); break;
        case TPO_SYNC:
          HIPCHK(hipStreamSynchronize(stream_));
          check_device_err();
          break;
        case TPO_SLOT_BEGIN: {
          const int slot = m.get<int>(), n_keep = m.get<int>();
          const std::vector<int> prompt = m.get_vec<int>();
          slot_begin_impl(slot, prompt, n_keep, get_sp(m));
          break;
        }
        case TPO_SLOTS_BEGIN: {
          const int n = m.get<int>();
          const std::vector<int> slots = m.get_vec<int>(), keep = m.get_vec<int>();
          std::vector<std::vector<int>> prompts(n);
          std::vector<SamplingOpts> sps(n);
          for (int i = 0; i < n; ++i) {
            prompts[i] = m.get_vec<int>();
            sps[i] = get_sp(m);
          }
          slots_begin_impl(slots, prompts, keep, sps);
          break;
        }
        case TPO_BATCH_STEP: batch_step_impl(m.get_vec<int>()); break;
        case TPO_BATCH_LAUNCH: batch_launch_impl(m.get_vec<int>()); break;
        case TPO_BATCH_COLLECT: batch_collect_impl(); break;
        case TPO_EVAL_LOGITS: {
          const int pos0 = m.get<int>();
          eval_logits_impl(m.get_vec<int>(), pos0);
          break;
        }
        case TPO_DECODE_LOGITS: {
          const int tok = m.get<int>(), pos = m.get<int>();
          decode_logits_impl(tok, pos);
          break;
        }
        case TPO_BATCH_LOGITS: batch_logits_impl(m.get<int>()); break;
        case TPO_BENCH_DECODE: {
          const int n = m.get<int>(), pos0 = m.get<int>();
          bench_decode_impl(n, pos0);
          break;
        }
        default: throw std::runtime_error("follow: unknown command " + std::to_string(op));
      }
    } catch (const std::exception& e) {
      healthy_ = false;
      last_error_ = std::string("follower rank ") + std::to_string(opt_.tp_rank) + ": " + e.what();
      fprintf(stderr, "[lfk] %s\n", last_error_.c_str());
      // rank 0 must learn of it (its next command or collect fails, /health turns false) and the
      // other ranks' kernels must stop waiting for this one: the channel word and the region's
      try {
        tp_ctl_->report_fault(e.what());
        // (a group already poisoned keeps the code of the rank that failed first)
        if (p2p_ && p2p_->ready() && p2p_->fault_report().empty()) p2p_->raise_fault(1000 + opt_.tp_rank);
      } catch (...) {
      }
    }
  }
}

// ------------------------------------------------------------------------ serving entry points
// Each takes the execution guard, validates its arguments (so a follower never receives a
// command that fails validation), publishes the command under TP, then runs the *_impl.

void Engine::prefill_chunk(int slot, const int* toks, int T, int pos, bool head) {
  kv_slot_ = slot;
  try {
    std::memcpy(h_tokens_, toks, sizeof(int) * T);
    HIPCHK(hipMemcpyAsync(tokens_, h_tokens_, sizeof(int) * T, hipMemcpyHostToDevice, stream_));
    enqueue_prefill(T, pos, stream_);
    if (head) enqueue_head(x_ + (size_t)(T - 1) * hp_.n_embd, 0, stream_, slot);
    HIPCHK(hipStreamSynchronize(stream_));  // h_tokens_ is reused by the next chunk
  } catch (...) {
    kv_slot_ = 0;
    throw;
  }
  kv_slot_ = 0;
}

int Engine::slot_begin(int slot, const std::vector<int>& prompt, int n_keep, const SamplingOpts& sp) {
  ExecGuard guard(this);
  if (!bmax_) throw std::runtime_error("slot_begin: the engine was built with one KV slot");
  if (slot < 0 || slot >= opt_.n_slots) throw std::runtime_error("slot_begin: slot out of range");
  const int n_prompt = (int)prompt.size();
  if (n_prompt == 0) throw std::runtime_error("empty prompt");
  if (n_prompt >= opt_.n_ctx) throw std::runtime_error("prompt exceeds context window");
  (void)make_sparams(sp);  // validates top_k / logit_bias before any rank starts
  if (n_keep < 0 || n_keep >= n_prompt) n_keep = 0;
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_SLOT_BEGIN); m.put(slot); m.put(n_keep); m.put_vec(prompt); put_sp(m, sp);
    mirror(m);
  }
  return slot_begin_impl(slot, prompt, n_keep, sp);
}

int Engine::slot_begin_part(int slot, const std::vector<int>& prompt, int n_keep, int n_done, int n,
                            const SamplingOpts& sp) {
  ExecGuard guard(this);
  if (!bmax_ || tp_on_) throw std::runtime_error("slot_begin_part: batching engines on one GPU only");
  if (slot < 0 || slot >= opt_.n_slots) throw std::runtime_error("slot_begin_part: slot out of range");
  const int n_prompt = (int)prompt.size();
  if (n_prompt == 0) throw std::runtime_error("empty prompt");
  if (n_prompt >= opt_.n_ctx) throw std::runtime_error("prompt exceeds context window");
  if (n_keep < 0 || n_keep >= n_prompt) n_keep = 0;
  if (n_done < n_keep || n_done >= n_prompt || n < 1) throw std::runtime_error("slot_begin_part: bad part");
  if (n_done == n_keep) {
    (void)make_sparams(sp);
    begin_slot_state(slot, prompt, sp);
  }
  const int end = std::min(n_prompt, n_done + n);
  for (int pos = n_done; pos < end;) {
    const int T = std::min(opt_.n_batch, end - pos);
    prefill_chunk(slot, prompt.data() + pos, T, pos, pos + T == n_prompt);
    pos += T;
  }
  if (end < n_prompt) return -1;
  int tok = 0;
  HIPCHK(hipMemcpy(&tok, state_ + (size_t)S_NSTATE * slot + S_TOKEN, sizeof(int), hipMemcpyDeviceToHost));
  check_device_err();
  return tok;
}

int Engine::slot_begin_impl(int slot, const std::vector<int>& prompt, int n_keep, const SamplingOpts& sp) {
  const int n_prompt = (int)prompt.size();
  begin_slot_state(slot, prompt, sp);
  int pos = n_keep;
  while (pos < n_prompt) {
    const int T = std::min(opt_.n_batch, n_prompt - pos);
    prefill_chunk(slot, prompt.data() + pos, T, pos, pos + T == n_prompt);
    pos += T;
  }
  int tok = 0;
  HIPCHK(hipMemcpy(&tok, state_ + (size_t)S_NSTATE * slot + S_TOKEN, sizeof(int), hipMemcpyDeviceToHost));
  check_device_err();
  return tok;
}

std::vector<int> Engine::slots_begin(const std::vector<int>& slots, const std::vector<std::vector<int>>& prompts,
                                     const std::vector<int>& n_keep, const std::vector<SamplingOpts>& sps) {
  ExecGuard guard(this);
  const size_t n = slots.size();
  if (!bmax_) throw std::runtime_error("slots_begin: the engine was built with one KV slot");
  if (prompts.size() != n || n_keep.size() != n || sps.size() != n) throw std::runtime_error("slots_begin: sizes");
  std::vector<int> keep(n_keep);
  for (size_t i = 0; i < n; ++i) {
    if (slots[i] < 0 || slots[i] >= opt_.n_slots) throw std::runtime_error("slots_begin: slot out of range");
    for (size_t j = 0; j < i; ++j)
      if (slots[j] == slots[i]) throw std::runtime_error("slots_begin: duplicate slot");
    const int np = (int)prompts[i].size();
    if (np == 0) throw std::runtime_error("empty prompt");
    if (np >= opt_.n_ctx) throw std::runtime_error("prompt exceeds context window");
    (void)make_sparams(sps[i]);
    if (keep[i] < 0 || keep[i] >= np) keep[i] = 0;
  }
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_SLOTS_BEGIN); m.put((int)n); m.put_vec(slots); m.put_vec(keep);
    for (size_t i = 0; i < n; ++i) {
      m.put_vec(prompts[i]);
      put_sp(m, sps[i]);
    }
    mirror(m);
  }
  return slots_begin_impl(slots, prompts, keep, sps);
}

std::vector<int> Engine::slots_begin_impl(const std::vector<int>& slots, const std::vector<std::vector<int>>& prompts,
                                          const std::vector<int>& n_keep, const std::vector<SamplingOpts>& sps) {
  const size_t n = slots.size();
  for (size_t i = 0; i < n; ++i) begin_slot_state(slots[i], prompts[i], sps[i]);
  const int NB = nb_cap_, d = hp_.n_embd;
  int* h_tok = h_rmeta_;
  int* h_pos = h_rmeta_ + NB;
  int* h_slot = h_rmeta_ + 2 * NB;
  std::vector<PrefillSeg> segs;
  int rows = 0;
  // one packed chunk: tokens / positions / slots up, every layer over its rows, then the
  // logits row of each prompt that ends in it (sampled into that slot's state)
  auto flush = [&]() {
    if (!rows) return;
    HIPCHK(hipMemcpyAsync(tokens_, h_tok, sizeof(int) * rows, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(rpos_, h_pos, sizeof(int) * rows, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipMemcpyAsync(rslots_, h_slot, sizeof(int) * rows, hipMemcpyHostToDevice, stream_));
    segs_ = &segs;
    try {
      enqueue_prefill(rows, 0, stream_);
    } catch (...) {
      segs_ = nullptr;
      throw;
    }
    segs_ = nullptr;
    for (const PrefillSeg& g : segs)
      if (g.last) enqueue_head(x_ + (size_t)(g.row + g.n - 1) * d, 0, stream_, g.slot);
    HIPCHK(hipStreamSynchronize(stream_));  // the pinned row metadata is rewritten next
    segs.clear();
    rows = 0;
  };
  for (size_t i = 0; i < n; ++i) {
    const std::vector<int>& pr = prompts[i];
    int pos = n_keep[i];
    const int np = (int)pr.size();
    while (pos < np) {
      if (rows == NB) flush();
      const int take = std::min(NB - rows, np - pos);
      for (int j = 0; j < take; ++j) {
        h_tok[rows + j] = pr[pos + j];
        h_pos[rows + j] = pos + j;
        h_slot[rows + j] = slots[i];
      }
      segs.push_back({rows, take, slots[i], pos, pos + take == np});
      rows += take;
      pos += take;
    }
  }
  flush();
  std::vector<int> out(n);
  for (size_t i = 0; i < n; ++i)
    HIPCHK(hipMemcpy(&out[i], state_ + (size_t)S_NSTATE * slots[i] + S_TOKEN, sizeof(int), hipMemcpyDeviceToHost));
  check_device_err();
  return out;
}

void Engine::check_batch_rows(const std::vector<int>& slots) const {
  const int B = (int)slots.size();
  if (!bmax_) throw std::runtime_error("batch_step: the engine was built with one KV slot");
  if (B < 1 || B > bmax_) throw std::runtime_error("batch_step: 1 <= rows <= max_batch");
  for (int b = 0; b < B; ++b) {
    if (slots[b] < 0 || slots[b] >= opt_.n_slots) throw std::runtime_error("batch_step: slot out of range");
    for (int c = 0; c < b; ++c)
      if (slots[c] == slots[b]) throw std::runtime_error("batch_step: duplicate slot");
  }
}

// Pipelined steps under TP: rank 0 publishes every launch and collect, the followers replay them in
// the same order (their step k + 1 queued behind step k, the collectives pairing up as in
// synchronous steps); a follower's collect only waits for its own step.
void Engine::batch_launch(const std::vector<int>& slots) {
  ExecGuard guard(this);
  if (!can_pipeline()) throw std::runtime_error("batch_launch: not available on this engine");
  if (fl_n_ >= 2) throw std::runtime_error("batch_launch: two steps already in flight");
  check_batch_rows(slots);
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_BATCH_LAUNCH); m.put_vec(slots);
    mirror(m);
  }
  batch_launch_impl(slots);
}

void Engine::batch_launch_impl(const std::vector<int>& slots) {
  if (fl_n_ >= 2) throw std::runtime_error("batch_launch: two steps already in flight");
  const int B = (int)slots.size();
  // a changed row -> slot map is rewritten in pinned memory: no copy of it may still be queued
  const bool remap = B != bslots_n_ || std::memcmp(h_bslots_, slots.data(), sizeof(int) * B) != 0;
  if (remap && fl_n_ > 0) HIPCHK(hipStreamSynchronize(stream_));
  const int i = (fl_head_ + fl_n_) & 1;
  struct Par {  // the flight's graph instantiation, reset on every exit
    int& p;
    ~Par() { p = 0; }
  } par{launch_par_};
  launch_par_ = i;
  enqueue_batch_launch(slots, h_btok2_[i]);
  HIPCHK(hipEventRecord(bev_[i], stream_));
  fl_B_[i] = B;
  fl_b1_[i] = last_b1_;
  ++fl_n_;
}

std::vector<int> Engine::batch_collect() {
  ExecGuard guard(this);
  if (fl_n_ <= 0) throw std::runtime_error("batch_collect: no step in flight");
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_BATCH_COLLECT);
    mirror(m);
  }
  return batch_collect_impl();
}

std::vector<int> Engine::batch_collect_impl() {
  if (fl_n_ <= 0) throw std::runtime_error("batch_collect: no step in flight");
  const int i = fl_head_;
  fl_head_ ^= 1;
  --fl_n_;
  HIPCHK(hipEventSynchronize(bev_[i]));
  HIPCHK(hipGetLastError());
  check_device_err();
  last_batch_ = fl_B_[i];
  last_b1_ = fl_b1_[i];
  return std::vector<int>(h_btok2_[i], h_btok2_[i] + fl_B_[i]);
}

std::vector<int> Engine::batch_step(const std::vector<int>& slots) {
  ExecGuard guard(this);
  if (fl_n_ > 0) throw std::runtime_error("batch_step: pipelined steps in flight (batch_collect them first)");
  check_batch_rows(slots);
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_BATCH_STEP); m.put_vec(slots);
    mirror(m);
  }
  return batch_step_impl(slots);
}

std::vector<int> Engine::batch_step_impl(const std::vector<int>& slots) {
  const int B = (int)slots.size();
  // (launch_par_ is 0 outside a pipelined launch: graph instance 0, whose sampler writes h_btok2_[0])
  int* dst = h_btok2_[0] ? h_btok2_[0] : h_btok_;
  enqueue_batch_launch(slots, dst);
  HIPCHK(hipStreamSynchronize(stream_));
  HIPCHK(hipGetLastError());
  check_device_err();
  last_batch_ = B;
  return std::vector<int>(dst, dst + B);
}

// Queue one batch step of `slots` and the copy of its tokens to the pinned h_dst (no sync).
void Engine::enqueue_batch_launch(const std::vector<int>& slots, int* h_dst) {
  const int B = (int)slots.size();
  if (B == 1) {
    // one active row: the single-row GEMV decode of that slot beats the batched projections
    launch_step(slots[0]);
    HIPCHK(hipMemcpyAsync(h_dst, state_ + (size_t)S_NSTATE * slots[0] + S_TOKEN, sizeof(int),
                          hipMemcpyDeviceToHost, stream_));
    last_b1_ = true;
    return;
  }
  last_b1_ = false;
  // the row -> slot map goes up only when it changed (a steady batch re-sends nothing; each
  // step ends in a stream sync, so the pinned copy is never rewritten under an in-flight copy)
  if (B != bslots_n_ || std::memcmp(h_bslots_, slots.data(), sizeof(int) * B) != 0) {
    std::memcpy(h_bslots_, slots.data(), sizeof(int) * B);
    HIPCHK(hipMemcpyAsync(bslots_, h_bslots_, sizeof(int) * B, hipMemcpyHostToDevice, stream_));
    bslots_n_ = B;
  }
  if (opt_.use_graph) {
    if ((int)bgraph_.size() <= B) {
      bgraph_.resize(B + 1, nullptr);
      bgraph2_.resize(B + 1, nullptr);
    }
    if (!bgraph_[B]) {
      // one capture per flight parity: instance i's sampler stores the tokens straight into the
      // host-mapped h_btok2_[i] (no D2H copy node behind every step - 4 us of GPU time per step)
      for (int i = 0; i < 2; ++i) {
        hipGraph_t g = nullptr;
        sample_host_ = btok_dev_[i];
        HIPCHK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
        enqueue_batch_step(B, stream_);
        HIPCHK(hipStreamEndCapture(stream_, &g));
        sample_host_ = nullptr;
        const hipError_t e = hipGraphInstantiate(i ? &bgraph2_[B] : &bgraph_[B], g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        HIPCHK(e);
      }
    }
    HIPCHK(hipGraphLaunch(launch_par_ ? bgraph2_[B] : bgraph_[B], stream_));
    if (h_dst == h_btok2_[launch_par_ ? 1 : 0]) return;  // (the graph's sampler stored them there)
  } else {
    enqueue_batch_step(B, stream_);
  }
  HIPCHK(hipMemcpyAsync(h_dst, btok_out_, sizeof(int) * B, hipMemcpyDeviceToHost, stream_));
}

// Rows [0, B) of a logits buffer with row pitch ld_src holding this rank's vocabulary shard
// -> full rows [B][n_vocab] on the host (under TP: one all-gather of the shards).
void Engine::gather_logits_rows(int B, size_t ld_src, const float* src, std::vector<float>& out) {
  const int V = hp_.n_vocab, tp = opt_.tp_size;
  out.assign((size_t)B * V, 0.f);
  if (tp == 1) {
    HIPCHK(hipMemcpy2DAsync(out.data(), sizeof(float) * V, src, sizeof(float) * ld_src, sizeof(float) * V, B,
                            hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    return;
  }
  // pack the shard rows [B][V_l] contiguously, all-gather -> [tp][B][V_l]
  // persistent (grow-only) scratch: no device alloc / free churn between TP collectives
  const size_t need = (size_t)B * V_l_ * (1 + tp);
  if (gather_cap_ < need) {
    gather_buf_ = (float*)dalloc(sizeof(float) * need);
    gather_cap_ = need;
  }
  float* packed = gather_buf_;
  float* all = gather_buf_ + (size_t)B * V_l_;
  HIPCHK(hipMemcpy2DAsync(packed, sizeof(float) * V_l_, src, sizeof(float) * ld_src, sizeof(float) * V_l_, B,
                          hipMemcpyDeviceToDevice, stream_));
  allgather_into(packed, all, (size_t)B * V_l_, stream_);
  std::vector<float> h((size_t)B * V_l_ * tp);
  HIPCHK(hipMemcpyAsync(h.data(), all, sizeof(float) * h.size(), hipMemcpyDeviceToHost, stream_));
  HIPCHK(hipStreamSynchronize(stream_));
  for (int r = 0; r < tp; ++r) {
    const int n = std::max(0, std::min(V_l_, V - r * V_l_));
    for (int b = 0; b < B; ++b)
      std::memcpy(out.data() + (size_t)b * V + (size_t)r * V_l_, h.data() + ((size_t)r * B + b) * V_l_,
                  sizeof(float) * n);
  }
}

std::vector<float> Engine::batch_logits(int B) {
  ExecGuard guard(this);
  if (!bmax_ || B < 1 || B > last_batch_) throw std::runtime_error("batch_logits: no such rows in the last batch_step");
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_BATCH_LOGITS); m.put(B);
    mirror(m);
  }
  return batch_logits_impl(B);
}

std::vector<float> Engine::batch_logits_impl(int B) {
  std::vector<float> out;
  if (last_b1_) gather_logits_rows(1, V_l_, tp_on_ ? logits_l_ : logits_, out);
  else gather_logits_rows(B, V_pad_, logits_b_, out);
  return out;
}

GenOut Engine::generate(const std::vector<int>& prompt, int n_keep, int max_new, const SamplingOpts& sp,
                        const std::vector<int>& stop_ids, const std::function<bool()>& poll,
                        const std::function<void(int)>& on_token) {
  if (!has_head()) throw std::runtime_error("generate: this layer-split stage holds no head (eval_stage)");
  ExecGuard guard(this);
  GenOut out;
  const int n_prompt = (int)prompt.size();
  if (n_prompt == 0) throw std::runtime_error("empty prompt");
  if (n_prompt >= opt_.n_ctx) throw std::runtime_error("prompt exceeds context window");
  (void)make_sparams(sp);
  if (n_keep < 0 || n_keep >= n_prompt) n_keep = 0;
  const double t0 = now_s();

  // per-request device state: sampling params, penalty ring (prompt tail), counters
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_SLOT_STATE); m.put<int>(0); m.put_vec(prompt); put_sp(m, sp);
    mirror(m);
  }
  begin_slot_state(0, prompt, sp);

  // prefill in n_batch chunks
  int pos = n_keep;
  {
    RoctxRange prefill_range("lfk.prefill");
    while (pos < n_prompt) {
      const int T = std::min(opt_.n_batch, n_prompt - pos);
      const bool head = pos + T == n_prompt;
      if (leader()) {
        TPMsg m;
        m.put<int32_t>(TPO_PREFILL); m.put<int>(0); m.put(pos); m.put<int>(head ? 1 : 0);
        m.put_vec(std::vector<int>(prompt.begin() + pos, prompt.begin() + pos + T));
        mirror(m);
      }
      prefill_chunk(0, prompt.data() + pos, T, pos, head);
      pos += T;
    }
  }
  HIPCHK(hipGetLastError());
  const double t1 = now_s();
  out.prefill_s = t1 - t0;
  out.n_prefilled = n_prompt - n_keep;

  auto is_stop = [&](int t) {
    for (int s : stop_ids) if (s == t) return true;
    return false;
  };
  // one decode step: the followers replay exactly the steps rank 0 launches, so a stop
  // token, a cancel or max_new on rank 0 ends every rank at the same step
  auto step = [&](int k) {
    if (leader()) {
      TPMsg m;
      m.put<int32_t>(TPO_DECODE_STEP);
      mirror(m);
    }
    launch_step();
    HIPCHK(hipEventRecord(step_ev_[k % kDepth], stream_));
  };
  RoctxRange decode_range("lfk.decode");
  int tok = h_ring_[0];
  out.tokens.push_back(tok);
  if (on_token) on_token(tok);
  out.finish = "length";
  const int max_steps = std::min(max_new - 1, opt_.n_ctx - n_prompt);
  if (is_stop(tok)) {
    out.finish = "stop";
  } else if (max_steps > 0) {
    int launched = 0;
    while (launched < std::min(kDepth, max_steps)) step(launched++);
    for (int i = 1; i <= max_steps; ++i) {
      HIPCHK(hipEventSynchronize(step_ev_[(i - 1) % kDepth]));
      tok = h_ring_[i & 63];
      out.tokens.push_back(tok);
      if (on_token) on_token(tok);
      if (is_stop(tok)) { out.finish = "stop"; break; }
      if (poll && (i & 3) == 0 && poll()) { out.finish = "cancelled"; break; }
      if (launched < max_steps) step(launched++);
    }
    HIPCHK(hipStreamSynchronize(stream_));
  }
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_SYNC);
    mirror(m);
  }
  HIPCHK(hipGetLastError());
  out.decode_s = now_s() - t1;
  check_device_err();
  out.n_evaluated = n_prompt + (int)out.tokens.size() - 1;
  return out;
}

// ------------------------------------------------------------------ layer-split chain
void Engine::enqueue_stage_decode(hipStream_t s) {
  int* st = state_ + (size_t)S_NSTATE * dslot_;
  // the attention -> Wo done counters: zeroed by the embedding's side job on the first stage, by
  // a memset node elsewhere
  if (tok_embd_.base) embed_rows(tok_embd_, st + S_TOKEN, 1, x_, s, dec_done_, 64 * hp_.n_layer);
  else if (dec_done_) HIPCHK(hipMemsetAsync(dec_done_, 0, sizeof(int) * 64 * hp_.n_layer, s));
  for (int l = opt_.layer_begin; l < layer_end_; ++l) enqueue_layer_decode(l, s);
  if (has_head()) enqueue_head(x_, 1, s, dslot_);
}

// one decode step of this stage: after `prev`'s step (or, on the first stage, after the last
// stage's state copy-back of the previous step), take prev's hidden row, run the stage graph;
// the last stage then copies its token / position state to every other stage
void Engine::chain_step(const Engine* prev, const Engine* last, const std::vector<Engine*>& others) {
  HIPCHK(hipSetDevice(opt_.device));
  const Engine* after = prev ? prev : last;
  HIPCHK(hipStreamWaitEvent(stream_, after->chain_ev_, 0));
  if (prev)
    HIPCHK(hipMemcpyPeerAsync(x_, opt_.device, prev->x_, prev->opt_.device, sizeof(float) * hp_.n_embd, stream_));
  if (!chain_graph_[0]) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    enqueue_stage_decode(stream_);
    HIPCHK(hipStreamEndCapture(stream_, &g));
    hipError_t e = hipGraphInstantiate(&chain_graph_[0], g, nullptr, nullptr, 0);
    if (e == hipSuccess) e = hipGraphInstantiate(&chain_graph_[1], g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    HIPCHK(e);
  }
  HIPCHK(hipGraphLaunch(chain_graph_[chain_par_], stream_));
  chain_par_ ^= 1;
  if (this == last)
    for (const Engine* o : others)
      HIPCHK(hipMemcpyPeerAsync(o->state_, o->opt_.device, state_, opt_.device, sizeof(int) * S_NSTATE, stream_));
  HIPCHK(hipEventRecord(chain_ev_, stream_));
}

GenOut Engine::chain_generate(const std::vector<Engine*>& st, const std::vector<int>& prompt, int n_keep,
                              int max_new, const SamplingOpts& sp, const std::vector<int>& stop_ids,
                              const std::function<bool()>& poll, const std::function<void(int)>& on_token) {
  const size_t n = st.size();
  if (n == 0) throw std::runtime_error("chain_generate: no stages");
  for (size_t i = 0; i < n; ++i) {
    const Engine* e = st[i];
    if (!e || e->tp_on_ || e->opt_.tp_size > 1) throw std::runtime_error("chain_generate: stages are single-rank engines");
    if (e->hp_.n_embd != st[0]->hp_.n_embd || e->opt_.n_ctx != st[0]->opt_.n_ctx)
      throw std::runtime_error("chain_generate: stages of one model and context");
    if ((i == 0 && e->opt_.layer_begin != 0) || (i > 0 && e->opt_.layer_begin != st[i - 1]->layer_end_))
      throw std::runtime_error("chain_generate: stages must cover the layers in order");
    for (size_t j = 0; j < i; ++j)
      if (st[j] == e) throw std::runtime_error("chain_generate: a stage listed twice");
  }
  Engine* last = st[n - 1];
#define CHAIN_CHK(x) last->check((x), #x)
  if (!last->has_head()) throw std::runtime_error("chain_generate: the last stage must hold the head");
  std::vector<std::unique_lock<std::mutex>> locks;  // every stage's guard, in chain order
  for (Engine* e : st) locks.emplace_back(e->exec_mu_);
  std::vector<Engine*> others(st.begin(), st.end() - 1);
  GenOut out;
  const int n_prompt = (int)prompt.size();
  if (n_prompt == 0) throw std::runtime_error("empty prompt");
  if (n_prompt >= last->opt_.n_ctx) throw std::runtime_error("prompt exceeds context window");
  (void)last->make_sparams(sp);
  if (n_keep < 0 || n_keep >= n_prompt) n_keep = 0;
  const double t0 = now_s();
  for (Engine* e : st) {
    CHAIN_CHK(hipSetDevice(e->opt_.device));
    if (!e->chain_ev_) CHAIN_CHK(hipEventCreateWithFlags(&e->chain_ev_, hipEventDisableTiming));
    e->begin_slot_state(0, prompt, sp);  // position / token on every stage, sampler state on the last
  }
  // prompt chunks: stage 0 embeds, every later stage takes the chunk's hidden rows peer to peer
  const int NB = std::min(st[0]->opt_.n_batch, last->opt_.n_batch);
  for (int pos = n_keep; pos < n_prompt;) {
    const int T = std::min(NB, n_prompt - pos);
    for (size_t i = 0; i < n; ++i) {
      Engine* e = st[i];
      if (T > e->opt_.n_batch) throw std::runtime_error("chain_generate: chunk exceeds a stage's n_batch");
      CHAIN_CHK(hipSetDevice(e->opt_.device));
      if (i == 0) {
        std::memcpy(e->h_tokens_, prompt.data() + pos, sizeof(int) * T);
        CHAIN_CHK(hipMemcpyAsync(e->tokens_, e->h_tokens_, sizeof(int) * T, hipMemcpyHostToDevice, e->stream_));
      } else {
        CHAIN_CHK(hipStreamWaitEvent(e->stream_, st[i - 1]->chain_ev_, 0));
        CHAIN_CHK(hipMemcpyPeerAsync(e->x_, e->opt_.device, st[i - 1]->x_, st[i - 1]->opt_.device,
                                  sizeof(float) * T * e->hp_.n_embd, e->stream_));
      }
      e->enqueue_prefill(T, pos, e->stream_, /*embed=*/i == 0);
      if (e == last && pos + T == n_prompt) e->enqueue_head(e->x_ + (size_t)(T - 1) * e->hp_.n_embd, 0, e->stream_, 0);
      CHAIN_CHK(hipEventRecord(e->chain_ev_, e->stream_));
    }
    CHAIN_CHK(hipSetDevice(st[0]->opt_.device));
    CHAIN_CHK(hipStreamSynchronize(st[0]->stream_));  // h_tokens_ is reused by the next chunk
    pos += T;
  }
  // the first token's state to every stage
  CHAIN_CHK(hipSetDevice(last->opt_.device));
  for (const Engine* o : others)
    CHAIN_CHK(hipMemcpyPeerAsync(o->state_, o->opt_.device, last->state_, last->opt_.device, sizeof(int) * S_NSTATE,
                              last->stream_));
  CHAIN_CHK(hipEventRecord(last->chain_ev_, last->stream_));
  CHAIN_CHK(hipStreamSynchronize(last->stream_));
  const double t1 = now_s();
  out.prefill_s = t1 - t0;
  out.n_prefilled = n_prompt - n_keep;
  auto is_stop = [&](int t) {
    for (int s : stop_ids) if (s == t) return true;
    return false;
  };
  auto step = [&](int k) {
    for (size_t i = 0; i < n; ++i) st[i]->chain_step(i ? st[i - 1] : nullptr, last, others);
    CHAIN_CHK(hipSetDevice(last->opt_.device));
    CHAIN_CHK(hipEventRecord(last->step_ev_[k % kDepth], last->stream_));
  };
  int tok = last->h_ring_[0];
  out.tokens.push_back(tok);
  if (on_token) on_token(tok);
  out.finish = "length";
  const int max_steps = std::min(max_new - 1, last->opt_.n_ctx - n_prompt);
  if (is_stop(tok)) {
    out.finish = "stop";
  } else if (max_steps > 0) {
    int launched = 0;
    while (launched < std::min(kDepth, max_steps)) step(launched++);
    for (int i = 1; i <= max_steps; ++i) {
      CHAIN_CHK(hipEventSynchronize(last->step_ev_[(i - 1) % kDepth]));
      tok = last->h_ring_[i & 63];
      out.tokens.push_back(tok);
      if (on_token) on_token(tok);
      if (is_stop(tok)) { out.finish = "stop"; break; }
      if (poll && (i & 3) == 0 && poll()) { out.finish = "cancelled"; break; }
      if (launched < max_steps) step(launched++);
    }
  }
  for (Engine* e : st) {
    CHAIN_CHK(hipSetDevice(e->opt_.device));
    CHAIN_CHK(hipStreamSynchronize(e->stream_));
    CHAIN_CHK(hipGetLastError());
  }
  out.decode_s = now_s() - t1;
  for (Engine* e : st) e->check_device_err();
  out.n_evaluated = n_prompt + (int)out.tokens.size() - 1;
  return out;
}
#undef CHAIN_CHK

std::vector<float> Engine::eval_logits(const std::vector<int>& tokens, int pos0) {
  if (!has_head()) throw std::runtime_error("eval_logits: this layer-split stage holds no head (eval_stage)");
  ExecGuard guard(this);
  const int T = (int)tokens.size();
  if (T <= 0 || T > opt_.n_batch || pos0 < 0 || pos0 + T > opt_.n_ctx) throw std::runtime_error("eval_logits: bad size");
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_EVAL_LOGITS); m.put(pos0); m.put_vec(tokens);
    mirror(m);
  }
  return eval_logits_impl(tokens, pos0);
}

std::vector<float> Engine::eval_logits_impl(const std::vector<int>& tokens, int pos0) {
  const int T = (int)tokens.size();
  SamplerParamsDev p;
  p.greedy = 1; p.top_k = 1; p.repeat_penalty = 1.f;
  int hstate[S_NSTATE] = {0};
  hstate[S_POS] = pos0 + T;
  HIPCHK(hipMemcpyAsync(sparams_, &p, sizeof(p), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemcpyAsync(state_, hstate, sizeof(hstate), hipMemcpyHostToDevice, stream_));
  std::memcpy(h_tokens_, tokens.data(), sizeof(int) * T);
  HIPCHK(hipMemcpyAsync(tokens_, h_tokens_, sizeof(int) * T, hipMemcpyHostToDevice, stream_));
  enqueue_prefill(T, pos0, stream_);
  enqueue_head(x_ + (size_t)(T - 1) * hp_.n_embd, 0, stream_);
  std::vector<float> out;
  gather_logits_rows(1, V_l_, tp_on_ ? logits_l_ : logits_, out);
  return out;
}

std::vector<float> Engine::eval_hidden(const float* x, int T, int pos0) {
  ExecGuard guard(this);
  if (tp_on_) throw std::runtime_error("eval_hidden: not available with tensor parallelism");
  if (T <= 0 || T > opt_.n_batch || pos0 + T > opt_.n_ctx) throw std::runtime_error("eval_hidden: bad size");
  HIPCHK(hipMemcpyAsync(x_, x, sizeof(float) * T * hp_.n_embd, hipMemcpyHostToDevice, stream_));
  enqueue_prefill(T, pos0, stream_, /*embed=*/false);
  enqueue_head(x_ + (size_t)(T - 1) * hp_.n_embd, 0, stream_);
  std::vector<float> out(hp_.n_vocab);
  HIPCHK(hipMemcpyAsync(out.data(), logits_, sizeof(float) * hp_.n_vocab, hipMemcpyDeviceToHost, stream_));
  HIPCHK(hipStreamSynchronize(stream_));
  return out;
}

std::vector<float> Engine::eval_stage(const float* x, const int* tokens, int T, int pos0, bool to_host) {
  if (has_head()) {
    if (x) return eval_hidden(x, T, pos0);
    return eval_logits(std::vector<int>(tokens, tokens + T), pos0);
  }
  ExecGuard guard(this);
  if (tp_on_) throw std::runtime_error("eval_stage: not available with tensor parallelism");
  if (T <= 0 || T > opt_.n_batch || pos0 < 0 || pos0 + T > opt_.n_ctx) throw std::runtime_error("eval_stage: bad size");
  if (x) {
    HIPCHK(hipMemcpyAsync(x_, x, sizeof(float) * T * hp_.n_embd, hipMemcpyHostToDevice, stream_));
  } else {
    if (opt_.layer_begin > 0) throw std::runtime_error("eval_stage: token input needs the first stage");
    for (int i = 0; i < T; ++i)
      if (tokens[i] < 0 || tokens[i] >= hp_.n_vocab) throw std::runtime_error("eval_stage: token out of range");
    std::memcpy(h_tokens_, tokens, sizeof(int) * T);
    HIPCHK(hipMemcpyAsync(tokens_, h_tokens_, sizeof(int) * T, hipMemcpyHostToDevice, stream_));
  }
  enqueue_prefill(T, pos0, stream_, /*embed=*/x == nullptr);
  std::vector<float> out(to_host ? (size_t)T * hp_.n_embd : 0);  // (else the next stage copies x_ peer to peer)
  if (to_host) HIPCHK(hipMemcpyAsync(out.data(), x_, sizeof(float) * out.size(), hipMemcpyDeviceToHost, stream_));
  HIPCHK(hipStreamSynchronize(stream_));
  return out;
}

std::vector<float> Engine::eval_stage_peer(const Engine& prev, int T, int pos0) {
  ExecGuard guard(this);
  if (tp_on_) throw std::runtime_error("eval_stage_peer: not available with tensor parallelism");
  if (prev.hp_.n_embd != hp_.n_embd || prev.layer_end_ != opt_.layer_begin)
    throw std::runtime_error("eval_stage_peer: prev must be the stage that ends where this one begins");
  if (T <= 0 || T > opt_.n_batch || T > prev.opt_.n_batch || pos0 < 0 || pos0 + T > opt_.n_ctx)
    throw std::runtime_error("eval_stage_peer: bad size");
  // (prev's eval synchronised its stream before returning: its x_ rows are final)
  HIPCHK(hipMemcpyPeerAsync(x_, opt_.device, prev.x_, prev.opt_.device, sizeof(float) * T * hp_.n_embd, stream_));
  enqueue_prefill(T, pos0, stream_, /*embed=*/false);
  std::vector<float> out;
  if (has_head()) {
    enqueue_head(x_ + (size_t)(T - 1) * hp_.n_embd, 0, stream_);
    out.resize(hp_.n_vocab);
    HIPCHK(hipMemcpyAsync(out.data(), logits_, sizeof(float) * hp_.n_vocab, hipMemcpyDeviceToHost, stream_));
  }
  HIPCHK(hipStreamSynchronize(stream_));
  return out;
}

void Engine::kv_transfer(void* buf, int n, bool load) {
  ExecGuard guard(this);
  if (tp_on_)
    throw std::runtime_error("KV snapshots hold one rank's heads: not available with tensor parallelism");
  if (n < 0 || n > opt_.n_ctx) throw std::runtime_error("kv_transfer: n out of range");
  if (n == 0) return;
  const size_t row = (size_t)n * hp_.head_dim * 2, pitch = (size_t)opt_.n_ctx * hp_.head_dim * 2;
  const size_t rows = (size_t)(layer_end_ - opt_.layer_begin) * nkv_l_;
  char* b = static_cast<char*>(buf);
  for (int which = 0; which < 2; ++which) {
    char* cache = reinterpret_cast<char*>(which == 0 ? kc_ : vc_);
    char* packed = b + which * rows * row;
    if (load)
      HIPCHK(hipMemcpy2DAsync(cache, pitch, packed, row, row, rows, hipMemcpyDefault, stream_));
    else
      HIPCHK(hipMemcpy2DAsync(packed, row, cache, pitch, row, rows, hipMemcpyDefault, stream_));
  }
  HIPCHK(hipStreamSynchronize(stream_));
}

std::vector<float> Engine::decode_logits(int token, int pos) {
  if (!has_head()) throw std::runtime_error("decode_logits: this layer-split stage holds no head (eval_stage)");
  ExecGuard guard(this);
  if (pos < 0 || pos >= opt_.n_ctx) throw std::runtime_error("decode_logits: pos out of range");
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_DECODE_LOGITS); m.put(token); m.put(pos);
    mirror(m);
  }
  return decode_logits_impl(token, pos);
}

std::vector<float> Engine::decode_logits_impl(int token, int pos) {
  SamplerParamsDev p;
  p.greedy = 1; p.top_k = 1; p.repeat_penalty = 1.f;
  int hstate[S_NSTATE] = {0};
  hstate[S_TOKEN] = token;
  hstate[S_POS] = pos;
  HIPCHK(hipMemcpyAsync(sparams_, &p, sizeof(p), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemcpyAsync(state_, hstate, sizeof(hstate), hipMemcpyHostToDevice, stream_));
  launch_step();
  std::vector<float> out;
  gather_logits_rows(1, V_l_, tp_on_ ? logits_l_ : logits_, out);
  check_device_err();
  return out;
}

void Engine::bench_decode(int n_steps, int pos0, double* ms_per_step) {
  ExecGuard guard(this);
  if (n_steps < 1 || pos0 < 0 || pos0 + n_steps + 1 > opt_.n_ctx) throw std::runtime_error("bench_decode: exceeds n_ctx");
  if (leader()) {
    TPMsg m;
    m.put<int32_t>(TPO_BENCH_DECODE); m.put(n_steps); m.put(pos0);
    mirror(m);
  }
  *ms_per_step = bench_decode_impl(n_steps, pos0);
}

double Engine::bench_decode_impl(int n_steps, int pos0) {
  SamplerParamsDev p;
  p.greedy = 1; p.top_k = 1;
  int hstate[S_NSTATE] = {0};
  hstate[S_TOKEN] = 1;
  hstate[S_POS] = pos0;
  HIPCHK(hipMemcpyAsync(sparams_, &p, sizeof(p), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemcpyAsync(state_, hstate, sizeof(hstate), hipMemcpyHostToDevice, stream_));
  launch_step();  // warm (captures the graph on first use)
  HIPCHK(hipStreamSynchronize(stream_));
  const double t0 = now_s();
  for (int i = 0; i < n_steps; ++i) launch_step();
  HIPCHK(hipStreamSynchronize(stream_));
  const double ms = (now_s() - t0) * 1e3 / n_steps;
  check_device_err();
  return ms;
}

}  // namespace lfk
