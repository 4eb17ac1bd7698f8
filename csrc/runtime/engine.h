// MI355X inference engine: owns the device weights, KV cache,
// workspaces and RCCL communicator of ONE rank, and runs prefill / decode /
// sampling as a fixed kernel schedule (no graph IR, no allocator at run time).
//
// One process drives one GPU. Tensor parallelism (split_mode=row, the
// `tensor_split` path of the reference) shards heads and FFN
// features across ranks; each rank runs the same schedule with two RCCL
// all-reduces per layer and one all-gather of vocabulary-sharded logits.
// The decode step (embedding -> layers -> lm_head -> sampler -> token D2H) is
// captured once into a hipGraph and replayed per token.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../kernels/kernels.h"
#include "gguf.h"
#include "p2p.h"
#include "slots.h"
#include "tp_channel.h"

namespace lfk {

struct HParams {
  int n_vocab = 0, n_embd = 0, n_layer = 0, n_head = 0, n_head_kv = 0, head_dim = 0, n_ff = 0;
  int n_expert = 0, n_expert_used = 0, n_ctx_train = 0;
  float rope_base = 10000.f, rms_eps = 1e-5f;
};
HParams read_hparams(const GGUFFile& f);

struct EngineOptions {
  int n_ctx = 1024;
  int n_batch = 512;
  int device = 0;
  bool use_graph = true;
  int tp_rank = 0;
  int tp_size = 1;
  std::string nccl_id;  // ncclUniqueId bytes (tp_size > 1, comm != "ipc")
  // tensor-parallel collectives: "auto" = one-shot P2P kernel for decode-sized messages +
  // RCCL for the rest; "ipc" = P2P for every message, no RCCL (ranks may share a GPU - the
  // one-GPU test box); "rccl" = RCCL only
  std::string comm = "auto";
  std::vector<float> tensor_split;  // per-rank weights (empty = even); see shard.h
  int layer_begin = 0;  // hybrid placement: layers [0, layer_begin) run on the CPU backend
  int layer_end = -1;   // layer split: this engine runs layers [layer_begin, layer_end) (-1: n_layer);
                        // the output norm and head are loaded only by the stage ending at n_layer
  // KV slots (continuous batching): slot 0 serves generate() / the graph decode path, slots
  // [0, n_slots) can decode together through batch_step() (also under tensor parallelism)
  int n_slots = 1;
  bool verbose = false;
  // fault-injection test hook, "<rank>:<n>[:dev|:shard]" (empty in production; set only by the tests
  // through the Python backend's explicit opt-in, runtime/hip_backend.py): follower <rank> fails its
  // n-th command (host failure, or ":dev" a device-side fault word), or ":shard" (n = 0) loads the
  // NEXT shard's FFN features - a deliberately wrong shard the TP acceptance must catch
  std::string test_fault;
};


struct GenOut {
  std::vector<int> tokens;
  std::string finish;
  int n_evaluated = 0;
  int n_prefilled = 0;
  double prefill_s = 0, decode_s = 0;
};

struct Layer {
  float* attn_norm = nullptr;
  float* ffn_norm = nullptr;
  QMat wq, wk, wv, wo;
  QMat w_gu, w_down;                 // dense FFN (gate/up interleaved in 32-row groups)
  QMat router, gu_exps, down_exps;   // MoE
  // batched decode (bmm.hip): tile16 copies of the projections (base = the copy)
  QMat t_wq, t_wk, t_wv, t_wo, t_gu, t_down;
};

class Engine : public SlotBackend {
 public:
  Engine(const std::string& path, const EngineOptions& opts);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  GenOut generate(const std::vector<int>& prompt, int n_keep, int max_new, const SamplingOpts& sp,
                  const std::vector<int>& stop_ids, const std::function<bool()>& poll,
                  const std::function<void(int)>& on_token);
  // test hooks (numerics vs the reference model)
  std::vector<float> eval_logits(const std::vector<int>& tokens, int pos0);  // prefill path
  std::vector<float> decode_logits(int token, int pos);                      // decode path (eager)
  // KV state of positions [0, n) for save/load_state and prompt caches: `buf` holds
  // [K|V][n_layer][nkv_l][n][hd] f16, in host OR device memory (one strided copy each way;
  // a device-resident snapshot is an HBM-to-HBM copy)
  // per-block timeline of one layer of the batch step (LFK_STEP_CLK=<layer>, tools/step_blocks.py):
  // [5 kernels: Q|K|V, attention, Wo, gate/up, down][kStepClkBlocks][16] wall_clock64 stamps
  static constexpr int kStepClkBlocks = 8192;
  std::vector<long long> step_clk();
  void step_clk_zero();
  size_t kv_state_bytes(int n) const { return 2ull * (layer_end_ - opt_.layer_begin) * nkv_l_ * (size_t)n * hp_.head_dim * 2; }
  void kv_transfer(void* buf, int n, bool load);
  // hybrid placement: hidden states [T][d] of layer `layer_begin` in, last-row logits out
  std::vector<float> eval_hidden(const float* x, int T, int pos0);
  // layer split (runtime/layer_split_backend.py): tokens (x == nullptr, first stage) or hidden
  // states [T][d] in; the hidden states after layer_end - 1 out ([T][d]), or the last row's logits
  // when this stage holds the head
  std::vector<float> eval_stage(const float* x, const int* tokens, int T, int pos0, bool to_host = true);
  // the same, with the hidden states taken device to device from the previous stage's engine
  // (its last eval_stage / eval_stage_peer output, T rows; hipMemcpyPeerAsync across GPUs): no
  // host round trip between stages. Returns the last row's logits at the head stage, else nothing
  std::vector<float> eval_stage_peer(const Engine& prev, int T, int pos0);
  void bench_decode(int n_steps, int pos0, double* ms_per_step);             // raw decode timing
  // layer split, whole generation natively (runtime/layer_split_backend.py): `stages` hold
  // contiguous layer ranges (stage 0 the embedding, the last the head), each on its own device.
  // Prompt chunks and decode steps hand the hidden states stage to stage device to device; each
  // stage's decode step is ONE captured hipGraph; the last stage samples on the device (the
  // engine's sampler: same chain, same uniforms as generate) and its token / position state is
  // copied back to every stage, so the host only reads tokens - kDepth steps in flight, as in
  // generate. Cross-stage order by events, never a host wait.
  static GenOut chain_generate(const std::vector<Engine*>& stages, const std::vector<int>& prompt, int n_keep,
                               int max_new, const SamplingOpts& sp, const std::vector<int>& stop_ids,
                               const std::function<bool()>& poll, const std::function<void(int)>& on_token);

  const HParams& hparams() const { return hp_; }
  size_t device_bytes() const { return dev_bytes_; }
  int tp_rank() const { return opt_.tp_rank; }
  int tp_size() const { return opt_.tp_size; }
  // tensor parallelism: one-shot P2P all-reduce for decode-sized messages (p2p.h);
  // the caller exchanges every rank's handle, then opens them (before the first decode)
  std::string p2p_handle();
  void p2p_open(const std::vector<std::string>& handles);
  bool p2p_ready() const { return p2p_ && p2p_->ready(); }
  // which path each tensor-parallel message takes, and the communicator as RCCL reports it
  // (bench.py's TP pass records it): key -> value strings
  std::vector<std::pair<std::string, std::string>> comm_info() const;
  // tensor parallelism: the host control channel (tp_channel.h). Rank 0 creates it, the
  // followers attach and then sit in follow() replaying rank 0's commands until tp_stop().
  void tp_ctl_create(const std::string& name);
  void tp_ctl_attach(const std::string& name);
  void follow();
  void tp_stop();
  bool tp_ctl_open() const { return tp_ctl_ != nullptr; }
  // (a TP leader also reports its followers' published failures and exits: TPChannel::fault_report)
  bool healthy() const { return healthy_ && group_fault().empty(); }
  std::string last_error() const { return healthy_ ? group_fault() : last_error_; }
  int n_ctx() const override { return opt_.n_ctx; }
  int layer_begin() const { return opt_.layer_begin; }
  int layer_end() const { return layer_end_; }
  bool has_head() const { return layer_end_ == hp_.n_layer; }
  int device() const { return opt_.device; }

  // ---- continuous batching over KV slots (EngineOptions::n_slots > 1, one rank, all layers)
  int n_slots() const override { return opt_.n_slots; }
  int max_batch() const override { return bmax_; }
  // 0: batch_step on the prefill GEMM; 1: attention/head on the batched GEMV; 2: every projection
  int batch_gemv() const { return bg_ffn_ ? 2 : bg_ ? 1 : 0; }
  // prompt chunks run on the tile16 copies (gemm_t16, f16 activations) instead of gemm_dq
  bool prefill_t16() const { return prefill_t16_; }
  // Prefill prompt[n_keep:] into `slot` (positions [0, n_keep) of the slot are reused),
  // set the slot's sampling state and sample its first token (synchronous).
  int slot_begin(int slot, const std::vector<int>& prompt, int n_keep, const SamplingOpts& sp) override;
  // chunked admission (scheduler): parts of 1024 tokens between decode steps of the other rows;
  // single-GPU engines (under TP admission stays whole). Parts of 256 hurt the 6-client bench
  // (decode 438 -> 418 tok/s per request, p50 1.51 -> 1.57 s): its ~390-token prompts arriving
  // a few ms apart lost the joint admission (one weight pass for all of them) to 2-part
  // admissions each; 1024-token parts leave prompts below that whole and bound the stall a
  // long-context prompt imposes on the decoding rows to ~20 ms per part (8B).
  int prefill_part_tokens() const override { return bmax_ > 0 && !tp_on_ ? 1024 : 0; }
  int slot_begin_part(int slot, const std::vector<int>& prompt, int n_keep, int n_done, int n,
                      const SamplingOpts& sp) override;
  // Admission of several requests in ONE prefill: the prompts' rows are packed into shared
  // chunks of up to n_batch rows (per-row KV slot / position for RoPE and the KV append,
  // one attention launch per prompt piece), so every weight is streamed once per chunk for
  // all of them instead of once per prompt; returns each slot's first token.
  std::vector<int> slots_begin(const std::vector<int>& slots, const std::vector<std::vector<int>>& prompts,
                               const std::vector<int>& n_keep, const std::vector<SamplingOpts>& sps) override;
  // One decode step of every listed slot, each at its own position: embeds each slot's
  // current token, runs all layers over the B rows (MFMA GEMMs, per-row RoPE/KV append,
  // batched split-L attention), the lm_head GEMM and the batched sampler; returns the
  // next token of each slot (synchronous).
  std::vector<int> batch_step(const std::vector<int>& slots) override;
  // Pipelined batch_step (the scheduler's decode loop, slots.h): without it the host turnaround
  // between steps - stream-sync wake-up, token hand-off, graph launch - left the GPU idle
  // ~60-80 us per 2.3 ms step. Under TP rank 0 publishes each launch and collect and the
  // followers replay them in order (their steps queue the same way).
  bool can_pipeline() const override { return bmax_ > 0; }
  void batch_launch(const std::vector<int>& slots) override;
  std::vector<int> batch_collect() override;
  std::vector<float> batch_logits(int B);  // test hook: logits [B][n_vocab] of the last batch_step

 private:
  // Every public entry point that runs device work takes this guard: it serialises the
  // callers (the batch scheduler's thread and request threads of the legacy path) and makes
  // the engine's device current on the calling thread - HIP's current device is per thread,
  // and the threads that call in are not the one that built the engine (one process per GPU
  // runs on device LOCAL_RANK, not 0).
  struct ExecGuard {
    std::lock_guard<std::mutex> lk;
    explicit ExecGuard(Engine* e) : lk(e->exec_mu_) { (void)hipSetDevice(e->opt_.device); }
  };
  std::mutex exec_mu_;

  void* dalloc(size_t bytes);
  // model load: two pinned staging buffers alternate - the host repacks tensor i + 1 into one
  // while the DMA engine copies tensor i out of the other (upload_stream_)
  struct Staging {
    uint8_t* buf[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
    hipEvent_t done[2] = {nullptr, nullptr};
    int cur = 0;
  } stage_;
  hipStream_t upload_stream_ = nullptr;
  uint8_t* stage_acquire(size_t bytes);          // the free buffer, >= bytes
  void stage_commit(void* dev, size_t bytes);    // async copy of it to dev; flips buffers
  void stage_release();                          // waits for the copies, frees the buffers
  QMat upload_matrix(const GGUFFile& f, const std::string& name, size_t r0, size_t R, size_t c0, size_t K,
                     int n_expert = 0);
  QMat upload_gate_up(const GGUFFile& f, const std::string& gate, const std::string& up, size_t f0, size_t F,
                      int n_expert = 0);
  float* upload_f32(const GGUFFile& f, const std::string& name);
  void load(const GGUFFile& f);
  void alloc_buffers();
  void build_rope();

  void allreduce_into(const float* send, float* recv, size_t n, hipStream_t s);
  bool tp_epilogue(GemvArgs& g) const;
  void allgather_into(const float* send, float* recv, size_t n, hipStream_t s);  // recv [tp][n]
  // the sampler over this rank's logits rows (vocabulary shard under TP): stage 1, the
  // candidate all-gather, stage 2 (single row: slot; batched: the bslots_ rows)
  void enqueue_sample(const float* logits, int rows, size_t ld, int slot, int advance_pos, hipStream_t s);
  void gather_logits_rows(int B, size_t ld_src, const float* src, std::vector<float>& out);
  // tensor parallelism: publish a command to the followers (rank 0); no-op on one rank
  bool leader() const { return opt_.tp_size > 1 && opt_.tp_rank == 0; }
  std::string group_fault() const;  // leader: the followers' failures as the channel holds them ("" = none)
  bool tp_epi_ = true;
  bool pieces_attn_ = true;  // a joint admission's prompt pieces in one attention launch
  // rows of the activation buffers: n_batch, or kJointRows for a joint admission (alloc_buffers)
  static constexpr int kJointRows = 4096;
  int nb_cap_ = 0;              // GEMV-epilogue all-reduce allowed (LFK_TP_EPILOGUE=0: the collective kernel)
  int fault_after_ = 0;             // follower test hook (EngineOptions::test_fault): fail the n-th command
  bool fault_dev_ = false;          // ... as a device-side fault word instead of a host failure
  void mirror(const TPMsg& m);
  void prefill_chunk(int slot, const int* toks, int T, int pos, bool head);
  int slot_begin_impl(int slot, const std::vector<int>& prompt, int n_keep, const SamplingOpts& sp);
  std::vector<int> slots_begin_impl(const std::vector<int>& slots, const std::vector<std::vector<int>>& prompts,
                                    const std::vector<int>& n_keep, const std::vector<SamplingOpts>& sps);
  // a piece of one prompt inside a packed prefill chunk: rows [row, row + n) at positions
  // pos.. of KV slot `slot`; `last` = the prompt ends here (its logits row is sampled)
  struct PrefillSeg {
    int row, n, slot, pos;
    bool last;
  };
  const std::vector<PrefillSeg>* segs_ = nullptr;  // set while a packed chunk is enqueued
  int* rpos_ = nullptr;     // [n_batch] per-row position of a packed chunk
  int* rslots_ = nullptr;   // [n_batch] per-row KV slot
  int* h_rmeta_ = nullptr;  // pinned [3][n_batch]: tokens | positions | slots
  std::vector<int> batch_step_impl(const std::vector<int>& slots);
  std::vector<float> eval_logits_impl(const std::vector<int>& tokens, int pos0);
  std::vector<float> decode_logits_impl(int token, int pos);
  std::vector<float> batch_logits_impl(int B);
  double bench_decode_impl(int n_steps, int pos0);
  void enqueue_layer_decode(int l, hipStream_t s);
  void enqueue_decode(hipStream_t s);
  void enqueue_prefill(int T, int pos0, hipStream_t s, bool embed = true);
  // one layer over T activation rows: a prompt chunk at positions pos0.. of KV slot kv_slot_
  // (batched == false) or T decode rows of slots bslots_ at positions bpos_ (batched == true)
  void enqueue_rows_layer(int l, int T, int pos0, bool batched, hipStream_t s);
  void enqueue_rows_ffn(int l, int T, hipStream_t s, bool t16 = false);
  void enqueue_head(const float* xrow, int advance_pos, hipStream_t s, int slot = 0);
  // batch_step on the MFMA batched projections (bmm.hip): one layer over the B decode rows
  void enqueue_batch_layer(int l, int B, hipStream_t s);
  void enqueue_batch_step(int B, hipStream_t s);
  void bmm_rows(const QMat& w, const __half* xh, int ldh, float* out, int ldo, int n_out, int B, hipStream_t s,
                long long* dbg = nullptr);
  void down_rows(const QMat& w, const __half* xh, int ldh, float* out, int B, hipStream_t s, bool zero_qkv,
                 long long* dbg = nullptr);
  void bprep_rows(const float* x, int ldx, bool swiglu, const float* norm_w, int K, int B, float* zero, int zero_n,
                  hipStream_t s, int swiglu_group = 32);
  void setup_batch_mfma();
  SamplerParamsDev make_sparams(const SamplingOpts& sp) const;
  void begin_slot_state(int slot, const std::vector<int>& prompt, const SamplingOpts& sp);
  void launch_step(int slot = 0);  // one decode step of `slot` on the single-row GEMV path
  void check(hipError_t e, const char* what);
  void check_device_err();

  HParams hp_;
  EngineOptions opt_;
  hipStream_t stream_ = nullptr;
  void* comm_ = nullptr;  // ncclComm_t
  std::unique_ptr<P2PComm> p2p_;
  int p2p_max_n_ = 0;       // floats per P2P message (decode-sized, or everything in "ipc" mode)
  std::unique_ptr<TPChannel> tp_ctl_;
  bool tp_stopped_ = false;
  std::vector<void*> allocs_;
  float* gather_buf_ = nullptr;  // gather_logits_rows scratch (TP), grow-only
  size_t gather_cap_ = 0;
  size_t dev_bytes_ = 0;
  bool healthy_ = true;
  std::string last_error_;

  // local (per-rank) sizes
  int nh_l_ = 0, nkv_l_ = 0, nq_ = 0, nkvd_ = 0, F_l_ = 0, V_l_ = 0, V_pad_ = 0;
  int V_real_l_ = 0;          // real vocabulary rows of this rank's shard (<= V_l_)
  size_t q0_ = 0, kv0_ = 0, f0_ = 0;   // this rank's first q row / kv row / FFN feature

  // weights
  QMat tok_embd_, output_;
  float* out_norm_ = nullptr;
  std::vector<Layer> layers_;

  // buffers
  float* x_ = nullptr;        // [n_batch][d]
  float* tmp_ = nullptr;      // [n_batch][d]  (TP partial / MoE expert output)
  float* tmp_b_ = nullptr;    // [bmax][d] TP: batched row-parallel partials, kept zero by the accumulating all-reduce
  __hip_bfloat16* xb_ = nullptr;    // [n_batch][d]
  float* qkv_ = nullptr;      // [n_batch][nq + 2 nkvd]
  float* q_ = nullptr;        // [n_batch][nq]
  float* attn_ = nullptr;     // [n_batch][nq]
  __hip_bfloat16* attnb_ = nullptr; // [n_batch][nq]
  __hip_bfloat16* h_ = nullptr;     // [n_batch][F_l]
  float* hf_ = nullptr;       // [n_expert_used or 1][F_l]
  float* logits_ = nullptr;   // [V_pad]
  float* logits_l_ = nullptr; // [V_l]
  __half* kc_ = nullptr;      // [n_layer][nkv_l][n_ctx][hd]
  __half* vc_ = nullptr;
  float2* rope_ = nullptr;
  float* rope_freq_ = nullptr;  // [hd / 2]: the pairs' angular frequencies (deferred batched RoPE)
  float* attn_part_ = nullptr;
  // [64] per-kv-head split counters (last-arriver combine); word 63 is reserved as the
  // weight touch's pf_sink, which is why the touch needs nkv_l_ < 63
  int* attn_cnt_ = nullptr;
  // decode attention pre-touches this layer's Wo into the memory-side cache (LFK_ATTN_TOUCH=0:
  // off, A/B; touching the next Q|K|V or the gate/up heads too measured neutral, r2-r3)
  bool attn_touch_ = true;
  size_t cand_words_ = 0;     // sampler candidate block of one row (sampler_cand_words(V_l))
  unsigned* cand_ = nullptr;  // [cand_words_] this rank's stage-1 block (single row)
  unsigned* cand_all_ = nullptr;   // [tp][cand_words_] gathered blocks (tp > 1)
  int* state_ = nullptr;
  int* ring_ = nullptr;
  int* out_tokens_ = nullptr;
  int* tokens_ = nullptr;     // [n_batch]
  SamplerParamsDev* sparams_ = nullptr;
  float* router_logits_ = nullptr;  // [n_batch][E]
  // grouped MoE prefill (moe.hip): routing lists and gathered row buffers, [n_batch * k] rows
  int* moe_sel_ = nullptr; float* moe_selw_ = nullptr; int* moe_off_ = nullptr; int* moe_tok_ = nullptr;
  float* moe_gw_ = nullptr; int* moe_pos_ = nullptr;
  __hip_bfloat16* moe_xg_ = nullptr; __hip_bfloat16* moe_hg_ = nullptr; float* moe_yg_ = nullptr;
  int* moe_ids_ = nullptr;
  float* moe_w_ = nullptr;
  int* h_ring_ = nullptr;     // pinned [64]
  int* h_tokens_ = nullptr;   // pinned [n_batch]

  // KV slots: kc_/vc_ hold n_slots caches of slot_stride_ halves each; state_/ring_/sparams_
  // hold n_slots entries (slot 0 first)
  size_t slot_stride_ = 0;
  int kv_slot_ = 0;           // the slot enqueue_prefill writes
  int bmax_ = 0;              // batch_step rows (min(n_slots, n_batch)); 0 = no batching
  int* bslots_ = nullptr;     // [bmax] device: slot of each batch row
  int* bpos_ = nullptr;       // [bmax] position of each row's current token
  int* btok_ = nullptr;       // [bmax] current token of each row
  int* btok_out_ = nullptr;   // [bmax] sampled tokens
  float* logits_b_ = nullptr; // [bmax][V_pad]
  unsigned* cand_b_ = nullptr;      // [bmax][cand_words_]
  unsigned* cand_all_b_ = nullptr;  // [tp][bmax][cand_words_]
  float* attn_part_b_ = nullptr;   // [bmax][attn_decode_workspace_floats]
  int* attn_cnt_b_ = nullptr;      // [bmax][64]
  int* h_bslots_ = nullptr;   // pinned [bmax]
  int* h_btok_ = nullptr;     // pinned [bmax]
  // steps in flight (batch_launch / batch_collect): a ring of two, each with its own pinned
  // token buffer and completion event
  int* h_btok2_[2] = {nullptr, nullptr};
  // h_btok2_[i] are host-mapped (fine-grained): the batch-step graph of flight parity i has its
  // sampler store the tokens there directly (btok_dev_[i]: their device addresses; sample_host_ is
  // the one the step being captured writes)
  int* btok_dev_[2] = {nullptr, nullptr};
  int* sample_host_ = nullptr;
  hipEvent_t bev_[2] = {nullptr, nullptr};
  int fl_B_[2] = {0, 0};
  bool fl_b1_[2] = {false, false};
  int fl_head_ = 0, fl_n_ = 0;
  void check_batch_rows(const std::vector<int>& slots) const;
  void enqueue_batch_launch(const std::vector<int>& slots, int* h_dst);
  void batch_launch_impl(const std::vector<int>& slots);
  std::vector<int> batch_collect_impl();
  int bslots_n_ = -1;         // rows of the row -> slot map last uploaded to bslots_
  int last_batch_ = 0;
  // batch_step projections on the MFMA batched projection (bmm.hip: weights streamed once per
  // step for all rows) instead of the prefill GEMM: attention/head (bg_) and the dense FFN
  // (bg_ffn_); shapes bmm does not take keep the GEMM path
  bool bg_ = false, bg_ffn_ = false;
  bool prefill_t16_ = false;  // LFK_PREFILL_T16=0: the planar bf16 gemm_dq (A/B)
  // MoE FFN on the batched projections: the experts as one stacked SwiGLU matrix and one
  // K-concatenated down matrix (t_gu / t_down of each layer), routed by dense per-row expert
  // weights ew_b_ [bmax][E] (bmm.hip, BmmArgs::ew)
  bool moe_b_ = false;
  float* ew_b_ = nullptr;
  __half* xh_b_ = nullptr;    // [bmax][max(d, nq, F)] prepared f16 projection input
  QMat t_output_;             // tile16 copy of the output head
  float* gu_b_ = nullptr;     // [bmax][2 F_l] gate/up pre-activations (32-row interleaved)
  __half* hh_b_ = nullptr;    // [bmax][F_l] (MoE: [bmax][E F_l]) down input written by the SwiGLU epilogue
  // RMSNorm folded into the one-part projections' staging where the rows fit (Q|K|V, gate/up: no
  // prep launch; the head as one part with the folded final norm measured neutral-to-slower)
  // Q|K|V as a split-K projection (bmm.hip BmmArgs::qkv_sk, B <= 8): RoPE'd partial sums added
  // into qkv_b_ [bmax][nq + 2 nkvd] (+ the rows' sums of squares ss_b_ [16]); the batched
  // attention normalises them and appends the new K / V, the Wo launch re-zeroes both
  // (LFK_QKV_SK=0: the one-part Q|K|V with the RoPE / KV-append epilogue, A/B)
  bool qkv_sk_ = true;
  bool tp_on_ = false;        // the tensor-parallel code paths (tp_size > 1, or comm=rccl at one rank)
  int layer_end_ = 0;         // layers [opt_.layer_begin, layer_end_) live here
  long long* step_clk_ = nullptr;
  int step_clk_layer_ = -1;
  long long* clk_of(int l, int k) const {
    return l == step_clk_layer_ && step_clk_ ? step_clk_ + (size_t)k * kStepClkBlocks * 16 : nullptr;
  }
  float* qkv_b_ = nullptr;
  float* ss_b_ = nullptr;
  // the single-row decode's attention and Wo in one launch (no TP; gemv.hip attn_wo1): Wo
  // streams its weights while the attention runs and starts once every kv head is done
  // (dec_done_); a timed-out wait sets *wo_err_ (host-mapped). LFK_WO_FUSE=0: two launches (A/B).
  bool wo_fuse_ = true;
  bool moe_route_fuse_ = true;  // single-row MoE: the router inside the gate/up GEMV (LFK_MOE_ROUTE_FUSE A/B)
  int* wo_err_h_ = nullptr;   // host view
  int* wo_err_ = nullptr;     // device view
  // batched dense FFN as one launch (bmm_ffn_chain): per-layer K-part counters (64 per layer),
  // zeroed by each step's first kernel; a timed-out consumer wait sets *chain_err_ (host-mapped)
  // in-launch chains of the batched layer: 1 = gate/up + down in one launch (Wo its own launch),
  // 2 = Wo + gate/up + down in one launch (measured the same as 1: 2.209 vs 2.204 ms per B = 6
  // step, r5g), 0 = three launches (LFK_FFN_CHAIN, A/B)
  int ffn_chain_ = 1;
  int* chain_cnt_ = nullptr;
  int* chain_err_h_ = nullptr;
  int* chain_err_ = nullptr;
  int* dec_done_ = nullptr;   // single-row decode: [n_layer][64] done counters (attn_wo1)
  size_t qkv_b_zero_n() const { return (size_t)bmax_ * (nq_ + 2 * nkvd_) + 16; }

  std::vector<hipGraphExec_t> bgraph_;  // captured batch steps, one per row count
  // a second instantiation of each, for the pipelined launches: consecutive in-flight steps
  // alternate between the two (a graph exec relaunched while its previous launch is still
  // queued may be held back by the runtime until that one completes)
  std::vector<hipGraphExec_t> bgraph2_;
  int launch_par_ = 0;  // which instantiation enqueue_batch_launch uses (0: bgraph_, 1: bgraph2_)
  // single-row decode (GEMV path) of KV slot dslot_: enqueue_decode reads it while capturing;
  // one graph per slot (slot 0's is graph_exec_). batch_step over ONE row takes this path
  // (the faster one at B = 1: 1.65 vs 2.18 ms)
  int dslot_ = 0;
  std::vector<hipGraphExec_t> sgraph_, sgraph2_;  // (second instances: pipelined one-row steps)
  bool last_b1_ = false;      // the last batch_step ran its one row on the single-row path
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t graph_exec_ = nullptr, graph_exec2_ = nullptr;
  // layer-split chain (chain_generate): this stage's decode step (layers, + embedding on the first
  // stage, + head and sampler on the last), two graph instances alternating by step parity
  void enqueue_stage_decode(hipStream_t s);
  void chain_step(const Engine* prev, const Engine* last, const std::vector<Engine*>& others);
  hipGraphExec_t chain_graph_[2] = {nullptr, nullptr};
  int chain_par_ = 0;
  hipEvent_t chain_ev_ = nullptr;
  static constexpr int kDepth = 2;
  hipEvent_t step_ev_[kDepth] = {};
};

}  // namespace lfk
