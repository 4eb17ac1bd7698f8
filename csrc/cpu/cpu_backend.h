// C++ CPU backend (SURVEY U12 / N0a `cpu/`): runs a GGUF model entirely on the
// host for n_gpu_layers = 0 (BASELINE config #1, TinyLlama Q8_0), and serves as
// the CPU half of a hybrid (partial-offload) placement.
//
// Same weight layout (planar repack) and the same numerics as the GPU kernels:
// activations are quantised to int8 per 32 values, weights stay block-quantised,
// dot products are integer per 32-weight chunk with the per-sub-block scales
// applied once per chunk; KV cache is f16. Prefill is batched (every weight row
// is decoded once per prompt chunk and reused for all tokens). OpenMP over rows.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../common.h"
#include "../runtime/shard.h"

namespace lfk {

struct CpuMat {
  std::vector<uint8_t> data;
  int type = 0, rows = 0, K = 0;
  size_t expert_stride = 0;
  Planes P{};
};

struct CpuLayer {
  std::vector<float> attn_norm, ffn_norm;
  CpuMat wq, wk, wv, wo, w_gu, w_down, router, gu_exps, down_exps;
};

struct CpuSampling {
  int top_k = 40;
  float top_p = 0.95f, min_p = 0.05f, temp = 0.8f, repeat_penalty = 1.1f, freq_penalty = 0.f, presence_penalty = 0.f;
  int last_n = 64;
  uint64_t seed = 0;
};

struct CpuGenOut {
  std::vector<int> tokens;
  std::string finish;
  int n_evaluated = 0, n_prefilled = 0;
  double prefill_s = 0, decode_s = 0;
};

struct CpuOptions {
  int n_ctx = 512, n_threads = 0, n_batch = 64;
  int tp_rank = 0, tp_size = 1;   // tensor parallel (same shard plan as the GPU engine)
  std::vector<float> tensor_split;  // per-rank weights (empty = even); see runtime/shard.h
  int layer_end = -1;             // hybrid placement: only layers [0, layer_end) are resident
  bool load_head = true;          // output norm + lm_head resident
};

class CpuEngine {
 public:
  CpuEngine(const std::string& path, const CpuOptions& opts);
  // collectives for tp_size > 1 (e.g. torch.distributed gloo from Python):
  // allreduce(buf, n) sums in place; allgather(local, all, n_local) concatenates rank shards
  void set_comm(std::function<void(float*, size_t)> allreduce,
                std::function<void(const float*, float*, size_t)> allgather);
  CpuGenOut generate(const std::vector<int>& prompt, int n_keep, int max_new, const CpuSampling& sp,
                     const std::vector<int>& stop, const std::function<bool()>& poll,
                     const std::function<void(int)>& on_token);
  // logits of the last token after evaluating `tokens` at positions pos0..
  std::vector<float> eval_logits(const std::vector<int>& tokens, int pos0);

  // hybrid placement hooks: embed, run a layer range on hidden states, head
  void embed(const int* tokens, int T, float* x) const;
  void run_layers(float* x, int T, int pos0, int l0, int l1);
  void head(const float* xrow, float* logits);
  // hybrid: hidden states after layers [0, layer_end) for tokens at pos0.. ([T][n_embd])
  std::vector<float> eval_hidden(const std::vector<int>& tokens, int pos0);
  // KV state of positions [0, n): [K|V][n_layer][local kv heads][n][hd] f16 (save/load_state)
  size_t kv_state_bytes(int n) const { return 2 * (kc_.size() / (size_t)n_ctx_) * (size_t)n * sizeof(uint16_t); }
  void kv_transfer(void* buf, int n, bool load);

  int n_vocab() const { return n_vocab_; }
  int n_embd() const { return n_embd_; }
  int n_layer() const { return n_layer_; }
  int n_ctx() const { return n_ctx_; }
  int layer_end() const { return layer_end_; }
  int tp_rank() const { return sp_.rank; }
  int tp_size() const { return sp_.tp; }

 private:
  void matmul(const CpuMat& W, const float* x, int T, int ldx, float* y, int ldy, const std::vector<float>* norm,
              bool add) const;
  void attention(int l, const float* q, int T, int pos0, float* out) const;
  void ffn(const CpuLayer& L, float* x, int T);
  void reduce(float* y, size_t n);

  CpuOptions opt_;
  ShardPlan sp_;
  int layer_end_ = 0;
  std::function<void(float*, size_t)> allreduce_;
  std::function<void(const float*, float*, size_t)> allgather_;

  int n_vocab_ = 0, n_embd_ = 0, n_layer_ = 0, n_head_ = 0, n_head_kv_ = 0, head_dim_ = 0, n_ff_ = 0;
  int n_expert_ = 0, n_expert_used_ = 0, n_ctx_ = 0, n_threads_ = 1, n_batch_ = 64;
  float eps_ = 1e-5f, rope_base_ = 10000.f;
  CpuMat tok_embd_, output_;
  std::vector<float> out_norm_;
  std::vector<CpuLayer> layers_;
  std::vector<uint16_t> kc_, vc_;      // [layer][local kv_head][n_ctx][hd] f16
  std::vector<float> rope_cos_, rope_sin_;
};

// shared host reference of the sampler chain (same semantics as engine/sampling.py)
int cpu_sample(std::vector<float> logits, const std::vector<int>& window, const CpuSampling& sp, int step);
float splitmix_uniform(uint64_t seed, uint64_t step);

}  // namespace lfk
