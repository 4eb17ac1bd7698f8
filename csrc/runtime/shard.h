// Tensor-parallel shard plan shared by the GPU engine and the CPU backend
// (SURVEY §2.5 "Tensor parallelism": Megatron-style column split of Q/K/V and
// gate/up, row split of Wo and down, vocab split of the output head).
//
// Rank r of tp owns
//   q heads   [r*nh_l, (r+1)*nh_l)      -> rows  [r*nq,  (r+1)*nq)  of attn_q
//   kv heads  [r*nkv_l, (r+1)*nkv_l)    -> rows  [r*nkvd,(r+1)*nkvd) of attn_k / attn_v
//   Wo        all rows, columns [r*nq, (r+1)*nq)
//   FFN       features [r*F_l, (r+1)*F_l) of gate/up (rows) and down (columns)
//   lm_head   vocab rows [r*V_l, (r+1)*V_l) (zero-padded past n_vocab)
// Every cut is a multiple of 32 columns, so the per-32 q8 activation blocks of a
// shard are exactly the blocks of the unsharded vector and TP changes only the
// float summation order of the partial sums (no extra quantisation error).
// Uneven `tensor_split` ratios are rejected: ranks are symmetric by design.
#pragma once
#include <stdexcept>
#include <string>

namespace lfk {

struct ShardPlan {
  int tp = 1, rank = 0;
  int nh_l = 0, nkv_l = 0, nq = 0, nkvd = 0, F_l = 0, V_l = 0, V_pad = 0;
  size_t q_row0() const { return (size_t)rank * nq; }
  size_t kv_row0() const { return (size_t)rank * nkvd; }
  size_t f0() const { return (size_t)rank * F_l; }
  size_t v_row0() const { return (size_t)rank * V_l; }
};

inline ShardPlan make_shard_plan(int n_head, int n_head_kv, int head_dim, int n_ff, int n_vocab, int tp, int rank) {
  if (tp < 1 || rank < 0 || rank >= tp) throw std::runtime_error("bad tensor-parallel rank/size");
  if (n_head % tp || n_head_kv % tp)
    throw std::runtime_error("tensor parallel degree " + std::to_string(tp) + " must divide the head counts (" +
                             std::to_string(n_head) + "/" + std::to_string(n_head_kv) + ")");
  if (n_ff % tp || (n_ff / tp) % 32)
    throw std::runtime_error("tensor parallel degree must divide n_ff into multiples of 32");
  ShardPlan p;
  p.tp = tp;
  p.rank = rank;
  p.nh_l = n_head / tp;
  p.nkv_l = n_head_kv / tp;
  p.nq = p.nh_l * head_dim;
  p.nkvd = p.nkv_l * head_dim;
  if (tp > 1 && (p.nq % 32 || p.nkvd % 32)) throw std::runtime_error("per-rank head slice must be a multiple of 32");
  p.F_l = n_ff / tp;
  p.V_l = (n_vocab + tp - 1) / tp;
  p.V_pad = p.V_l * tp;
  return p;
}

}  // namespace lfk
