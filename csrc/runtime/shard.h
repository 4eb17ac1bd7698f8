// Tensor-parallel shard plan shared by the GPU engine and the CPU backend
// (SURVEY §2.5 "Tensor parallelism": Megatron-style column split of Q/K/V and
// gate/up, row split of Wo and down, vocab split of the output head; §3.5:
// `tensor_split` ratios mapped to kv-head and 256-superblock granularity).
//
// Rank r owns
//   kv heads  [kv_h0, kv_h0 + nkv_l)  and the q heads of those GQA groups
//             -> rows [q0, q0 + nq) of attn_q, [kv0, kv0 + nkvd) of attn_k / attn_v,
//                columns [q0, q0 + nq) of attn_output
//   FFN       features [f0, f0 + F_l) of gate/up (rows) and down (columns)
//   lm_head   vocab rows [r*V_l, (r+1)*V_l) (even split, zero-padded past n_vocab:
//             the logit all-gather moves equal counts)
// Heads are apportioned in whole kv heads (a GQA group never straddles ranks;
// groups of kv heads whose q columns fill whole 256-wide superblocks of attn_output)
// and FFN features in units of 256 (one K-quant superblock of the down
// projection's columns; 32 when n_ff is not a multiple of 256), proportionally
// to `tensor_split` by largest remainder, at least one unit per rank. Uniform or
// absent ratios with divisible counts give the plain even split. Every cut is a
// multiple of 32 columns, so the per-32 q8 activation blocks of a shard are the
// blocks of the unsharded vector and TP changes only the float summation order.
#pragma once
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

namespace lfk {

struct ShardPlan {
  int tp = 1, rank = 0;
  int nh_l = 0, nkv_l = 0, nq = 0, nkvd = 0, F_l = 0, V_l = 0, V_pad = 0;
  size_t q0 = 0, kv0 = 0, f0_ = 0;
  size_t q_row0() const { return q0; }
  size_t kv_row0() const { return kv0; }
  size_t f0() const { return f0_; }
  size_t v_row0() const { return (size_t)rank * V_l; }
};

// units split over ranks proportionally to w (largest remainder, >= 1 each)
inline std::vector<int> apportion(int units, const std::vector<double>& w) {
  const int n = (int)w.size();
  if (units < n) throw std::runtime_error("tensor split: fewer units than ranks");
  double tot = 0;
  for (double v : w) tot += v;
  std::vector<int> out(n, 1);
  const int rest = units - n;
  std::vector<std::pair<double, int>> frac;
  int given = 0;
  for (int i = 0; i < n; ++i) {
    const double q = rest * w[i] / tot;
    const int f = (int)std::floor(q);
    out[i] += f;
    given += f;
    frac.push_back({q - f, -i});  // ties: lower rank first
  }
  std::sort(frac.rbegin(), frac.rend());
  for (int k = 0; k < rest - given; ++k) out[-frac[k].second] += 1;
  return out;
}

inline ShardPlan make_shard_plan(int n_head, int n_head_kv, int head_dim, int n_ff, int n_vocab, int tp, int rank,
                                 const std::vector<float>& tensor_split = {}) {
  if (tp < 1 || rank < 0 || rank >= tp) throw std::runtime_error("bad tensor-parallel rank/size");
  if (n_head_kv <= 0 || n_head % n_head_kv) throw std::runtime_error("n_head must be a multiple of n_head_kv");
  std::vector<double> w(tp, 1.0);
  if (!tensor_split.empty()) {
    if ((int)tensor_split.size() != tp)
      throw std::runtime_error("tensor_split has " + std::to_string(tensor_split.size()) + " entries for " +
                               std::to_string(tp) + " ranks");
    for (int i = 0; i < tp; ++i) {
      if (!(tensor_split[i] > 0)) throw std::runtime_error("tensor_split entries must be > 0");
      w[i] = tensor_split[i];
    }
  }
  if (n_head_kv < tp)
    throw std::runtime_error("tensor parallel degree " + std::to_string(tp) + " exceeds the kv-head count " +
                             std::to_string(n_head_kv));
  const int unit = (n_ff % 256 == 0) ? 256 : 32;
  if (n_ff % unit) throw std::runtime_error("n_ff must be a multiple of 32");
  const int g = n_head / n_head_kv;
  // kv heads move in groups whose q columns span whole 256-wide superblocks: attn_output's
  // column slice starts at q0, and a K-quant block must not straddle ranks
  int ukv = 1;
  if (tp > 1)
    while (ukv < n_head_kv && ((size_t)ukv * g * head_dim) % 256) ++ukv;
  if (n_head_kv % ukv || n_head_kv / ukv < tp)
    throw std::runtime_error("cannot split " + std::to_string(n_head_kv) + " kv heads over " + std::to_string(tp) +
                             " ranks in superblock-aligned groups of " + std::to_string(ukv));
  std::vector<int> kv = apportion(n_head_kv / ukv, w);
  for (int& v : kv) v *= ukv;
  const std::vector<int> fu = apportion(n_ff / unit, w);
  ShardPlan p;
  p.tp = tp;
  p.rank = rank;
  int kv_before = 0, f_before = 0;
  for (int i = 0; i < rank; ++i) { kv_before += kv[i]; f_before += fu[i]; }
  p.nkv_l = kv[rank];
  p.nh_l = p.nkv_l * g;
  p.nq = p.nh_l * head_dim;
  p.nkvd = p.nkv_l * head_dim;
  p.q0 = (size_t)kv_before * g * head_dim;
  p.kv0 = (size_t)kv_before * head_dim;
  if (tp > 1 && (p.nq % 32 || p.nkvd % 32)) throw std::runtime_error("per-rank head slice must be a multiple of 32");
  p.F_l = fu[rank] * unit;
  p.f0_ = (size_t)f_before * unit;
  p.V_l = (n_vocab + tp - 1) / tp;
  p.V_pad = p.V_l * tp;
  return p;
}

}  // namespace lfk
