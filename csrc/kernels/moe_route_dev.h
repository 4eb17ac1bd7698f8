// MoE routing finish shared by moe.hip's router kernel and the routed SwiGLU GEMV (gemv.hip):
// one wave turns the per-wave partial router sums into logits, softmax, top-k (lowest index on
// ties) and renormalised weights. Both callers reduce in the same order (per-thread float4
// partials -> wave_sum_fast -> waves 0..NW-1 in order), so their routing is bit-identical.
#pragma once
#include "qdot.h"

namespace lfk {

// red[w][e] (e < EM): wave w's router partial of expert e; red[w][EM]: its sum of squares.
// Lane j < k returns (id_j, w_j / sum of the k picks); lane e < E returns its logit in *logit.
template <int EM, int NW>
__device__ __forceinline__ void moe_route_finish(const float (*red)[EM + 1], int E, int k, int d, float eps, int lane,
                                                 int& my_id, float& my_w, float& sel_sum, float& logit) {
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) tot += red[w][EM];
  const float sc = rsqrtf(tot / (float)d + eps);
  float v = -INFINITY;
  if (lane < E) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += red[w][lane];
    v = sum * sc;
  }
  logit = v;
  const float m = wave_max(v);
  float p = lane < E ? __expf(v - m) : 0.f;
  p /= wave_sum(p);
  float taken = lane < E ? p : -1.f;
  sel_sum = 0.f;
  my_w = 0.f;
  my_id = 0;
  for (int j = 0; j < k; ++j) {
    float best = taken;
    int bi = lane;
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == j) { my_id = bi; my_w = best; }
    sel_sum += best;
    if (lane == bi) taken = -1.f;
  }
}

}  // namespace lfk
