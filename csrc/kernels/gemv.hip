// Decode GEMV family (T = 1): y = W x with W block-quantised (Q4_K/Q5_K/Q6_K/Q8_0,
// F16/F32) in the planar layout and x quantised to q8 in the kernel prologue.
//
// Replaces upstream MMVQ (`mul_mat_vec_q` + `quantize_q8_1`) and the
// ops it is chained with (RMSNorm K2, RoPE K5, KV store K6, SwiGLU K11, residual
// add K10) by ONE launch per projection:
//
//   prologue  : [RMSNorm(x)*w] -> per-32 int8 quantisation -> LDS (K B + K/8 B)
//   body      : each wave owns NR output rows; lane l streams chunks l, l+64, ...
//               (16 B of 4/6-bit weights per lane per chunk = 1 KiB per wave
//               instruction, non-temporal: weights are read once per token)
//   epilogue  : wave-reduce, then store / residual add / SwiGLU / RoPE+KV append
//
// Geometry: 256-thread blocks (4 waves), grid-stride over row groups with the
// grid capped at 4 blocks per CU so the prologue is amortised over many rows.
#include <algorithm>
#include <map>
#include <mutex>

#include "attn_dev.h"
#include "gemv_dev.h"
#include "moe_route_dev.h"

namespace lfk {

// One wave = one item of NR rows (NF outputs); 4 waves per block; grid capped at
// 4 blocks/CU and strided over items. Latency hiding: the first weight loads
// of a wave go out BEFORE the block's x prologue (norm + q8 quantisation into
// LDS), and the next item's first loads go out before the current item's
// cross-lane reduction and epilogue.
// SPLITK (EPI_ADD only): an item is NR rows x one group of 64*U chunks, and its
// partial dot products are atomically added to the residual. Every item is a
// single load round trip, so waves stream continuously instead of walking a
// long row pass by pass (the FFN down projection, K = 14336).
// EARLY (1024-thread blocks, one per CU): the first weight loads go out right
// after the x loads and BEFORE the prologue waits for x, so the weight stream
// starts at block entry; with one block per CU no other block's weight stream
// sits in front of this CU's x loads (in-order returns per CU).
// TP epilogue all-reduce of one output row (GemvArgs::tp_*): this rank's partial goes to every
// rank as a {value, epoch} granule, then the row's granules of every rank are read back from this
// rank's own area until they carry this launch's epoch and summed in rank order (bit-identical
// ranks). The epoch is per ROW (every launch writes every row exactly once on every rank, whatever
// the item shape of the launch), so a granule of an older launch is never taken for a newer one;
// a rank rewrites parity e & 1 of a row at epoch e + 2 only after it received every peer's
// granule of that row at e + 1, i.e. after the peer's launch e (its reads of parity e & 1) ended.
__device__ __forceinline__ void tp_store_row(const GemvArgs& a, int row, float v) {
  typedef unsigned long long u64;
  const int W = a.tp_world, R = a.tp_rank;
  const unsigned e = (unsigned)(a.tp_epochs[row] + 1);
  a.tp_epochs[row] = (int)e;  // lane-private word
  const size_t par = e & 1;
  const u64 g = ((u64)e << 32) | __float_as_uint(v);
#pragma unroll
  for (int p = 0; p < kP2PMaxRanks; ++p)
    if (p < W)
      __hip_atomic_store(reinterpret_cast<u64*>(a.tp_peers.data[p]) + (par * W + R) * a.tp_stride + a.tp_off + row, g,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const u64* mine = reinterpret_cast<const u64*>(a.tp_peers.data[R]) + par * W * a.tp_stride + a.tp_off + row;
  float val[kP2PMaxRanks];
  unsigned pending = (1u << W) - 1;
  const long long t0 = wall_clock64();
  for (int spins = 0; pending; ++spins) {
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p) {
      if (p < W && (pending >> p & 1)) {
        const u64 x = __hip_atomic_load(const_cast<u64*>(mine + (size_t)p * a.tp_stride), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM);
        if ((unsigned)(x >> 32) == e) {
          val[p] = __uint_as_float((unsigned)x);
          pending &= ~(1u << p);
        }
      }
    }
    if (!pending) break;
    if ((spins & 255) == 255) {
      if (wall_clock64() - t0 > 2000000000LL) {  // 20 s (100 MHz clock)
        __hip_atomic_store(a.tp_err, 300 + __builtin_ctz(pending), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        p2p_raise(a.tp_peers, W, R, 300 + __builtin_ctz(pending));  // poison the group
        return;
      }
      if (p2p_poisoned(a.tp_peers, W, R)) return;  // another rank failed: stop waiting
    }
    __builtin_amdgcn_s_sleep(1);
  }
  float sum = 0.f;
#pragma unroll
  for (int p = 0; p < kP2PMaxRanks; ++p)
    if (p < W) sum += val[p];
  a.out[row] = (a.resid ? a.resid[row] : 0.f) + sum;
}

// WAIT (SPLITK, not EARLY; attn_wo1): the first item's weights go out first, then the block waits
// for the in-flight producer of x (GemvArgs::wait) and loads x with sc1 loads.
// (bid, nblk): the block's index and count in the GEMV's grid (a plane of attn_wo1's grid).
// ROUTE (EARLY SwiGLU, BLOCK = 1024, K = 4096, NORM): the block routes the token itself (GemvArgs::route_w)
template <int QT, int EPI, int NR, int U, bool NORM, int BLOCK, bool TL = false, bool SPLITK = false,
          bool EARLY = false, bool WAIT = false, bool ROUTE = false>
__device__ __forceinline__ void gemv_body(const GemvArgs& a, const int bid, const int nblk) {
  static_assert(!WAIT || (SPLITK && !EARLY && !TL), "the in-flight wait is a split-K, non-EARLY form");
  static_assert(!ROUTE || (EARLY && !SPLITK && NORM && BLOCK == 1024 && EPI == EPI_SWIGLU), "routed form");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the prologue's kernarg fields in ONE batch of scalar loads (read where first used, each behind
  // its own s_waitcnt, they were 4-5 dependent round trips before the first weight load)
  {
    const void *p0 = a.w.base, *p1 = a.x, *p2 = a.norm_w, *p3 = a.out, *p4 = a.expert_ids, *p5 = a.dbg_clk,
               *p6 = a.resid, *p7 = a.wait;
    const int f0 = a.w.K, f1 = a.n_out, f2 = a.n_slots, f3 = a.debug, f4 = a.wait_n, f5 = a.grid_div, f6 = a.w.rows;
    const size_t z0 = a.w.P.p0, z1 = a.w.P.p1, z2 = a.w.P.p2, z3 = a.w.P.p3, z4 = a.w.P.s0, z5 = a.w.P.s1,
                 z6 = a.w.P.s2, z7 = a.w.P.s3;
    asm volatile("" ::"s"(p0), "s"(p1), "s"(p2), "s"(p3), "s"(p4), "s"(p5), "s"(p6), "s"(p7), "s"(f0), "s"(f1), "s"(f2),
                 "s"(f3), "s"(f4), "s"(f5), "s"(f6), "s"(z0), "s"(z1), "s"(z2), "s"(z3), "s"(z4), "s"(z5), "s"(z6),
                 "s"(z7), "s"(nblk));
  }
  // TL: per-block timeline (wall_clock64 ticks, microbenchmarks only):
  // [entry, prologue done, first item done, exit, items done by wave 0]
  long long* tl = nullptr;
  if constexpr (TL) {
    tl = a.dbg_clk + (size_t)bid * 5;
    if (threadIdx.x == 0) tl[0] = wall_clock64();
  }
  int n_done = 0;
  const int K = a.w.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + K);
  float* red = xd + (K >> 5);
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int nchunks = K >> 5;
  constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
  const int groups = (a.n_out + NF - 1) / NF;
  const int kparts = SPLITK ? (nchunks + 64 * U - 1) / (64 * U) : 1;
  const int total = groups * a.n_slots * kparts;
  constexpr int WPB = BLOCK / 64;
  // EARLY launches are one block per CU: each block takes a contiguous range of
  // items so every CU streams the same bytes (a grid-stride walk with 16 waves
  // per block left the last quarter of the CUs with half the items of the rest).
  int item, stride, item_end;
  if constexpr (EARLY) {
    const int per = (total + nblk - 1) / nblk;
    const int b0 = min(total, bid * per);
    item = b0 + wave;
    stride = WPB;
    item_end = min(total, b0 + per);
  } else {
    item = bid * WPB + wave;
    stride = nblk * WPB;
    item_end = total;
  }
  RowPtr R[NR];
  int slot = 0, f0 = 0;
  WStream<QT, NR, U> ws;
  XPrologue<NORM, BLOCK, WAIT> xp;
  int kp = 0;
  if constexpr (WAIT) {
    // the weights stream while the producer (the attention planes of this launch) finishes
    if (item < total) {
      item_rows<EPI, NR>(a, item / kparts, groups, R, slot, f0, a.expert_ids);
      kp = item % kparts;
      ws.load(R, kp * 64 * U, nchunks, lane);
    }
    if (threadIdx.x == 0) {
      for (int h = 0; h < a.wait_cnt; ++h) {
        for (int spins = 0; __hip_atomic_load(const_cast<int*>(a.wait) + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                            a.wait_n; ++spins) {
          if (spins > (1 << 22)) {
            __hip_atomic_store(a.wait_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    asm volatile("s_barrier" ::: "memory");  // the other waves load x after the poll matched
  }
  // The x prologue runs BEFORE the first weight loads: measured on MI355X, a
  // prologue whose L2 reads queue behind a saturated weight stream (its own CU's
  // or its neighbours') costs more than the latency its prefetch would hide.
  if (a.debug != 1 || ROUTE) xp.load(a.x, a.norm_w, K);
  const int* ids = a.expert_ids;
  if constexpr (ROUTE) {
    // the router, exactly as moe_router_fused_kernel sums it: thread t's float4 at k = 4t
    // (K == 4 * BLOCK), wave sums, waves in order (moe_route_dev.h)
    constexpr int EM = 8, NWV = BLOCK / 64;
    __shared__ float rred[NWV][EM + 1];
    __shared__ int rids[EM];
    const int E = a.route_E, i4 = threadIdx.x * 4;
    float4 rw[EM];
#pragma unroll
    for (int e = 0; e < EM; ++e) rw[e] = *reinterpret_cast<const float4*>(a.route_w + (size_t)min(e, E - 1) * K + i4);
    const float4 xv = xp.v[0], wv = xp.w[0];
    float ss = xv.x * xv.x + xv.y * xv.y + xv.z * xv.z + xv.w * xv.w;
    const float4 n = make_float4(xv.x * wv.x, xv.y * wv.y, xv.z * wv.z, xv.w * wv.w);
    float racc[EM];
#pragma unroll
    for (int e = 0; e < EM; ++e) racc[e] = e < E ? n.x * rw[e].x + n.y * rw[e].y + n.z * rw[e].z + n.w * rw[e].w : 0.f;
    ss = wave_sum_fast(ss);
#pragma unroll
    for (int e = 0; e < EM; ++e) racc[e] = e < E ? wave_sum_fast(racc[e]) : 0.f;
    if (lane == 0) {
      rred[wave][EM] = ss;
#pragma unroll
      for (int e = 0; e < EM; ++e) rred[wave][e] = racc[e];
    }
    __syncthreads();
    if (wave == 0) {
      int my_id;
      float my_w, sel_sum, v;
      moe_route_finish<EM, NWV>(rred, E, a.route_k, K, a.eps, lane, my_id, my_w, sel_sum, v);
      if (lane < a.route_k) rids[lane] = my_id;
      if (bid == 0) {  // the picks for the down projection (the next launch)
        if (a.route_logits && lane < E) a.route_logits[lane] = v;
        if (lane < a.route_k) {
          a.route_ids[lane] = my_id;
          a.route_wts[lane] = my_w / sel_sum;
        }
      }
    }
    __syncthreads();
    ids = rids;
  }
  if constexpr (EARLY) {  // unconditional (clamped) so no control-flow join sits between these loads and finish()
    const int it0 = min(item, total - 1);
    item_rows<EPI, NR>(a, SPLITK ? it0 / kparts : it0, groups, R, slot, f0, ids);
    if constexpr (SPLITK) kp = it0 % kparts;
    ws.load(R, kp * 64 * U, nchunks, lane);
  }
  const float xs = a.debug != 1 ? xp.finish(a.x, a.norm_w, a.eps, K, xq, xd, red) : 1.f;
  if constexpr (!EARLY && !WAIT) {
    if (item < total) {
      item_rows<EPI, NR>(a, SPLITK ? item / kparts : item, groups, R, slot, f0, ids);
      if constexpr (SPLITK) kp = item % kparts;
      ws.load(R, kp * 64 * U, nchunks, lane);
    }
  }
  if constexpr (TL) { if (threadIdx.x == 0) tl[1] = wall_clock64(); }
  if (a.debug == 2) {
    if (threadIdx.x == 0) a.out[0] = (float)xq[5] * xs;
    return;
  }
  while (item < item_end) {
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    if constexpr (SPLITK) ws.dot(kp * 64 * U, nchunks, xq, xd, acc, lane);
    else ws.finish_rows(R, nchunks, xq, xd, acc, lane);
    const int cs = slot, cf = f0;
    const int next = item + stride;
    if (next < item_end) {
      item_rows<EPI, NR>(a, SPLITK ? next / kparts : next, groups, R, slot, f0, ids);
      if constexpr (SPLITK) kp = next % kparts;
      ws.load(R, kp * 64 * U, nchunks, lane);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] *= xs;
    const float v = reduce_rows<NR>(acc, lane);        // lane l: row l % NR
    if constexpr (EPI == EPI_SWIGLU) {
      const float u = __shfl(v, (lane + NF) & 63);      // up row NF + r sits in lane NF + r
      if (lane < NF && cf + lane < a.n_out) a.out[(size_t)cs * a.out_slot_stride + cf + lane] = silu(v) * u;
    } else if (EPI == EPI_STORE && !SPLITK && a.tp_world > 0) {
      if (lane < NF && cf + lane < a.n_out) tp_store_row(a, cf + lane, v);
    } else if (lane < NF && cf + lane < a.n_out) {
      float* o = a.out + (size_t)cs * a.out_slot_stride + cf + lane;
      if constexpr (EPI == EPI_STORE) *o = a.resid ? v + a.resid[cf + lane] : v;
      else if constexpr (SPLITK) atomicAdd(o, v);
      else *o += v;
    }
    item = next;
    if constexpr (TL) {
      if (threadIdx.x == 0 && n_done == 0) tl[2] = wall_clock64();
      ++n_done;
    }
  }
  if constexpr (TL) {
    if (threadIdx.x == 0) { tl[3] = wall_clock64(); tl[4] = n_done; }
  }
}

template <int QT, int EPI, int NR, int U, bool NORM, int BLOCK, bool TL = false, bool SPLITK = false,
          bool EARLY = false, bool ROUTE = false>
__global__ __launch_bounds__(BLOCK) void gemv_kernel(GemvArgs a) {
  // the body reads the arguments through the kernarg segment pointer (a reference to the by-value
  // parameter would make the compiler copy it to scratch)
  const GemvArgs* ka = (const GemvArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  gemv_body<QT, EPI, NR, U, NORM, BLOCK, TL, SPLITK, EARLY, false, ROUTE>(*ka, blockIdx.x, gridDim.x);
  (void)a;
}

// ---------------------------------------------------------------- fused decode attention + Wo
// One launch for the single-row decode's attention AND its Wo projection: grid (kv heads,
// splits, 1 + Wo planes). Plane 0 is the attention (attn_dev.h) with done counters (each kv
// head's output stored sc1, counted once); the planes past it are the split-K Wo GEMV (4 rows x
// 64 chunks per wave item, atomics into the residual) whose blocks issue their first item's
// weights at once, wait for every kv head's counter and quantise x from sc1 loads. Wo's weight
// stream overlaps the latency-bound attention, and the launch replaces two (4 per layer).
struct AttnWo1Args {
  AttnDecodeArgs att;
  GemvArgs wo;
  int n_wo = 0;  // Wo blocks
};

template <int QT, int HD, int G>
__global__ __launch_bounds__(256) void attn_wo1_kernel(AttnWo1Args p) {
  const AttnWo1Args* k = (const AttnWo1Args*)__builtin_amdgcn_kernarg_segment_ptr();
  if (blockIdx.z == 0) {
    attn_decode_body<HD, G, false>(k->att);
    return;
  }
  const int per = gridDim.x * gridDim.y;
  const int vb = ((int)blockIdx.z - 1) * per + blockIdx.y * gridDim.x + blockIdx.x;
  if (vb >= k->n_wo) return;
  gemv_body<QT, EPI_ADD, 4, 1, false, 256, false, true, false, true>(k->wo, vb, k->n_wo);
  (void)p;
}

bool attn_wo1(const AttnDecodeArgs& aa, const GemvArgs& wo, hipStream_t s) {
  const int G = aa.n_kv_head > 0 ? aa.n_head / aa.n_kv_head : 0;
  // (G = 8, the 70B: the one launch measured 9.88 vs 9.74 ms per token for two, r4 - the G = 8
  // attention body's registers (168) leave the Wo planes 2-3 waves per SIMD: not taken)
  if (aa.head_dim != 128 || G != 4 || aa.batch != 0 || !aa.done || !aa.out || aa.out_h || aa.qkv_raw ||
      (wo.w.type != T_Q4_K && wo.w.type != T_Q6_K) || wo.norm_w || wo.n_slots != 1 || wo.expert_ids || wo.resid ||
      wo.debug || wo.dbg_clk || wo.w.K % 2048)
    return false;
  for (int r = 0; r < AttnDecodeArgs::kTouchRanges; ++r)
    if (aa.pf[r]) return false;
  if (!wo.wait || wo.wait != aa.done || wo.wait_cnt != aa.n_kv_head || wo.wait_n != 1 || !wo.wait_err ||
      wo.x != aa.out)
    throw std::runtime_error("attn_wo1: the Wo must wait for this attention's done counters");
  AttnWo1Args p;
  p.att = aa;
  p.wo = wo;
  // 4-row x 64-chunk items, grid-strided over at most 512 blocks (2 per CU): at d = 4096 one item
  // per wave - every weight of Wo in flight before the wait; at d = 8192 (70B) 4 per wave, the
  // x prologue (each block quantises all of x) amortised as the separate GEMV's grid cap does
  // (one item per wave there cost 2048 prologues: 29.7 vs ~15 us per layer, r4 profile)
  const int items = (wo.n_out + 3) / 4 * (wo.w.K / 2048);
  p.n_wo = std::min((items + 3) / 4, 512);
  const int splits = (aa.n_ctx + 63) / 64, per = aa.n_kv_head * splits;
  const dim3 grid(aa.n_kv_head, splits, 1 + (p.n_wo + per - 1) / per);
  const size_t lds = wo.w.K + (wo.w.K / 32) * 4 + 128;
  if (wo.w.type == T_Q4_K) hipLaunchKernelGGL((attn_wo1_kernel<T_Q4_K, 128, 4>), grid, dim3(256), lds, s, p);
  else hipLaunchKernelGGL((attn_wo1_kernel<T_Q6_K, 128, 4>), grid, dim3(256), lds, s, p);
  return true;
}

QMat make_qmat(const void* base, int type, int rows, int K, size_t expert_stride) {
  QMat m;
  m.base = static_cast<const uint8_t*>(base);
  m.type = type;
  m.rows = rows;
  m.K = K;
  m.P = planes_of(type, rows, K);
  m.expert_stride = expert_stride;
  return m;
}

static inline int grid_for(int items, int per_block = 4) {
  int b = (items + per_block - 1) / per_block;
  return b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b);
}

// Blocks of `kern` that are resident at once on the device (occupancy x CUs):
// the grid-stride GEMVs launch at most this many so no block waits for a second
// dispatch wave (its x prologue would be exposed after the first wave drains).
template <typename F>
static int resident_blocks(F kern, size_t lds, int block = 256) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  const auto key = std::make_pair(reinterpret_cast<const void*>(kern), lds * 4096 + (size_t)block);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, lds) != hipSuccess)
    throw std::runtime_error("gemv: device / occupancy query failed");
  const int r = std::max(1, per_cu) * std::max(1, cus);
  cache[key] = r;
  return r;
}
template <typename F>
static dim3 gemv_grid(F kern, size_t lds, int items, int block = 256, int div = 1) {
  const int wpb = block / 64;
  const int want = std::max(1, (items + wpb - 1) / wpb);
  return dim3(std::min(want, std::max(1, resident_blocks(kern, lds, block) / std::max(1, div))));
}

// (rows per item, passes per load group) for a weight type and shape.
// Items: prefer >= 2048 (8 waves per CU) so the grid is latency-tolerant;
// loads in flight per lane NR*U <= LB (register budget of the type's WRaw).
struct GemvCfg {
  int nr, u;
};
static int pow2_floor(int v) {
  int p = 1;
  while (p * 2 <= v) p *= 2;
  return p;
}
static GemvCfg pick_cfg(int qt, int rows, int nchunks, int min_nr) {
  const int LB = (qt == T_F32) ? 2 : ((qt == T_F16 || nchunks > 128) ? 4 : 8);
  // measured on MI355X with weights streamed from HBM (tools/gemv_sweep.sh):
  //   K > 4096 (FFN down)         : one row per wave, 4 passes (Q6_K: 2) in flight
  //   >= 16384 rows (gate/up, head): 4 rows per wave, 1 pass
  if (qt != T_F32 && qt != T_F16) {
    if (nchunks > 128) {  // long rows run on 1024-thread blocks: NR * U <= 4 (128 VGPRs)
      const int nr = std::max(1, min_nr);
      return {nr, std::max(1, (qt == T_Q6_K ? 2 : 4) / nr)};
    }
    if (rows >= 16384) return {4, 1};
  }
  int nr = (qt == T_F32 || qt == T_F16) ? 2 : 4;
  while (nr > min_nr && rows / nr < 2048) nr /= 2;
  const int passes = (nchunks + 63) / 64;
  int u = pow2_floor(std::max(1, std::min(LB / nr, passes)));
  if (nr * u > LB) u = std::max(1, LB / nr);
  return {nr, u};
}

// EARLY launches: 1024-thread blocks pinned to one per CU by their LDS request
// (> half of the 160 KiB), so the grid is exactly one block per CU.
static constexpr size_t kOnePerCuLds = 80 * 1024 + 256;
// classes: the SwiGLU gate/up, the long-K split-K (down) and the long-K Q|K|V, measured in-situ
// (decode step) on MI355X; pinning the others, or loading x before the weights in the pinned
// blocks, was slower (r2 sweeps)
enum EarlyCls : int { EC_SWIGLU = 1, EC_SPLITK_LONG = 2, EC_SPLITK = 4, EC_STORE = 8, EC_QKV = 16, EC_QKV_LONG = 32 };
static bool gemv_early(int cls) { return (cls & (EC_SWIGLU | EC_SPLITK_LONG | EC_QKV_LONG)) != 0; }
static int early_cls(int epi, int K) {
  if (epi == EPI_SWIGLU) return EC_SWIGLU;
  if (epi == EPI_ADD) return K > 4096 ? EC_SPLITK_LONG : EC_SPLITK;
  return EC_STORE;
}
template <typename F>
static void launch_early(F kern, size_t lds, int items, const GemvArgs& a, hipStream_t s) {
  const size_t l = std::max(lds, kOnePerCuLds);
  hipLaunchKernelGGL(kern, gemv_grid(kern, l, items, 1024), dim3(1024), l, s, a);
}

#define LFK_NRU_DISPATCH(NR_, U_, ...)                                              \
  do {                                                                               \
    if (NR_ == 4 && U_ >= 2) { constexpr int NR = 4, U = 2; __VA_ARGS__; }           \
    else if (NR_ == 4) { constexpr int NR = 4, U = 1; __VA_ARGS__; }                 \
    else if (NR_ == 2 && U_ >= 4) { constexpr int NR = 2, U = 4; __VA_ARGS__; }      \
    else if (NR_ == 2 && U_ == 2) { constexpr int NR = 2, U = 2; __VA_ARGS__; }      \
    else if (NR_ == 2) { constexpr int NR = 2, U = 1; __VA_ARGS__; }                 \
    else if (U_ >= 4) { constexpr int NR = 1, U = 4; __VA_ARGS__; }                  \
    else if (U_ == 2) { constexpr int NR = 1, U = 2; __VA_ARGS__; }                  \
    else { constexpr int NR = 1, U = 1; __VA_ARGS__; }                               \
  } while (0)

template <int QT, int EPI, int NR, int U>
static void launch_gemv_cfg(const GemvArgs& a, hipStream_t s) {
  if constexpr (EPI == EPI_SWIGLU && NR < 2) {
    throw std::runtime_error("gemv: swiglu needs >= 2 rows per item");
  } else if constexpr ((QT == T_F32 || QT == T_F16) && NR * U > 4) {
    throw std::runtime_error("gemv: config exceeds the F16/F32 register budget");
  } else {
    constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
    const size_t lds = a.w.K + (a.w.K / 32) * 4 + 128;
    const int items = (a.n_out + NF - 1) / NF * a.n_slots;
    // K > 4096 (FFN down, 70B): 1024-thread blocks so the x prologue is one batch
    // of loads per thread (issued before the weights) and 16 waves share its LDS
    // copy; 16 waves per CU cap the registers at 128, hence NR*U <= 4 there
    if constexpr (NR * U <= 4) {
      if (gemv_early(early_cls(EPI, a.w.K))) {
        if constexpr (EPI == EPI_SWIGLU) {
          if (a.route_w) {
            if (!a.norm_w || a.w.K != 4096 || a.route_E < 1 || a.route_E > 8 || a.route_k < 1 || a.route_k > a.route_E ||
                a.route_k != a.n_slots || !a.route_ids || !a.route_wts || !a.w.expert_stride)
              throw std::runtime_error("gemv: routed SwiGLU needs K = 4096, norm, E <= 8, k = n_slots, outputs");
            launch_early(gemv_kernel<QT, EPI, NR, U, true, 1024, false, false, true, true>, lds, items, a, s);
            return;
          }
        }
        if (a.route_w) throw std::runtime_error("gemv: routing is a SwiGLU form");
        if (a.norm_w) launch_early(gemv_kernel<QT, EPI, NR, U, true, 1024, false, false, true>, lds, items, a, s);
        else launch_early(gemv_kernel<QT, EPI, NR, U, false, 1024, false, false, true>, lds, items, a, s);
        return;
      }
    }
    if (a.route_w) throw std::runtime_error("gemv: routing needs the one-block-per-CU SwiGLU form");
    if (a.w.K > 4096) {
      if constexpr (NR * U <= 4) {
        if (a.norm_w) {
          auto k = gemv_kernel<QT, EPI, NR, U, true, 1024>;
          hipLaunchKernelGGL(k, gemv_grid(k, lds, items, 1024, a.grid_div), dim3(1024), lds, s, a);
        } else {
          auto k = gemv_kernel<QT, EPI, NR, U, false, 1024>;
          hipLaunchKernelGGL(k, gemv_grid(k, lds, items, 1024, a.grid_div), dim3(1024), lds, s, a);
        }
      } else {
        throw std::runtime_error("gemv: K > 4096 needs rows*passes <= 4");
      }
    } else if (a.norm_w) {
      auto k = gemv_kernel<QT, EPI, NR, U, true, 256>;
      hipLaunchKernelGGL(k, gemv_grid(k, lds, items, 256, a.grid_div), dim3(256), lds, s, a);
    } else {
      auto k = gemv_kernel<QT, EPI, NR, U, false, 256>;
      hipLaunchKernelGGL(k, gemv_grid(k, lds, items, 256, a.grid_div), dim3(256), lds, s, a);
    }
  }
}

// microbenchmark: the heuristic's config, instrumented (TL) - Q4_K/Q6_K only
template <int QT, int EPI>
static void launch_gemv_tl(const GemvArgs& a, hipStream_t s) {
  const int rows = (EPI == EPI_SWIGLU ? 2 * a.n_out : a.n_out) * a.n_slots;
  const GemvCfg c = pick_cfg(QT, rows, a.w.K >> 5, EPI == EPI_SWIGLU ? 2 : 1);
  LFK_NRU_DISPATCH(c.nr, c.u, ({
    if constexpr (!(EPI == EPI_SWIGLU && NR < 2) && NR * U <= 4) {
      constexpr int NF = (EPI == EPI_SWIGLU) ? NR / 2 : NR;
      const size_t lds = a.w.K + (a.w.K / 32) * 4 + 128;
      const int items = (a.n_out + NF - 1) / NF * a.n_slots;
      if (gemv_early(early_cls(EPI, a.w.K))) {
        if (a.norm_w) launch_early(gemv_kernel<QT, EPI, NR, U, true, 1024, true, false, true>, lds, items, a, s);
        else launch_early(gemv_kernel<QT, EPI, NR, U, false, 1024, true, false, true>, lds, items, a, s);
      } else if (a.w.K > 4096) {
        auto k = gemv_kernel<QT, EPI, NR, U, false, 1024, true>;
        hipLaunchKernelGGL(k, gemv_grid(k, lds, items, 1024), dim3(1024), lds, s, a);
      } else if (a.norm_w) {
        auto k = gemv_kernel<QT, EPI, NR, U, true, 256, true>;
        hipLaunchKernelGGL(k, gemv_grid(k, lds, items), dim3(256), lds, s, a);
      } else {
        auto k = gemv_kernel<QT, EPI, NR, U, false, 256, true>;
        hipLaunchKernelGGL(k, gemv_grid(k, lds, items), dim3(256), lds, s, a);
      }
    } else {
      throw std::runtime_error("gemv timeline: config not instrumented");
    }
  }));
}

// split-K residual GEMV (EPI_ADD): 4 rows x 64 chunks per item
template <int QT>
static void launch_gemv_splitk(const GemvArgs& a, hipStream_t s) {
  const size_t lds = a.w.K + (a.w.K / 32) * 4 + 128;
  const int items = (a.n_out + 3) / 4 * a.n_slots * ((a.w.K / 32 + 63) / 64);
  if (gemv_early(early_cls(EPI_ADD, a.w.K))) {
    if (a.norm_w) launch_early(gemv_kernel<QT, EPI_ADD, 4, 1, true, 1024, false, true, true>, lds, items, a, s);
    else launch_early(gemv_kernel<QT, EPI_ADD, 4, 1, false, 1024, false, true, true>, lds, items, a, s);
    return;
  }
  if (a.w.K > 4096) {  // long rows: 1024-thread blocks, one-batch x prologue
    auto k = a.norm_w ? gemv_kernel<QT, EPI_ADD, 4, 1, true, 1024, false, true>
                      : gemv_kernel<QT, EPI_ADD, 4, 1, false, 1024, false, true>;
    hipLaunchKernelGGL(k, gemv_grid(k, lds, items, 1024), dim3(1024), lds, s, a);
  } else if (a.norm_w) {
    auto k = gemv_kernel<QT, EPI_ADD, 4, 1, true, 256, false, true>;
    hipLaunchKernelGGL(k, gemv_grid(k, lds, items), dim3(256), lds, s, a);
  } else {
    auto k = gemv_kernel<QT, EPI_ADD, 4, 1, false, 256, false, true>;
    hipLaunchKernelGGL(k, gemv_grid(k, lds, items), dim3(256), lds, s, a);
  }
}

template <int QT, int EPI>
static void launch_gemv(const GemvArgs& a, hipStream_t s) {
  if constexpr (EPI == EPI_ADD && (QT == T_Q4_K || QT == T_Q5_K || QT == T_Q6_K || QT == T_Q8_0)) {
    if (!a.dbg_clk && a.w.K >= 4096 && !a.debug) return launch_gemv_splitk<QT>(a, s);
  }
  if (a.dbg_clk) {
    if constexpr (QT == T_Q4_K || QT == T_Q6_K) return launch_gemv_tl<QT, EPI>(a, s);
    else throw std::runtime_error("gemv timeline: Q4_K / Q6_K only");
  }
  const int rows = (EPI == EPI_SWIGLU ? 2 * a.n_out : a.n_out) * a.n_slots;
  const GemvCfg c = pick_cfg(QT, rows, a.w.K >> 5, EPI == EPI_SWIGLU ? 2 : 1);
  LFK_NRU_DISPATCH(c.nr, c.u, (launch_gemv_cfg<QT, EPI, NR, U>(a, s)));
}

template <int QT>
static void gemv_t(const GemvArgs& a, int epi, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: launch_gemv<QT, EPI_STORE>(a, s); break;
    case EPI_ADD: launch_gemv<QT, EPI_ADD>(a, s); break;
    case EPI_SWIGLU: launch_gemv<QT, EPI_SWIGLU>(a, s); break;
    default: throw std::runtime_error("gemv: bad epilogue");
  }
}

void gemv(const GemvArgs& a, int epi, hipStream_t s) {
  if (epi == EPI_SWIGLU && (a.n_out % 32)) throw std::runtime_error("gemv: swiglu features must be a multiple of 32");
  if (a.w.K % 32) throw std::runtime_error("gemv: K must be a multiple of 32");
  if (a.n_out <= 0) return;
  switch (a.w.type) {
    case T_Q4_K: gemv_t<T_Q4_K>(a, epi, s); break;
    case T_Q5_K: gemv_t<T_Q5_K>(a, epi, s); break;
    case T_Q6_K: gemv_t<T_Q6_K>(a, epi, s); break;
    case T_Q8_0: gemv_t<T_Q8_0>(a, epi, s); break;
    case T_F16: gemv_t<T_F16>(a, epi, s); break;
    case T_F32: gemv_t<T_F32>(a, epi, s); break;
    default: throw std::runtime_error("gemv: unsupported weight type");
  }
}

// ------------------------------------------------------------------ QKV + RoPE + KV append
// One launch for the Q, K and V projections. Their rows form at most two runs of
// equal quant type (Q4_K_M: [Q,K] Q4_K + [V] Q6_K on the bumped layers; Mixtral:
// [Q] Q4_K + [K,V] Q8_0); each run gets its own contiguous range of blocks, so a
// block only ever executes one type's code (registers = max of the two paths,
// not the sum, and one kernel boundary instead of two). Items are NR (even)
// consecutive rows, so RoPE pairs (2j, 2j+1) meet in one wave after the
// reduction; the RoPE (cos, sin) of an item is loaded with its weights.
struct QkvSeg {
  const uint8_t* base;
  Planes P;
  int rows;
  int kind;  // 0 = Q, 1 = K, 2 = V
};
struct QkvLaunch {
  QkvSeg seg[3];
  int nseg;
  int g1;        // first segment of the second type run (== nseg: one run)
  int blocks0;   // blocks given to the first run
  int K;
  const float* x;
  const float* norm_w;
  float eps;
  float* q_out;
  __half* k_cache;
  __half* v_cache;
  int n_ctx, head_dim;
  const int* pos;
  const float2* rope;
};

template <int QT, int NR>
__device__ __forceinline__ void qkv_item(const QkvLaunch& a, int s_lo, int s_hi, int item, RowPtr (&R)[NR], int& si,
                                         int& r0) {
  int it = item;
  si = s_lo;
  while (si < s_hi - 1 && it >= a.seg[si].rows / NR) { it -= a.seg[si].rows / NR; ++si; }
  r0 = it * NR;
  const QkvSeg& sg = a.seg[si];
#pragma unroll
  for (int r = 0; r < NR; ++r) R[r] = row_ptr(sg.base, sg.P, (unsigned)(r0 + r));
}

template <int QT, int NR, int U, int BLOCK>
__device__ __forceinline__ void qkv_run(const QkvLaunch& a, int s_lo, int s_hi, int blk, int nblk, int pos,
                                        XPrologue<true, BLOCK>& xp, int8_t* xq, float* xd, float* red) {
  const int wave = wave_id(), lane = threadIdx.x & 63;
  int total = 0;
  for (int i = s_lo; i < s_hi; ++i) total += a.seg[i].rows / NR;
  const int nchunks = a.K >> 5;
  const int hd = a.head_dim;
  constexpr int WPB = BLOCK / 64;
  // one-CU blocks (BLOCK 1024): contiguous per-block item ranges (equal bytes per CU)
  int stride, item, item_end;
  if constexpr (BLOCK == 1024) {
    const int per = (total + nblk - 1) / nblk;
    const int b0 = min(total, blk * per);
    item = b0 + wave;
    stride = WPB;
    item_end = min(total, b0 + per);
  } else {
    stride = nblk * WPB;
    item = blk * WPB + wave;
    item_end = total;
  }
  RowPtr R[NR];
  int si = s_lo, r0 = 0;
  WStream<QT, NR, U> ws;
  float2 cs = make_float2(1.f, 0.f);
  auto rope_of = [&](int r) { return a.rope[(size_t)pos * (hd >> 1) + ((r % hd) >> 1)]; };
  {  // unconditional (clamped item): no control-flow join between these loads and finish()'s x wait
    qkv_item<QT, NR>(a, s_lo, s_hi, min(item, total - 1), R, si, r0);
    ws.load(R, 0, nchunks, lane);
    if (lane < NR && a.seg[si].kind < 2) cs = rope_of(r0 + lane);
  }
  const float xs = xp.finish(a.x, a.norm_w, a.eps, a.K, xq, xd, red);
  while (item < item_end) {
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
    ws.finish_rows(R, nchunks, xq, xd, acc, lane);
    const int csi = si, cr0 = r0;
    const float2 ccs = cs;
    const int next = item + stride;
    if (next < item_end) {
      qkv_item<QT, NR>(a, s_lo, s_hi, next, R, si, r0);
      ws.load(R, 0, nchunks, lane);
      if (lane < NR && a.seg[si].kind < 2) cs = rope_of(r0 + lane);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] *= xs;
    float v = reduce_rows<NR>(acc, lane);
    const float partner = __shfl_xor(v, 1);
    const int kind = a.seg[csi].kind;
    if (lane < NR) {
      const int r = cr0 + lane;
      const int dd = r % hd;
      if (kind < 2) v = (lane & 1) ? partner * ccs.y + v * ccs.x : v * ccs.x - partner * ccs.y;
      if (kind == 0) {
        a.q_out[r] = v;
      } else {
        __half* c = (kind == 1 ? a.k_cache : a.v_cache) + ((size_t)(r / hd) * a.n_ctx + pos) * hd + dd;
        *c = __float2half(v);
      }
    }
    item = next;
  }
}

template <int QT0, int NR0, int U0, int QT1, int NR1, int U1, bool TWO, int BLOCK = 256>
__global__ __launch_bounds__(BLOCK) void gemv_qkv_kernel(QkvLaunch a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + a.K);
  float* red = xd + (a.K >> 5);
  // the prologue's kernarg fields in one scalar batch (as gemv_body's)
  asm volatile("" ::"s"(a.x), "s"(a.norm_w), "s"(a.K), "s"(a.pos), "s"(a.nseg), "s"(a.g1), "s"(a.blocks0),
               "s"(a.seg[0].base), "s"(a.seg[1].base), "s"(a.seg[2].base), "s"(a.seg[0].rows), "s"(a.seg[1].rows),
               "s"(a.seg[2].rows), "s"(a.seg[0].P.s0), "s"(a.seg[1].P.s0), "s"(a.seg[2].P.s0));
  const int pos = *a.pos;
  XPrologue<true, BLOCK> xp;   // QKV always follows the attention RMSNorm
  xp.load(a.x, a.norm_w, a.K);
  if (!TWO || (int)blockIdx.x < a.blocks0) {
    qkv_run<QT0, NR0, U0, BLOCK>(a, 0, a.g1, blockIdx.x, TWO ? a.blocks0 : gridDim.x, pos, xp, xq, xd, red);
  } else if constexpr (TWO) {
    qkv_run<QT1, NR1, U1, BLOCK>(a, a.g1, a.nseg, blockIdx.x - a.blocks0, gridDim.x - a.blocks0, pos, xp, xq, xd,
                                 red);
  }
}

static size_t qkv_lds(int K) { return K + (K / 32) * 4 + 128; }

template <int QT>
static void launch_qkv1(QkvLaunch L, int rows, hipStream_t s) {
  const GemvCfg c = pick_cfg(QT, rows, L.K >> 5, 2);
  const size_t lds = qkv_lds(L.K);
  L.g1 = L.nseg;
  L.blocks0 = 0;
  LFK_NRU_DISPATCH(c.nr, c.u, ({
    if constexpr (NR >= 2 && NR * U <= 4) {
      if (gemv_early(L.K > 4096 ? EC_QKV_LONG : EC_QKV)) {
        auto k = gemv_qkv_kernel<QT, NR, U, QT, NR, U, false, 1024>;
        const size_t l = std::max(lds, kOnePerCuLds);
        hipLaunchKernelGGL(k, gemv_grid(k, l, rows / NR, 1024), dim3(1024), l, s, L);
        return;
      }
    }
    if constexpr (NR >= 2 && !((QT == T_F32 || QT == T_F16) && NR * U > 4)) {
      auto k = gemv_qkv_kernel<QT, NR, U, QT, NR, U, false>;
      hipLaunchKernelGGL(k, gemv_grid(k, lds, rows / NR), dim3(256), lds, s, L);
    } else {
      throw std::runtime_error("gemv_qkv: bad config");
    }
  }));
}

// two type runs in one launch: (2 rows, 2 passes) items for the first run and
// (2 rows, 1 pass) for the second (keeps the combined kernel near 128 VGPRs)
template <int QT0, int QT1>
static void launch_qkv2(QkvLaunch L, int rows0, int rows1, hipStream_t s) {
  const double b0 = (double)qbytes(QT0, rows0, L.K), b1 = (double)qbytes(QT1, rows1, L.K);
  const int items = rows0 / 2 + rows1 / 2;
  if (gemv_early(L.K > 4096 ? EC_QKV_LONG : EC_QKV)) {
    auto k = gemv_qkv_kernel<QT0, 2, 2, QT1, 2, 1, true, 1024>;
    const size_t l = std::max(qkv_lds(L.K), kOnePerCuLds);
    const int nb = (int)gemv_grid(k, l, items, 1024).x;
    L.blocks0 = std::min(nb - 1, std::max(1, (int)std::lround(nb * b0 / (b0 + b1))));
    hipLaunchKernelGGL(k, dim3(nb), dim3(1024), l, s, L);
    return;
  }
  const size_t lds = qkv_lds(L.K);
  auto k = gemv_qkv_kernel<QT0, 2, 2, QT1, 2, 1, true>;
  const int nb = (int)gemv_grid(k, lds, items).x;
  L.blocks0 = std::min(nb - 1, std::max(1, (int)std::lround(nb * b0 / (b0 + b1))));
  hipLaunchKernelGGL(k, dim3(nb), dim3(256), lds, s, L);
}

void gemv_qkv(const QkvArgs& a, hipStream_t s) {
  const int K = a.wq.K;
  if (K % 32 || a.wk.K != K || a.wv.K != K) throw std::runtime_error("gemv_qkv: K mismatch");
  if (!a.norm_w) throw std::runtime_error("gemv_qkv: the attention RMSNorm weight is required");
  if (a.wq.rows % 4 || a.wk.rows % 4 || a.wv.rows % 4) throw std::runtime_error("gemv_qkv: rows must be multiples of 4");
  const QMat* m[3] = {&a.wq, &a.wk, &a.wv};
  QkvLaunch L{};
  L.K = K; L.x = a.x; L.norm_w = a.norm_w; L.eps = a.eps; L.q_out = a.q_out; L.k_cache = a.k_cache;
  L.v_cache = a.v_cache; L.n_ctx = a.n_ctx; L.head_dim = a.head_dim; L.pos = a.pos; L.rope = a.rope;
  // runs of equal type
  int run_start[3], run_type[3], nrun = 0;
  for (int i = 0; i < 3; ++i) {
    if (i == 0 || m[i]->type != m[i - 1]->type) { run_start[nrun] = i; run_type[nrun] = m[i]->type; ++nrun; }
  }
  for (int i = 0; i < 3; ++i) L.seg[i] = QkvSeg{m[i]->base, m[i]->P, m[i]->rows, i};
  L.nseg = 3;
  auto rows_of = [&](int lo, int hi) { int r = 0; for (int i = lo; i < hi; ++i) r += m[i]->rows; return r; };
  if (nrun == 1) {
    switch (run_type[0]) {
      case T_Q4_K: launch_qkv1<T_Q4_K>(L, rows_of(0, 3), s); return;
      case T_Q5_K: launch_qkv1<T_Q5_K>(L, rows_of(0, 3), s); return;
      case T_Q6_K: launch_qkv1<T_Q6_K>(L, rows_of(0, 3), s); return;
      case T_Q8_0: launch_qkv1<T_Q8_0>(L, rows_of(0, 3), s); return;
      case T_F16: launch_qkv1<T_F16>(L, rows_of(0, 3), s); return;
      case T_F32: launch_qkv1<T_F32>(L, rows_of(0, 3), s); return;
      default: throw std::runtime_error("gemv_qkv: unsupported type");
    }
  }
  if (nrun == 2) {
    L.g1 = run_start[1];
    const int r0 = rows_of(0, L.g1), r1 = rows_of(L.g1, 3);
    const int t0 = run_type[0], t1 = run_type[1];
    if (t0 == T_Q4_K && t1 == T_Q6_K) return launch_qkv2<T_Q4_K, T_Q6_K>(L, r0, r1, s);
    if (t0 == T_Q4_K && t1 == T_Q5_K) return launch_qkv2<T_Q4_K, T_Q5_K>(L, r0, r1, s);
    if (t0 == T_Q4_K && t1 == T_Q8_0) return launch_qkv2<T_Q4_K, T_Q8_0>(L, r0, r1, s);
    if (t0 == T_Q5_K && t1 == T_Q6_K) return launch_qkv2<T_Q5_K, T_Q6_K>(L, r0, r1, s);
    if (t0 == T_Q6_K && t1 == T_Q4_K) return launch_qkv2<T_Q6_K, T_Q4_K>(L, r0, r1, s);
  }
  // any other mix: one launch per segment
  for (int i = 0; i < 3; ++i) {
    QkvLaunch Li = L;
    Li.seg[0] = L.seg[i];
    Li.nseg = 1;
    switch (m[i]->type) {
      case T_Q4_K: launch_qkv1<T_Q4_K>(Li, m[i]->rows, s); break;
      case T_Q5_K: launch_qkv1<T_Q5_K>(Li, m[i]->rows, s); break;
      case T_Q6_K: launch_qkv1<T_Q6_K>(Li, m[i]->rows, s); break;
      case T_Q8_0: launch_qkv1<T_Q8_0>(Li, m[i]->rows, s); break;
      case T_F16: launch_qkv1<T_F16>(Li, m[i]->rows, s); break;
      case T_F32: launch_qkv1<T_F32>(Li, m[i]->rows, s); break;
      default: throw std::runtime_error("gemv_qkv: unsupported type");
    }
  }
}

// ------------------------------------------------------------------ MoE down projection
template <int QT>
__global__ __launch_bounds__(256) void gemv_moe_down_kernel(MoeDownArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NR = 2;
  const int K = a.w.K;
  int8_t* xq = reinterpret_cast<int8_t*>(smem);
  float* xd = reinterpret_cast<float*>(smem + (size_t)a.n_slots * K);
  float* red = xd + (size_t)a.n_slots * (K >> 5);
  for (int s = 0; s < a.n_slots; ++s)
    quantize_x<false>(a.h + (size_t)s * K, nullptr, 0.f, K, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), red);
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int nchunks = K >> 5;
  const int total = (a.w.rows + NR - 1) / NR;
  for (int item = blockIdx.x * 4 + wave; item < total; item += gridDim.x * 4) {
    const int r0 = item * NR;
    float tot[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) tot[r] = 0.f;
    for (int s = 0; s < a.n_slots; ++s) {
      const uint8_t* base = a.w.base + (size_t)a.expert_ids[s] * a.w.expert_stride;
      RowPtr R[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) R[r] = row_ptr(base, a.w.P, (unsigned)min(r0 + r, a.w.rows - 1));
      float acc[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[r] = 0.f;
      WStream<QT, NR, (QT == T_F32 ? 1 : 2)> wstr;
      wstr.load(R, 0, nchunks, lane);
      wstr.finish_rows(R, nchunks, xq + (size_t)s * K, xd + (size_t)s * (K >> 5), acc, lane);
      const float ws = a.expert_w[s];
#pragma unroll
      for (int r = 0; r < NR; ++r) tot[r] += ws * acc[r];
    }
    const float v = reduce_rows<NR>(tot, lane);
    if (lane < NR && r0 + lane < a.w.rows) a.out[r0 + lane] += v;
  }
}

void gemv_moe_down(const MoeDownArgs& a, hipStream_t s) {
  if (moe_down_splitk(a, s)) return;  // the split-K form where its types / shapes allow
  const int K = a.w.K;
  const size_t lds = (size_t)a.n_slots * (K + (K / 32) * 4) + 64;
  dim3 grid(grid_for((a.w.rows + 1) / 2)), block(256);
  switch (a.w.type) {
    case T_Q4_K: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q4_K>, grid, block, lds, s, a); break;
    case T_Q5_K: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q5_K>, grid, block, lds, s, a); break;
    case T_Q6_K: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q6_K>, grid, block, lds, s, a); break;
    case T_Q8_0: hipLaunchKernelGGL(gemv_moe_down_kernel<T_Q8_0>, grid, block, lds, s, a); break;
    case T_F16: hipLaunchKernelGGL(gemv_moe_down_kernel<T_F16>, grid, block, lds, s, a); break;
    case T_F32: hipLaunchKernelGGL(gemv_moe_down_kernel<T_F32>, grid, block, lds, s, a); break;
    default: throw std::runtime_error("moe_down: unsupported type");
  }
}

// ------------------------------------------------------------------ MoE router (one wave)
__global__ void moe_route_kernel(const float* logits, int E, int k, int* ids, float* w) {
  const int lane = threadIdx.x;
  float v = lane < E ? logits[lane] : -INFINITY;
  const float m = wave_max(v);
  float p = lane < E ? __expf(v - m) : 0.f;
  const float sum = wave_sum(p);
  p /= sum;
  float sel_sum = 0.f, my_w = 0.f;
  int my_id = 0;
  float taken = lane < E ? p : -1.f;
  for (int j = 0; j < k; ++j) {
    // arg-max with the lowest index on ties (matches a stable descending sort)
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
  if (lane < k) {
    ids[lane] = my_id;
    w[lane] = my_w / sel_sum;
  }
}

void moe_route(const float* logits, int n_expert, int k, int* ids, float* w, hipStream_t s) {
  if (n_expert > 64 || k > n_expert) throw std::runtime_error("moe_route: n_expert must be <= 64");
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(64), 0, s, logits, n_expert, k, ids, w);
}

}  // namespace lfk
