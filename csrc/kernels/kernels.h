// Host-side launch interface of the gfx950 kernels. Every launcher is
// asynchronous on the given stream, does no allocation and no host sync, and
// reads run-time scalars (position, KV length, sampled token) from device
// memory - so a whole decode step can be captured into one hipGraph and
// replayed unchanged.
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../common.h"

namespace lfk {

// ---------------------------------------------------------------- weights
struct QMat {
  const uint8_t* base = nullptr;
  int type = 0;
  int rows = 0;  // rows of ONE matrix (one expert)
  int K = 0;
  Planes P{};
  size_t expert_stride = 0;  // bytes between experts (0 = not an expert tensor)
};

QMat make_qmat(const void* base, int type, int rows, int K, size_t expert_stride = 0);

// Bytes spanned by one (non-expert) planar matrix: the end of its last non-empty plane.
inline size_t qmat_bytes(const QMat& m) {
  const size_t R = (size_t)m.rows;
  size_t e = m.P.p0 + R * m.P.s0;
  if (m.P.s1) e = m.P.p1 + R * m.P.s1 > e ? m.P.p1 + R * m.P.s1 : e;
  if (m.P.s2) e = m.P.p2 + R * m.P.s2 > e ? m.P.p2 + R * m.P.s2 : e;
  if (m.P.s3) e = m.P.p3 + R * m.P.s3 > e ? m.P.p3 + R * m.P.s3 : e;
  return e;
}

// ---------------------------------------------------------------- GEMV (decode, T = 1)
enum GemvEpi : int {
  EPI_STORE = 0,   // out[row] = acc
  EPI_ADD = 1,     // out[row] += acc            (residual, in place)
  EPI_SWIGLU = 2,  // out[f] = silu(acc_gate)*acc_up ; W = gate/up interleaved in 32-row groups
};

// peer receive regions of the tensor-parallel collectives (p2p_allreduce.hip, runtime/p2p.cpp)
static constexpr int kP2PMaxRanks = 8;
static constexpr int kP2PMaxBlocks = 64;
// fault[p][r]: rank r's fault code as stored in rank p's region (0 = none). A rank whose wait
// times out stores its code into EVERY rank's region, and every wait polls its own region's words
// between spins: the first fault poisons the group - no rank sits out its own 20 s bound, and
// every rank's host (the leader's included) sees who failed (P2PComm::fault_report)
struct P2PPeers {
  float* data[kP2PMaxRanks] = {};
  int* fault[kP2PMaxRanks] = {};
};

#ifdef __HIPCC__
__device__ __forceinline__ void p2p_raise(const P2PPeers& pe, int W, int R, int code) {
#pragma unroll
  for (int p = 0; p < kP2PMaxRanks; ++p)
    if (p < W) __hip_atomic_store(pe.fault[p] + R, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool p2p_poisoned(const P2PPeers& pe, int W, int R) {
  int any = 0;
#pragma unroll
  for (int p = 0; p < kP2PMaxRanks; ++p)
    if (p < W) any |= __hip_atomic_load(pe.fault[R] + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return any != 0;
}
#endif

struct GemvArgs {
  QMat w;
  const float* x = nullptr;       // [K] f32 activation
  const float* norm_w = nullptr;  // optional RMSNorm weight (fused into the prologue)
  float eps = 1e-5f;
  float* out = nullptr;
  int n_out = 0;                   // outputs per slot (rows, or features for SWIGLU)
  int n_slots = 1;                 // MoE: experts used per token
  const int* expert_ids = nullptr; // [n_slots] expert index per slot (device)
  int out_slot_stride = 0;
  // routed SwiGLU (the single-row MoE gate/up, K = 4 x 1024): every block computes the f32 router
  // itself - RMSNorm'd x . route_w^T, softmax, top-k - in place of reading expert_ids (one launch
  // and one dependent boundary less per MoE layer); block 0 writes the picks for the down
  // projection (route_ids / route_wts) and the logits (route_logits, optional)
  const float* route_w = nullptr;  // [route_E][K] f32 router
  int route_E = 0, route_k = 0;
  int* route_ids = nullptr;
  float* route_wts = nullptr;
  float* route_logits = nullptr;
  const float* resid = nullptr;    // EPI_STORE: out = acc + resid (TP rank 0 residual)
  int debug = 0;                   // microbenchmarks only: 1 = skip the x prologue, 2 = prologue only, 3 = weights after it
  long long* dbg_clk = nullptr;    // microbenchmarks only: per-block timeline [grid][5] (instrumented build)
  // in-flight producer (the decode attention of the same launch, attn_wo1): a block issues its
  // first item's weights, waits until wait[0 .. wait_cnt) >= wait_n (sc1 poll) and loads x with
  // sc1 loads; a timed-out wait sets *wait_err (host-mapped)
  const int* wait = nullptr;
  int wait_cnt = 0, wait_n = 0;
  int* wait_err = nullptr;
  // tensor-parallel all-reduce in the epilogue (EPI_STORE, the row-parallel Wo / down of a TP
  // decode step): each item's rows go to every rank as {value, epoch} granules (the fused area
  // of the P2P regions: tp_peers, granule tp_off + row of slot (parity, rank), tp_stride per
  // slot), the item waits for its rows from every rank and writes out[row] = resid[row] + the
  // rank-order sum. tp_epochs: one word per item (local, zero-initialised).
  P2PPeers tp_peers;
  int tp_world = 0, tp_rank = 0, tp_stride = 0, tp_off = 0;
  int* tp_epochs = nullptr;
  int* tp_err = nullptr;
  // grid cap: 1/grid_div of the resident blocks (TP ranks sharing one GPU: every rank's grid of
  // a waiting epilogue must be resident at once)
  int grid_div = 1;
};
void gemv(const GemvArgs& a, int epi, hipStream_t s);

// Batched decode projection on MFMA (bmm.hip): out[b][row] += W xh[b] for B <= 16 rows
// (split-K atomics: `out` holds the residual or zeros). xh rows come from bprep: f16, the
// k order inside each 4-group swizzled (0, 2, 1, 3) to match the dequantised A fragments.
static constexpr int kBmmMaxRows = 16;
struct BmmArgs {
  QMat w;                          // base = tile16 copy (t16_repack); type / rows / K as the matrix
  const __half* xh = nullptr;
  int ldh = 0;                     // halves between rows of xh (multiple of 8)
  float* out = nullptr;
  int ldo = 0;
  int n_out = 0;                   // rows of W
  int B = 0;
  int kparts = 1, spp = 1;         // set by the launcher (K parts, 256-k steps per part)
  // optional further matrices of the same type and K over the same xh (one launch for Q|K|V):
  // segment i > 0 uses seg_base[i], seg_rows[i], seg_out[i] (ldo shared)
  int nseg = 1;
  const uint8_t* seg_base[3] = {};
  int seg_rows[3] = {};
  float* seg_out[3] = {};
  // in-launch chain (bmm_ffn_chain: the SwiGLU gate/up and the down projection in ONE launch): the
  // producer run (chain_role 1) stores each finished tile's f16 outputs write-through and counts the
  // tile in chain_cnt[tile / chain_tpp]; the consumer run (2) issues its first weight steps, waits
  // until chain_cnt[its K part] holds all of that part's producer tiles, then stages its x with
  // L2-bypassing loads. Consumer blocks come after every producer block in the grid and a CU holds
  // one block of either (LDS), so a consumer only ever waits for blocks already running or done.
  int chain_role = 0;
  int* chain_cnt = nullptr;        // zeroed before the launch (per layer: the step's first kernel)
  int chain_tpp = 0;               // producer tiles per counter (= the consumer's K part / 8 features)
  int chain_tiles = 0;             // producer tiles in all
  int* chain_err = nullptr;        // host-mapped: a consumer's bounded wait timed out
  int chain_poll = 0;              // consumer poll interval: s_sleep units (64 clocks) between polls
  int chain_staged = 0;            // consumer: producer blocks that must have staged their x first
  int chain_wo = 0;                // kChainWaitWo: Wo blocks that must be done before the x staging
  int debug = 0;                   // microbenchmarks only: 1 = weight stream only (bmm_kernel); wave-owned
                                   // kernels: 2 = exit at entry, 3 = no epilogue writes, 4 = weight stream only,
                                   // 5 = x staging + weights, 6 = weights + MFMA, 7 = 6 without the
                                   // dequantisation (tools/boundary_bench.py)
  // Q|K|V epilogue (one K part only, see bmm_qkv_fits): instead of accumulating into `out`,
  // segment kinds seg_kind[i] (0 = Q, 1 = K, 2 = V) are finished in the epilogue - RoPE on
  // adjacent pairs for Q and K, Q rows to q_out[b][row], K / V rows as f16 into the slot
  // caches at the row's position (the batched rope_kv_prefill folded in)
  struct Qkv {
    int kind[3] = {0, 1, 2};
    float* q_out = nullptr;
    int q_ld = 0;
    __half* k_cache = nullptr;     // layer base of slot 0; + slot * slot_stride
    __half* v_cache = nullptr;
    size_t slot_stride = 0;
    int n_ctx = 0, head_dim = 0;
    const int* pos = nullptr;      // [B] position of each row
    const int* slots = nullptr;    // [B] KV slot of each row
    const float2* rope = nullptr;  // [n_ctx][head_dim / 2]
  } qkv;
  bool qkv_epi = false;
  // SwiGLU epilogue (gate/up, one K part, see bmm_qkv_fits): the tile16 copy is the SwiGLU
  // form (t16_repack swiglu = true): tile t holds the gate rows of features 8t .. 8t+7, then
  // their up rows, so every tile finishes its own features - silu(gate) * up as f16 in bmm's
  // 4-group k order to h_out[b * ldh_out + feature], the down projection's input - instead of
  // accumulating into `out` (no zeroed pre-activation buffer, no SwiGLU prep). Tiles are
  // split over the blocks in per-CU-balanced contiguous ranges (see bmm.hip).
  __half* h_out = nullptr;
  int ldh_out = 0;
  bool swiglu_epi = false;
  int tile_groups = 1;             // SwiGLU tile split: blocks b, b + tile_groups share a CU's quota (launcher)
  // RMSNorm folded into the x staging (one K part, K % 2048 == 0, see bmm_norm_fits): the
  // block reads the fp32 rows xf[b * ldxf + k], stages f16(x * norm_w) and the row sums of
  // squares; the epilogue scales each column by rsqrt(mean + eps) (xh is not read)
  const float* xf = nullptr;
  int ldxf = 0;
  const float* norm_w = nullptr;
  float eps = 1e-5f;
  bool store_out = false;          // plain epilogue: out = result (default: out += result)
  // MoE experts as ONE matrix (the batched decode FFN): gate/up = the experts' SwiGLU tile16
  // copies stacked (tile t belongs to expert t / tiles_per_expert), down = the experts' down
  // rows concatenated along K (256-k step s to expert s / steps_per_expert) over the stacked
  // SwiGLU output. ew [B][ew_ld] holds each row's routing weight per expert (0 = not routed):
  // the SwiGLU epilogue scales row b of expert e's features by ew[b][e] (so unrouted rows
  // contribute exactly 0 through the down projection) and the down blocks whose K part
  // covers no expert with a routed row exit before loading a byte.
  const float* ew = nullptr;
  int ew_ld = 0, tiles_per_expert = 0, steps_per_expert = 0;
  bool one_part = false;           // plain projection as one K part (8-wave blocks, no atomics)
  long long* dbg_clk = nullptr;    // microbenchmarks only: per-block wall_clock64 stamps [grid][8]
  int nb1 = 0;                     // bmm_qkv2: blocks of the first run; split-K Q|K|V: first group of run B
  // Split-K Q|K|V (qkv_sk, batched decode, B <= 8): segments 0..nseg-1 (Q, K, V rows; kinds in
  // qkv.kind) are summed over K parts into seg_out (atomic adds into zeroed rows, ldo shared),
  // Q and K partial tiles rotated by RoPE first (a rotation is linear, so the sum of rotated
  // partials is the rotated sum). The RMSNorm is folded in as: x staged as f16(x * norm_w) per
  // K part from xf, each row's partial sum of squares over the part added to ss_out[b] (by the
  // part's first tile group only); the consumer (the batched attention) scales row b by
  // rsqrt(ss_out[b] / K + eps). Segments [seg_split, nseg) are of the launch's second weight type.
  bool qkv_sk = false;
  float* ss_out = nullptr;
  int seg_split = 1;
  int type2 = 0;                   // weight type of segments [seg_split, nseg)
  int tpg = 8;                    // tiles per (K part) block group (set by the launcher)
  // side job of the split-K launches: zero [zero, zero + zero_n) floats (zero_n % 4 == 0)
  float* zero = nullptr;
  int zero_n = 0;
};
// split-K Q|K|V (BmmArgs::qkv_sk): false = unsupported shape / type mix (caller: one-part path)
bool bmm_qkv_sk_supported(int tq, int tk, int tv, int K, int B);
bool bmm_supported(int type, int K);
bool bmm_qkv_fits(int K, int B);   // the Q|K|V epilogue needs one K part (x slice in LDS)
bool bmm_norm_fits(int K, int B);  // one K part + the folded RMSNorm's staging shape
void bmm(const BmmArgs& a, hipStream_t s);
// two one-part Q|K|V runs of different weight types (Q|K Q4_K + V Q6_K / Q5_K: the bumped
// layers of the K-quant mixes) in one launch; false = unsupported pair or shape (caller
// launches them one by one)
// The dense SwiGLU gate/up (gu, swiglu_epi) and the down projection over its output (dn) in ONE
// launch with a per-K-part in-launch hand-off (BmmArgs::chain_*). cnt: kChainInts ints, zero
// before the launch (kChainXcds counters per K part, each on a 128-B line of its own); err: host-mapped
// word set if a consumer's bounded wait timed out.
// Each K part's count is sharded over the XCDs (the producer's XCC id picks the shard; the
// consumer sums the 8): same-address atomics serialise at ~12 ns each under load.
constexpr int kChainStride = 32, kChainXcds = 8, kChainMaxParts = 16;
constexpr int kChainInts = kChainStride * kChainXcds * kChainMaxParts;
constexpr int kChainStagedPart = kChainMaxParts - 1;  // the last part's counters: producers' x staged
constexpr int kChainWoPart = kChainMaxParts - 2;      // ... the one before: Wo blocks done (bmm_wo_ffn_chain)
// BmmArgs::chain_role bits
constexpr int kChainProduce = 1, kChainConsume = 2, kChainWoDone = 4, kChainWaitWo = 8;
bool bmm_ffn_chain_supported(const BmmArgs& gu, const BmmArgs& dn);
void bmm_ffn_chain(const BmmArgs& gu, const BmmArgs& dn, int* cnt, int* err, hipStream_t s);
// ... with the Wo projection (wo: split-K into the residual rows gu stages) in the same launch: the
// gate/up blocks issue their first weight steps, wait until every Wo block is done, then stage x
bool bmm_wo_ffn_chain_supported(const BmmArgs& wo, const BmmArgs& gu, const BmmArgs& dn);
void bmm_wo_ffn_chain(const BmmArgs& wo, const BmmArgs& gu, const BmmArgs& dn, int* cnt, int* err, hipStream_t s);
bool bmm_qkv2(const BmmArgs& a, const BmmArgs& b, hipStream_t s);
// the split-K Q|K|V leaves its sums un-RoPE'd (the batched attention rotates q and the new key:
// AttnDecodeArgs::rope) - the interleaved-step kernels, whose loop then loads weights only
bool bmm_qkv_sk_defers_rope();
// the batched path's weight copy: per 16-row tile and 256-k step one contiguous block
size_t t16_bytes(int type, int rows, int K);
// swiglu: `planar` is a gate/up matrix in 32-row gate / up groups (upload_gate_up); the copy
// regroups it per tile as 8 gate rows + the 8 up rows of the same features
void t16_repack(const QMat& planar, uint8_t* dst, hipStream_t s, bool swiglu = false);
// f32 rows -> bmm input: optional SwiGLU (x rows of 2K gate/up pre-activations, 32-feature
// interleaved groups), optional RMSNorm (* norm_w), f16 swizzled; also zeroes zero[0, zero_n)
struct BPrepArgs {
  const float* x = nullptr;
  int ldx = 0;
  bool swiglu = false;
  const float* norm_w = nullptr;
  float eps = 1e-5f;
  int K = 0, B = 0;
  __half* xh = nullptr;
  int ldh = 0;
  float* zero = nullptr;
  int zero_n = 0;
  int swiglu_group = 32;           // gate/up row groups of x: 32 (planar GEMV layout) or 8 (tile16 SwiGLU copy)
};
void bprep(const BPrepArgs& a, hipStream_t s);

// Fused QKV projection + RoPE (adjacent pairs) + KV-cache append.
struct QkvArgs {
  QMat wq, wk, wv;
  const float* x = nullptr;
  const float* norm_w = nullptr;
  float eps = 1e-5f;
  float* q_out = nullptr;          // [n_q] f32 (roped)
  __half* k_cache = nullptr;       // layer base, [n_kv_heads][n_ctx][head_dim]
  __half* v_cache = nullptr;
  int n_ctx = 0;
  int head_dim = 0;
  const int* pos = nullptr;        // device scalar: position of this token
  const float2* rope = nullptr;    // [n_ctx][head_dim/2] (cos, sin)
};
void gemv_qkv(const QkvArgs& a, hipStream_t s);

// MoE down projection: out[r] += sum_s w[s] * dot(W_{ids[s]}[r], h_s)
struct MoeDownArgs {
  QMat w;
  const float* h = nullptr;        // [n_slots][K]
  const int* expert_ids = nullptr;
  const float* expert_w = nullptr; // [n_slots]
  int n_slots = 2;
  float* out = nullptr;            // [rows]
};
void gemv_moe_down(const MoeDownArgs& a, hipStream_t s);
// split-K form (moe.hip), K-quant / Q8_0 experts; returns false if the shape/type is not covered
bool moe_down_splitk(const MoeDownArgs& a, hipStream_t s);
// decode router fused with the routing (F32 router weights, E <= 16): one launch
// (split over d into per-slice waves with a last-arriver sum it measured slower: 8.6 vs 7.7 us,
// the hand-off costing more than the one block's 144 KB read)
bool moe_router_fused_ok(int router_type, int E, int d);
// batched decode rows: RMSNorm(x_b) * w_norm -> f32 router -> softmax / top-k / renormalise
// per row, written DENSE: wd[b * ld + e] = the row's weight of expert e, 0 if not selected
void moe_router_rows(const float* x, int ldx, int B, const float* nw, float eps, const float* W, int d, int E, int k,
                     float* wd, int ld, hipStream_t s);
void moe_router_fused(const float* x, const float* nw, float eps, const float* W, int d, int E, int k, float* logits,
                      int* ids, float* w, hipStream_t s);

// Router: softmax over n_expert logits, top-k, renormalise -> ids / weights (device).
void moe_route(const float* logits, int n_expert, int k, int* ids, float* w, hipStream_t s);

// ---------------------------------------------------------------- tensor-parallel collectives
// One-shot push all-reduce / all-gather over peer memory (p2p_allreduce.hip). Rank p's
// receive region: data [2 slots][world][max_n + kP2PMaxBlocks] 8-byte granules {f32 value,
// u32 epoch} (max_n elements + one heartbeat per block; the `data` pointers address the region
// as floats, two per granule), then an unused flag area.
// Every launch runs exactly kP2PMaxBlocks blocks (the slot-reuse argument needs it).
struct P2PArgs {
  P2PPeers peers;                  // every rank's region as mapped in THIS process (own one included)
  const float* src = nullptr;      // [n] this rank's buffer
  float* dst = nullptr;            // all-reduce: [n] the sum; all-gather: [world][n]
  int n = 0, max_n = 0, rank = 0, world = 1;
  int stride = 0;                  // granules per (slot, rank): max_n + kP2PMaxBlocks (+ the fused area)
  int gather = 0;                  // 0: all-reduce (sum), 1: all-gather
  // all-reduce only: dst[i] += sum (instead of =), and src[i] is zeroed once pushed - the batched
  // row-parallel projections accumulate into a buffer that stays zero between launches, so no
  // copy / fill node seeds it per collective (and rank 0 needs no residual copy)
  int accumulate = 0;
  int* epochs = nullptr;           // [kP2PMaxBlocks] local, zero-initialised, advanced per launch
  int* err = nullptr;              // set on a timed-out wait
  // host-mapped mirror [kP2PMaxRanks] of this rank's fault words, refreshed by every launch: the
  // engine's per-step health check reads it with no copy (the sampler's all-gather runs every step)
  int* fault_h = nullptr;
};
void p2p_collective(const P2PArgs& a, hipStream_t s);

// ---------------------------------------------------------------- attention
// Decode: split-L flash decoding over chunks of 64 keys, GQA-packed.
struct AttnDecodeArgs {
  const float* q = nullptr;       // [n_head][hd]
  const __half* k_cache = nullptr;
  const __half* v_cache = nullptr;
  const int* pos = nullptr;       // KV length = *pos + 1
  int n_ctx = 0, n_head = 0, n_kv_head = 0, head_dim = 0;
  float scale = 1.f;
  float* part = nullptr;          // workspace [n_split][n_head][hd + 2]
  int* counters = nullptr;        // [n_kv_head] zero-initialised; each launch leaves them at 0
  float* out = nullptr;           // [n_head][hd]
  int debug_stop = 0;             // microbenchmarks only: 1..4 = exit after stage N (0 = full kernel)
  long long* dbg_clk = nullptr;   // microbenchmarks only: per-block wall_clock64 stamps [grid][16] (attention.hip)
  // optional: a second grid plane (blockIdx.z = 1) touches one dword per 128-B line of
  // [pf, pf + pf_bytes) so the next projection's weights are in the memory-side
  // cache when its GEMV starts (the attention blocks are latency bound and leave
  // HBM idle). pf_sink: a 4-B device word the touch result is conditionally stored to.
  // Up to 6 ranges, each spread over all touch blocks. A range is pf_nseg segments of
  // pf_bytes bytes, pf_seg_stride apart (nseg 1: one contiguous span).
  // batched decode (batch > 0): grid z = row b with query q + b*q_stride, KV slot
  // slots[b] (caches slots[b]*slot_stride halves in), length pos[b] + 1, partials
  // part + b*part_stride, split counters counters + 64*b, output out + b*out_stride.
  // No weight touch in this mode.
  int batch = 0;
  const int* slots = nullptr;
  size_t slot_stride = 0, q_stride = 0, out_stride = 0, part_stride = 0;
  // batched: also write the output as the next projection's bmm input (f16, bmm k swizzle)
  __half* out_h = nullptr;
  size_t out_h_stride = 0;
  // single row (attn_wo1): once kv head h's output is written (sc1 stores), done[h] += 1 (agent
  // scope) - the Wo GEMV planes of the same launch (GemvArgs::wait) poll it
  int* done = nullptr;
  // batched, split-K Q|K|V (BmmArgs::qkv_sk): q / k / v of row b are the RoPE'd but unnormalised
  // sums qkv_raw[b * qkv_ld + ...] (q at 0, k at k_off, v at v_off), the row's RMSNorm scale is
  // rsqrt(ss[b] * inv_k + eps); the block holding the new position scales its k / v, writes them
  // to the caches and uses them in place of the (not yet written) cache rows
  const float* qkv_raw = nullptr;
  size_t qkv_ld = 0, k_off = 0, v_off = 0;
  const float* ss = nullptr;
  float inv_k = 0.f, eps = 1e-5f;
  // split-K Q|K|V with its RoPE deferred (bmm_qkv_sk_defers_rope): q and the new key are rotated
  // here by pos * rope_freq[pair] (fp32; null: the sums arrive RoPE'd)
  const float* rope_freq = nullptr;
  static constexpr int kTouchRanges = 6;
  const uint8_t* pf[kTouchRanges] = {};
  size_t pf_bytes[kTouchRanges] = {};
  int pf_nseg[kTouchRanges] = {1, 1, 1, 1, 1, 1};
  size_t pf_seg_stride[kTouchRanges] = {};
  int* pf_sink = nullptr;
};
void attn_decode(const AttnDecodeArgs& a, hipStream_t s);
// The single-row decode attention and its Wo GEMV (split-K into the residual) in ONE launch
// (gemv.hip): `wo` waits for the attention's done counters (wo.wait == a.done, one per kv head).
// False: shape / weight type not covered.
bool attn_wo1(const AttnDecodeArgs& a, const GemvArgs& wo, hipStream_t s);
size_t attn_decode_workspace_floats(int n_ctx, int n_head, int head_dim);

// Prefill: causal attention of T queries at positions pos0.. over the cache.
struct AttnPrefillArgs {
  const float* q = nullptr;       // [T][n_head][hd] (roped)
  const __half* k_cache = nullptr;
  const __half* v_cache = nullptr;
  int T = 0, pos0 = 0, n_ctx = 0, n_head = 0, n_kv_head = 0, head_dim = 0;
  float scale = 1.f;
  float* out = nullptr;           // [T][n_head][hd] f32, or
  __hip_bfloat16* out_bf16 = nullptr;  // bf16 (the Wo GEMM's input; MFMA path only)
  __half* out_h = nullptr;        // or f16 in bmm's 4-group k order (gemm_t16's input; MFMA path)
  int out_stride = 0;
  // packed prompts in ONE launch (MFMA path; a joint admission's pieces): piece i = q / out rows
  // [pc_row, pc_row + pc_n) at positions pc_pos.., against KV slot pc_slot (caches + slot *
  // slot_stride halves); T / pos0 are then unused (grid z = pieces x head groups)
  static constexpr int kMaxPieces = 16;
  int n_pieces = 0;
  int pc_row[kMaxPieces] = {}, pc_n[kMaxPieces] = {}, pc_pos[kMaxPieces] = {}, pc_slot[kMaxPieces] = {};
  size_t slot_stride = 0;
};
void attn_prefill(const AttnPrefillArgs& a, hipStream_t s);

// ---------------------------------------------------------------- prefill GEMM (MFMA)
enum GemmEpi : int { GEMM_STORE = 0, GEMM_ADD = 1, GEMM_SWIGLU = 2 };
struct GemmArgs {
  QMat w;                          // [N][K] planar
  const __hip_bfloat16* x = nullptr;  // [T][K] bf16 (row stride K)
  int T = 0;
  float* out = nullptr;            // f32 [T][ldo] (STORE/ADD)
  __hip_bfloat16* out_bf16 = nullptr; // SWIGLU -> bf16 [T][N/2]
  int ldo = 0;
  const float* resid = nullptr;    // STORE: out = acc + resid[t][n] (TP rank 0)
  // grouped (MoE) form: rows [seg_dev[0], seg_dev[1]) of x / out, read on the device;
  // T is then only the launch bound (max rows) and rows_hint the expected count (split-K
  // sizing). Split-K STORE partials are atomically added: the caller pre-zeroes `out`.
  const int* seg_dev = nullptr;
  int rows_hint = 0;
  bool out_zeroed = false;         // STORE: the caller already zeroed `out` (no memset for split-K)
};
void gemm_dq(const GemmArgs& a, int epi, hipStream_t s);

// Prefill GEMM on the tile16 weight copy (bmm.hip): Y[T][N] = X[T][K] . W^T with X f16 in bmm's
// 4-group k order (rmsnorm_bf16(..., f16sw), attention prefill out_h, this kernel's SwiGLU
// epilogue) and W dequantised with bmm's f16 arithmetic into v_mfma_f32_16x16x32_f16 A
// fragments that serve 128 tokens each (the planar gemm_dq decodes to bf16 per 64-k step).
struct GemmT16Args {
  QMat w;                          // base = tile16 copy (the SwiGLU form for GEMM_SWIGLU)
  const __half* x = nullptr;       // [T][K] f16, bmm k order (row stride K)
  int T = 0;
  float* out = nullptr;            // f32 [T][ldo] (STORE / ADD)
  int ldo = 0;
  const float* resid = nullptr;    // STORE: out = acc + resid[t][n] (TP rank 0)
  bool out_zeroed = false;         // STORE: `out` already zeroed (no memset before split-K)
  __half* out_h = nullptr;         // SWIGLU: silu(gate) * up as f16 [T][ldh], bmm k order
  int ldh = 0;
  // grouped (MoE) form: rows [seg_dev[0], seg_dev[1]) of x / out / out_h, read on the device; T
  // is then only the launch bound and rows_hint the expected count (shape and split-K sizing;
  // split-K STORE partials are atomically added, so the caller pre-zeroes `out`)
  const int* seg_dev = nullptr;
  int rows_hint = 0;
  // a matrix inside a wider tile16 copy (the MoE down experts concatenated along K): bytes
  // between consecutive 16-row tiles (0: the matrix's own K / 256 steps) and its first 256-k
  // step inside each tile
  size_t tile_stride = 0;
  int step0 = 0;
  int cfg = 0;                     // block shape pin (waves * 1000 + tokens; tuning tools), 0: the measured rule
  // stacked matrices (Q|K|V in one launch): w.rows = every segment's rows, tiles [0, wseg_tiles[0])
  // from w.base, the next wseg_tiles[1] from wseg_base[1], the rest from wseg_base[2]; one type and
  // K; output column = stacked row (the segments' outputs adjacent in `out`)
  int nwseg = 1;
  const uint8_t* wseg_base[3] = {nullptr, nullptr, nullptr};
  int wseg_tiles[3] = {0, 0, 0};
};
void gemm_t16(const GemmT16Args& a, int epi, hipStream_t s);

// ---------------------------------------------------------------- MoE prefill (grouped experts)
// Device-side routing: per-expert row lists in ascending token order (moe.hip).
void moe_route_group(const float* logits, int T, int n_expert, int k, int* sel, float* selw, int* cnt_off, int* tok,
                     float* gw, int* pos, hipStream_t s);
void gather_rows_bf16(const __hip_bfloat16* src, const int* tok, int n_rows, int d, __hip_bfloat16* dst,
                      hipStream_t s);
void moe_scatter_add(float* acc, const float* y, const int* pos, const float* gw, int T, int k, int d, hipStream_t s);

// ---------------------------------------------------------------- elementwise / misc
// x[t][:] = dequant(token_embd[tokens[t]][:])
// (side job: zero [zero, zero + zero_n) ints)
void embed_rows(const QMat& emb, const int* tokens, int T, float* x, hipStream_t s, int* zero = nullptr,
                int zero_n = 0);
// y_bf16[t] = rmsnorm(x[t]) * w
// zero (optional): also zero rows [T][zero_ld] f32 (the next split-K GEMM's output)
// f16sw: write y as f16 in bmm's 4-group k order instead (gemm_t16's input; same 2-byte rows)
void rmsnorm_bf16(const float* x, const float* w, float eps, int T, int d, __hip_bfloat16* y, hipStream_t s,
                  float* zero = nullptr, int zero_ld = 0, bool f16sw = false);
// f32 activation [T][d] -> bf16 (for the next GEMM)
void to_bf16(const float* x, int n, __hip_bfloat16* y, hipStream_t s);
// prefill: rope q/k of QKV rows, write q (f32) and k/v to the caches at pos0+t.
// Batched decode (pos_arr != nullptr): row t is at position pos_arr[t] of KV slot
// slot_arr[t], whose caches start slot_arr[t] * slot_stride halves after k_cache / v_cache.
void rope_kv_prefill(const float* qkv, int T, int pos0, int n_q, int n_kv, int head_dim, int n_ctx,
                     const float2* rope, float* q_out, __half* k_cache, __half* v_cache, hipStream_t s,
                     const int* pos_arr = nullptr, const int* slot_arr = nullptr, size_t slot_stride = 0);
// batched decode: tok[b] / pos[b] = the current token / position of KV slot slots[b]
// (+ zero zero[i * zero_stride], i < zero_n: the step's in-launch chain counters)
void batch_gather(const int* slots, int B, const int* state, int* tok, int* pos, hipStream_t s, int* zero = nullptr,
                  int zero_n = 0, int zero_stride = 1);
// the same, and x[b] = the embedding of row b's token (one launch: the batched step's first)
void batch_gather_embed(const int* slots, int B, const int* state, int* tok, int* pos, const QMat& emb, float* x,
                        hipStream_t s, int* zero = nullptr, int zero_n = 0, int zero_stride = 1);
// out[i] = x[i] (+) ... small helpers
void add_inplace(float* x, const float* y, int n, hipStream_t s);
void set_i32(int* p, int v, hipStream_t s);
// microbenchmark: trivial kernel of a given launch shape (per-launch cost of the shape)
void launch_probe(int threads, int blocks, size_t lds, int iters, float* out, hipStream_t s);
// microbenchmark: out[0] = shader cycles, out[1] = wall ticks (100 MHz) of `iters` dependent FMAs
void clock_probe(long long* out, int iters, hipStream_t s);

// ---------------------------------------------------------------- sampling
// Sampling parameters live in DEVICE memory so a captured decode graph serves
// every request unchanged (they are written once per request, before replay).
static constexpr int kMaxLogitBias = 64;  // logit-bias entries applied by sampler stage 1
struct SamplerParamsDev {
  int top_k = 40;
  int last_n = 64;
  int greedy = 0;
  int n_bias = 0;                  // entries of bias_tok/bias_val in use (distinct tokens)
  float top_p = 0.95f, min_p = 0.05f, temp = 0.8f;
  float repeat_penalty = 1.1f, freq_penalty = 0.f, presence_penalty = 0.f;
  float tfs_z = 1.f, typical_p = 1.f;  // tail-free / locally-typical (1 = off)
  unsigned long long seed = 0;
  int bias_tok[kMaxLogitBias] = {};
  float bias_val[kMaxLogitBias] = {};
};
// Device state block (ints) shared by the decode kernels.
enum StateIdx : int { S_TOKEN = 0, S_POS = 1, S_STEP = 2, S_RING_LEN = 3, S_RING_HEAD = 4, S_NOUT = 5, S_NSTATE = 8 };

// Stage 1 writes, per row, one packed candidate block of sampler_cand_words(V_span) 4-byte
// words: [values nb*64 f32][global ids nb*64 i32][slice bounds nb][slice maxima nb]
// (nb = sampler_blocks(V_span)). Stage 2 reads `world` such blocks per row, laid out
// [world][rows][words] - under tensor parallelism each rank runs stage 1 on its vocabulary
// shard, the blocks are all-gathered (a few KB instead of the shard's logits) and every rank
// runs the identical stage 2 (same candidates, same RNG step -> the same token).
struct SamplerArgs {
  float* logits = nullptr;         // [V] this rank's logits; the penalty pass patches a copy in LDS
  int V = 0;                       // real logits in `logits` (this rank's shard)
  int vocab_off = 0;               // global id of logits[0] (tensor-parallel vocabulary shard)
  int V_glob = 0;                  // full vocabulary (0: V); sampled ids are clamped below it
  int V_span = 0;                  // stage-1 slices cover [0, V_span) (0: V); the same on every rank
  const SamplerParamsDev* p = nullptr;
  int* ring = nullptr;             // [64] penalty window ring (prompt + generated tokens)
  int* state = nullptr;            // [S_NSTATE]
  unsigned* cand = nullptr;        // stage-1 output [rows][sampler_cand_words(V)]
  const unsigned* cand_all = nullptr;  // stage-2 input [world][rows][words] (null: `cand`, world 1)
  int world = 1;
  long long* dbg_clk = nullptr;    // microbenchmarks only: stage-2 timeline stamps (instrumented build)
  int* out_tokens = nullptr;       // optional device ring of sampled tokens [out_cap]
  int out_cap = 0;
  int advance_pos = 1;             // also bump state.pos (decode) after sampling
  // batched (batch > 0): row b samples logits + b*logits_ld with the params / ring /
  // state of slot slots[b] (p + slot, ring + 64*slot, state + S_NSTATE*slot), its own
  // candidate block and writes its token to batch_out[b]
  int batch = 0;
  const int* slots = nullptr;
  size_t logits_ld = 0;
  int* batch_out = nullptr;
  // ... and to host-mapped pinned memory (the batch-step graph's token read-back: no copy node)
  int* batch_out_host = nullptr;
};
int sampler_blocks(int V);
size_t sampler_cand_words(int V);
void sample_stage1(const SamplerArgs& a, hipStream_t s);
void sample_stage2(const SamplerArgs& a, hipStream_t s);
void sample(const SamplerArgs& a, hipStream_t s);  // both stages (world 1)

// ---------------------------------------------------------------- synthetic fill
// Random valid quant blocks generated on device (for synthetic models without a file).
void fill_random_planar(uint8_t* base, int type, size_t rows, size_t K, float std, unsigned long long seed,
                        hipStream_t s);

}  // namespace lfk
