// Persistent decode step (pdecode.hip): ALL transformer layers of one batch-1
// decode token in ONE launch, one 512-thread workgroup per CU.
//
// Why (profiles/README.md, round 1): the five-launch-per-layer chain spent
// ~26 us of a 46 us Llama-3-8B layer in kernel boundaries, x prologues and
// launch ramps/tails while HBM idled; the weight stream could not cross a
// dependency edge. Here every CU owns a fixed slice of every projection and
// two loader waves per CU stream that CU's weights for the whole token into an
// LDS ring (global_load_lds, non-temporal) in consumption order, independent
// of the activations. Six consumer waves wait for activations at the
// dependency edges while the ring keeps filling, so the weight stream runs
// across every edge.
//
// Dataflow of one layer (u = CU, g = kv head = CU group of NCU/n_kv CUs):
//   HX  : every CU gathers x (q8 per 8 + sum of squares from its owner CU)
//   QKV : CU u: q rows [u*NQU..), k/v rows [u*NKU..) -> RoPE, f16 KV append,
//         publishes q/k/v to its group (HQKV)
//   ATT : split s of kv head g (CU (g, s)): keys [s*KPS, ..) of the cache
//         (the new key from HQKV), 4..8 query heads -> partial (o, m, l) (HATT)
//   MRG : one CU per query head merges the S partials -> q8 o_h (HO)
//   WO  : CU u: rows [u*NXU..) of Wo over all of o (HO gathered), residual x
//         rows owned by u -> publishes HX (ffn norm)
//   GU  : CU u: gate and up rows of features [u*NFU..) -> SwiGLU -> q8 h (HH)
//   DOWN: CU u: rows [u*NXU..) over all of h -> residual -> HX of layer l+1
// Hand-offs are 8-byte granules {tag = launch epoch, 32-bit value} written by
// ONE sc1 store and swept with sc1 loads until every tag matches
// (cdna_hip_programming.md Guideline 16, R2); every spin is bounded and sets
// an abort word that all waits observe.
#pragma once
#include "kernels.h"

namespace lfk {

// workgroup geometry (one per CU): loader waves stream the ring, consumer waves compute
static constexpr int kPdThreads = 512;
static constexpr int kPdLoaderWaves = 2;
static constexpr int kPdConsumerWaves = kPdThreads / 64 - kPdLoaderWaves;

enum PdStage : int { PD_Q = 0, PD_K = 1, PD_V = 2, PD_WO = 3, PD_GATE = 4, PD_UP = 5, PD_DOWN = 6 };

// One ring item: whole rows of one matrix slice of one CU. All CUs share the
// item table of a layer; CU u's copy starts at layer.wbase + u * layer.cu_bytes.
struct PdItem {
  uint32_t off;        // byte offset in the CU's layer span
  uint32_t row_bytes;  // bytes per row in the ring row format
  uint16_t dma_kb;     // 1-KiB LDS-DMA transfers (rounded up; the buffer is padded)
  uint16_t rows;
  uint16_t row0;       // first row index inside the stage's per-CU row list
  uint8_t stage;
  uint8_t type;
};

struct PdLayer {
  const uint8_t* wbase = nullptr;
  uint32_t cu_bytes = 0;
  int item0 = 0, nitems = 0;
  const float* attn_norm = nullptr;
  const float* ffn_norm = nullptr;
};

struct PDecodeArgs {
  const PdLayer* layers = nullptr;
  const PdItem* items = nullptr;
  int n_layer = 0;
  float* x = nullptr;                // [d] residual: in (embedding), out (last layer)
  __half* k_cache = nullptr;         // layer 0 base, [n_kv][n_ctx][hd] per layer
  __half* v_cache = nullptr;
  size_t kv_layer = 0;               // elements per layer
  const float2* rope = nullptr;      // [n_ctx][hd/2]
  const int* pos = nullptr;          // device: position of this token (KV length - 1)
  unsigned* epoch = nullptr;         // device: granule tag of this launch (CU 0 advances it at exit)
  unsigned long long* gran = nullptr;  // granule region of layer 0
  size_t gran_layer = 0;             // granules per layer
  int off_hx = 0, off_qkv = 0, off_att = 0, off_o = 0, off_hx2 = 0, off_hh = 0;  // per-layer offsets
  int d = 0, nq = 0, nkv = 0, hd = 0, F = 0, n_head = 0, n_kv_head = 0, n_ctx = 0;
  int ncu = 0, cpg = 0;              // CUs, CUs per kv head
  int nxu = 0, nqu = 0, nku = 0, nfu = 0;  // rows per CU: x/Wo/down, q, k (= v), ffn features
  int smax = 0;                      // attention splits per kv head (max)
  int nslot = 0, slot_bytes = 0;     // LDS ring
  int act_bytes = 0, part_floats = 0, res_rows = 0;  // LDS carve sizes
  float eps = 1e-5f, attn_scale = 1.f;
  int* err = nullptr;                // [0] error code, [1] abort flag (device)
  // debugging: when set, every layer's intermediates are stored at dbg + l * pd_dump_stride():
  // q (roped, unscaled) [nq] | k [nkv] | v [nkv] | attention output [nq] | x after Wo [d] |
  // SwiGLU output [F] | x after down [d]
  float* dbg = nullptr;
  // timeline: wall_clock64 stamps [ncu][n_layer][kPdStamps] (consumer stage ends, loader issue)
  long long* tl = nullptr;
  // item timeline of layer 2: [ncu][kPdItemStamps][8]: loader issue, -, consumer wait start,
  // item available, item released
  long long* tli = nullptr;
  // cycle accounting (LFK_PDECODE_ACCT=1): [ncu][16] shader-clock totals kept in registers and
  // stored once at the end (no memory traffic inside the step): consumer wave 0: 0 item code,
  // 1 waiting for ring items, 2 consumer barriers, 3 granule sweeps, 4 items, 5 attention,
  // 6 merge, 7 whole; loader wave 0: 8 blocked on free slots, 9 waiting for landings, 10 issue
  long long* acct = nullptr;
  // experiments only (LFK_PDECODE_DBG): 1 = consumers release ring items without computing,
  // 2 = the loader publishes items without loading them
  int dbg_mode = 0;
};
static constexpr int kPdStamps = 12;
static constexpr int kPdItemStamps = 48;

size_t pdecode_lds_bytes(const PDecodeArgs& a);
// every workgroup of the grid (one per CU) can be resident at once (host check)
bool pdecode_resident(const PDecodeArgs& a);
// a: host copy (launch geometry), a_dev: the same struct in device memory (what the kernel reads)
void pdecode(const PDecodeArgs& a, const PDecodeArgs* a_dev, hipStream_t s);
// copy rows_cu * ncu rows of a planar matrix into the ring row format: row i (source row
// map ? map[i] : i) goes to CU i / rows_cu, slot i % rows_cu of the stage at stage_off
void pd_pack_rows(uint8_t* region, uint32_t cu_bytes, uint32_t stage_off, int rows_cu, int ncu, const QMat& src,
                  const int* map_dev, hipStream_t s);
LFK_HD size_t pd_dump_stride(const PDecodeArgs& a) { return (size_t)2 * a.nq + 2 * a.nkv + 2 * a.d + a.F; }
// microbenchmark of the consumer item code alone: out[block * 8 + wave] = cycles per item
void pd_item_bench(int type, int rows, int K, int iters, int blocks, long long* out, hipStream_t s);
// ring row format size of one row
uint32_t pd_row_bytes(int type, int K);

}  // namespace lfk
