// Engine side of the persistent decode step (kernels/pdecode.h): eligibility,
// the per-CU weight layout ("ring row format", a second copy of the layer
// weights next to the planar copy the prefill GEMMs read - 288 GB of HBM holds
// both for every BASELINE model), the item tables, the granule buffers and the
// launch arguments.
//
// Layout of layer l: CU u's span at region_l + u * cu_bytes_l holds, in the
// order the loader streams and the consumers use them:
//   Q rows [u*NQU, +NQU) | K rows [u*NKU, +NKU) | V rows | Wo rows [u*NXU, +NXU)
//   | gate rows of features [u*NFU, +NFU) | up rows of the same features | down rows [u*NXU, +NXU)
// Each stage is cut into ring items of whole rows of at most one ring slot.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "../kernels/pdecode.h"
#include "engine.h"

namespace lfk {

#define HIPCHK(x) check((x), #x)

namespace {
bool pd_type_ok(int t) { return t == T_Q4_K || t == T_Q5_K || t == T_Q6_K || t == T_Q8_0; }
}  // namespace

std::string Engine::setup_pdecode() {
  pdec_ = false;
  const char* env = std::getenv("LFK_PDECODE");
  if (!env || env[0] != '1') return "off (LFK_PDECODE != 1)";
  if (opt_.tp_size > 1) return "tensor parallel";
  if (hp_.n_expert > 0) return "MoE";
  if (opt_.layer_begin != 0) return "hybrid placement";
  int dev = 0, ncu = 0;
  HIPCHK(hipGetDevice(&dev));
  HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int d = hp_.n_embd, hd = hp_.head_dim, nh = hp_.n_head, nkv = hp_.n_head_kv, F = hp_.n_ff;
  const int nq = nh * hd, nkvd = nkv * hd, G = nkv ? nh / nkv : 0;
  if (hd != 128) return "head_dim != 128";
  if (G != 4 && G != 8) return "gqa group not 4 or 8";
  if (ncu % 8 || ncu % nkv || d % ncu || nq % ncu || nkvd % ncu || F % ncu) return "shape does not split over the CUs";
  const int cpg = ncu / nkv, nxu = d / ncu, nqu = nq / ncu, nku = nkvd / ncu, nfu = F / ncu;
  if (nxu % 8 || nxu > 64 || nqu % 2 || nku % 2 || nfu % 8) return "per-CU slices not whole q8 blocks / rope pairs";
  if (nqu * cpg != G * hd || nku * cpg != hd) return "kv head groups do not map onto CU groups";
  if (cpg - G < 1) return "no CUs left for the merges";
  if (nqu + 2 * nku > 64) return "too many qkv rows per CU";
  for (int l = 0; l < hp_.n_layer; ++l) {
    const Layer& L = layers_[l];
    for (const QMat* m : {&L.wq, &L.wk, &L.wv, &L.wo, &L.w_gu, &L.w_down})
      if (!pd_type_ok(m->type) || m->K % 256) return "weight type";
  }

  PDecodeArgs a;
  a.d = d; a.nq = nq; a.nkv = nkvd; a.hd = hd; a.F = F; a.n_head = nh; a.n_kv_head = nkv; a.n_ctx = opt_.n_ctx;
  a.ncu = ncu; a.cpg = cpg; a.nxu = nxu; a.nqu = nqu; a.nku = nku; a.nfu = nfu;
  a.smax = cpg - G;
  a.eps = hp_.rms_eps; a.attn_scale = 1.f / std::sqrt((float)hd);
  a.slot_bytes = 16 * 1024;
  // LDS carve
  const int actn = (std::max(std::max(d, nq), F) + 63) & ~63;
  const int act_norm = actn + actn / 2 + ncu * 4;
  const int act_att = G * hd * 2 + 2 * hd * 2 + 4 * 16 * (hd + 8) * 2 + 4 * G * 16 * 4 + 2 * 4 * G * 4 + 4 * G * hd * 4;
  a.act_bytes = (std::max(act_norm, act_att) + 15) & ~15;
  // per-CU stage partials [row][block group] (kernel: stage_map)
  auto ngroup = [](int K) {
    const int nblk = ((K / 32) + 63) / 64;
    const int wpb = std::max(1, kPdConsumerWaves / nblk);
    return kPdConsumerWaves / wpb;
  };
  for (int K : {d, nq, F}) {
    const int nblk = ((K / 32) + 63) / 64;
    if (nblk > 2 * ngroup(K)) return "activation longer than two blocks per consumer wave";
  }
  a.part_floats = std::max({(nqu + 2 * nku) * ngroup(d), nxu * ngroup(nq), 2 * nfu * ngroup(d), nxu * ngroup(F)});
  const size_t fixed = 128 + 256 + ((a.part_floats * 4 + 15) & ~15) + a.act_bytes;
  const size_t lds_max = 160 * 1024;
  if (fixed + 3 * (size_t)a.slot_bytes > lds_max) return "LDS";
  a.nslot = (int)std::min<size_t>(8, (lds_max - fixed) / a.slot_bytes);
  a.res_rows = 0;

  // ---- item tables + region layout
  struct StageSpec { int stage; const QMat* m; int rows_cu; int row0; int map; };  // map: 0 none, 1 gate, 2 up
  std::vector<PdLayer> hl(hp_.n_layer);
  std::vector<PdItem> items;
  std::vector<size_t> region_off(hp_.n_layer);
  size_t total = 0;
  for (int l = 0; l < hp_.n_layer; ++l) {
    const Layer& L = layers_[l];
    const StageSpec st[7] = {{PD_Q, &L.wq, nqu, 0, 0},         {PD_K, &L.wk, nku, nqu, 0},
                             {PD_V, &L.wv, nku, nqu + nku, 0}, {PD_WO, &L.wo, nxu, 0, 0},
                             {PD_GATE, &L.w_gu, nfu, 0, 1},    {PD_UP, &L.w_gu, nfu, nfu, 2},
                             {PD_DOWN, &L.w_down, nxu, 0, 0}};
    hl[l].item0 = (int)items.size();
    size_t off = 0;
    for (const StageSpec& s : st) {
      const uint32_t rb = pd_row_bytes(s.m->type, s.m->K);
      if (rb == 0 || rb > (uint32_t)a.slot_bytes) return "row larger than a ring slot";
      // the loader keeps up to four items in flight and counts their transfers with vmcnt, a
      // 6-bit counter: together they must stay below 64 one-KiB transfers
      const int item_max = std::min(a.slot_bytes, 15 * 1024);
      const int per_slot = item_max / (int)rb;
      if (per_slot < 1) return "row larger than a ring item";
      const int nit = (s.rows_cu + per_slot - 1) / per_slot;
      for (int i = 0; i < nit; ++i) {
        const int r0 = (int)((long long)s.rows_cu * i / nit), r1 = (int)((long long)s.rows_cu * (i + 1) / nit);
        PdItem it;
        it.off = (uint32_t)(off + (size_t)r0 * rb);
        it.row_bytes = rb;
        it.rows = (uint16_t)(r1 - r0);
        it.row0 = (uint16_t)(s.row0 + r0);
        it.dma_kb = (uint16_t)(((size_t)(r1 - r0) * rb + 1023) / 1024);
        it.stage = (uint8_t)s.stage;
        it.type = (uint8_t)s.m->type;
        if (it.dma_kb * 1024 > a.slot_bytes || it.dma_kb > 15) return "item exceeds a ring slot";
        items.push_back(it);
      }
      off += (size_t)s.rows_cu * rb;
    }
    hl[l].nitems = (int)items.size() - hl[l].item0;
    hl[l].cu_bytes = (uint32_t)((off + 255) & ~(size_t)255);
    region_off[l] = total;
    total += (size_t)hl[l].cu_bytes * ncu;
    hl[l].attn_norm = L.attn_norm;
    hl[l].ffn_norm = L.ffn_norm;
  }
  // the loader rounds every item up to whole KiB: pad the end
  uint8_t* mk = static_cast<uint8_t*>(dalloc(total + (size_t)a.slot_bytes));
  HIPCHK(hipMemsetAsync(mk, 0, total + (size_t)a.slot_bytes, stream_));
  // gate / up source rows in the planar matrix (32-row interleave, engine.cpp upload_gate_up)
  std::vector<int> gmap(F), umap(F);
  for (int f = 0; f < F; ++f) {
    gmap[f] = (f >> 5) * 64 + (f & 31);
    umap[f] = gmap[f] + 32;
  }
  int* gmap_d = static_cast<int*>(dalloc(sizeof(int) * F));
  int* umap_d = static_cast<int*>(dalloc(sizeof(int) * F));
  HIPCHK(hipMemcpy(gmap_d, gmap.data(), sizeof(int) * F, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(umap_d, umap.data(), sizeof(int) * F, hipMemcpyHostToDevice));
  for (int l = 0; l < hp_.n_layer; ++l) {
    const Layer& L = layers_[l];
    hl[l].wbase = mk + region_off[l];
    uint8_t* region = mk + region_off[l];
    const uint32_t cb = hl[l].cu_bytes;
    uint32_t off = 0;
    auto put = [&](const QMat& m, int rows_cu, const int* map) {
      pd_pack_rows(region, cb, off, rows_cu, ncu, m, map, stream_);
      off += (uint32_t)rows_cu * pd_row_bytes(m.type, m.K);
    };
    put(L.wq, nqu, nullptr);
    put(L.wk, nku, nullptr);
    put(L.wv, nku, nullptr);
    put(L.wo, nxu, nullptr);
    put(L.w_gu, nfu, gmap_d);
    put(L.w_gu, nfu, umap_d);
    put(L.w_down, nxu, nullptr);
  }
  HIPCHK(hipGetLastError());

  // ---- granule buffers (one region per layer, tags = launch epoch)
  size_t o = 0;
  a.off_hx = (int)o; o += (size_t)ncu * (nxu / 4 + nxu / 8 + 1);
  a.off_qkv = (int)o; o += (size_t)ncu * (nqu / 2 + nku);
  a.off_att = (int)o; o += (size_t)nkv * a.smax * G * (hd + 2);
  a.off_o = (int)o; o += (size_t)nh * (hd / 4 + hd / 8);
  a.off_hx2 = (int)o; o += (size_t)ncu * (nxu / 4 + nxu / 8 + 1);
  a.off_hh = (int)o; o += (size_t)ncu * (nfu / 4 + nfu / 8);
  a.gran_layer = (o + 63) & ~(size_t)63;
  const size_t gbytes = sizeof(unsigned long long) * a.gran_layer * hp_.n_layer;
  a.gran = static_cast<unsigned long long*>(dalloc(gbytes));
  HIPCHK(hipMemsetAsync(a.gran, 0, gbytes, stream_));
  a.epoch = static_cast<unsigned*>(dalloc(sizeof(unsigned) * 4));
  const unsigned one[4] = {1, 0, 0, 0};
  HIPCHK(hipMemcpy(a.epoch, one, sizeof(one), hipMemcpyHostToDevice));

  PdLayer* hl_d = static_cast<PdLayer*>(dalloc(sizeof(PdLayer) * hl.size()));
  PdItem* it_d = static_cast<PdItem*>(dalloc(sizeof(PdItem) * items.size()));
  HIPCHK(hipMemcpy(hl_d, hl.data(), sizeof(PdLayer) * hl.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(it_d, items.data(), sizeof(PdItem) * items.size(), hipMemcpyHostToDevice));
  a.layers = hl_d;
  a.items = it_d;
  a.n_layer = hp_.n_layer;
  a.x = x_;
  a.k_cache = kc_;
  a.v_cache = vc_;
  a.kv_layer = (size_t)nkv_l_ * opt_.n_ctx * hd;
  a.rope = rope_;
  a.pos = state_ + S_POS;
  a.err = dev_err_;
  if (!pdecode_resident(a)) return "one workgroup per CU is not resident";
  if (const char* dm = std::getenv("LFK_PDECODE_DBG")) a.dbg_mode = std::atoi(dm);
  if (const char* ac = std::getenv("LFK_PDECODE_ACCT"); ac && ac[0] == '1') {
    pd_acct_n_ = (size_t)ncu * 16;
    a.acct = static_cast<long long*>(dalloc(sizeof(long long) * pd_acct_n_));
    HIPCHK(hipMemsetAsync(a.acct, 0, sizeof(long long) * pd_acct_n_, stream_));
  }
  if (const char* tm = std::getenv("LFK_PDECODE_TIMELINE"); tm && tm[0] == '1') {
    pd_tl_n_ = (size_t)ncu * hp_.n_layer * kPdStamps + (size_t)ncu * kPdItemStamps * 8;
    a.tl = static_cast<long long*>(dalloc(sizeof(long long) * pd_tl_n_));
    a.tli = a.tl + (size_t)ncu * hp_.n_layer * kPdStamps;
    HIPCHK(hipMemsetAsync(a.tl, 0, sizeof(long long) * pd_tl_n_, stream_));
  }
  if (const char* dm = std::getenv("LFK_PDECODE_DUMP"); dm && dm[0] == '1') {
    pd_dump_n_ = pd_dump_stride(a) * hp_.n_layer;
    a.dbg = static_cast<float*>(dalloc(sizeof(float) * pd_dump_n_));
    HIPCHK(hipMemsetAsync(a.dbg, 0, sizeof(float) * pd_dump_n_, stream_));
  }
  pda_dev_ = static_cast<PDecodeArgs*>(dalloc(sizeof(PDecodeArgs)));
  HIPCHK(hipMemcpyAsync(pda_dev_, &a, sizeof(PDecodeArgs), hipMemcpyHostToDevice, stream_));
  HIPCHK(hipStreamSynchronize(stream_));
  pda_ = a;
  pdec_ = true;
  if (opt_.verbose)
    std::fprintf(stderr, "[lfk] persistent decode: %d CUs, ring %d x %d KiB, %zu items, %.2f GB ring-format weights\n",
                 ncu, a.nslot, a.slot_bytes / 1024, items.size(), total / 1e9);
  return "on";
}

std::vector<long long> Engine::pdecode_acct() {
  std::vector<long long> out(pd_acct_n_);
  if (pd_acct_n_) {
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(out.data(), pda_.acct, sizeof(long long) * pd_acct_n_, hipMemcpyDeviceToHost));
  }
  return out;
}

std::vector<long long> Engine::pdecode_timeline() {
  std::vector<long long> out(pd_tl_n_);
  if (pd_tl_n_) {
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(out.data(), pda_.tl, sizeof(long long) * pd_tl_n_, hipMemcpyDeviceToHost));
  }
  return out;
}

std::vector<float> Engine::pdecode_dump() {
  std::vector<float> out(pd_dump_n_);
  if (pd_dump_n_) {
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(out.data(), pda_.dbg, sizeof(float) * pd_dump_n_, hipMemcpyDeviceToHost));
  }
  return out;
}

}  // namespace lfk
