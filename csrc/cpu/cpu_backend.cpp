#include "cpu_backend.h"

#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <stdexcept>

#include "../runtime/gguf.h"
#include "../runtime/repack.h"
#include "../runtime/shard.h"

namespace lfk {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline float h2f(uint16_t h) { return _cvtsh_ss(h); }
inline uint16_t f2h(float f) { return _cvtss_sh(f, 0); }

// rows [r0, r0+R) x columns [c0, c0+K) of a (per-expert) ggml matrix -> planar; rows past the
// source are zero (vocab padding of the last TP shard). R < 0 / K < 0 = everything.
CpuMat load_mat(const GGUFFile& f, const std::string& name, int n_expert = 0, size_t r0 = 0, long R = -1,
                size_t c0 = 0, long K = -1) {
  const GGUFTensor* t = f.find(name);
  if (!t) throw std::runtime_error("missing tensor " + name);
  const size_t K_src = (size_t)t->ne[0], R_src = (size_t)t->ne[1];
  CpuMat m;
  m.type = t->type;
  m.K = K < 0 ? (int)K_src : (int)K;
  m.rows = R < 0 ? (int)R_src : (int)R;
  const int E = n_expert > 0 ? n_expert : 1;
  const size_t one = qbytes(m.type, m.rows, m.K);
  const size_t src_one = qbytes(m.type, R_src, K_src);
  const size_t avail = r0 < R_src ? std::min((size_t)m.rows, R_src - r0) : 0;
  m.data.assign(one * E, 0);
  for (int e = 0; e < E; ++e)
    repack_planar(m.type, f.data(*t) + src_one * e, K_src, r0, avail, c0, m.K, m.data.data() + one * e, m.rows, 0,
                  0);
  m.P = planes_of(m.type, m.rows, m.K);
  m.expert_stride = n_expert > 0 ? one : 0;
  return m;
}

// gate/up features [f0, f0+F) interleaved in 32-row groups (the GPU layout)
CpuMat load_gate_up(const GGUFFile& f, const std::string& g, const std::string& u, int n_expert, size_t f0,
                    long F) {
  const GGUFTensor* tg = f.find(g);
  const GGUFTensor* tu = f.find(u);
  if (!tg || !tu) throw std::runtime_error("missing " + g);
  if (tg->type != tu->type) throw std::runtime_error("gate/up projections must share a quant type");
  CpuMat m;
  m.type = tg->type;
  m.K = (int)tg->ne[0];
  const size_t F_src = (size_t)tg->ne[1];
  if (F < 0) F = (long)F_src;
  m.rows = 2 * (int)F;
  const int E = n_expert > 0 ? n_expert : 1;
  const size_t one = qbytes(m.type, m.rows, m.K);
  const size_t src_one = qbytes(m.type, F_src, m.K);
  m.data.resize(one * E);
  for (int e = 0; e < E; ++e) {
    repack_planar(m.type, f.data(*tg) + src_one * e, m.K, f0, F, 0, m.K, m.data.data() + one * e, m.rows, 32, 0);
    repack_planar(m.type, f.data(*tu) + src_one * e, m.K, f0, F, 0, m.K, m.data.data() + one * e, m.rows, 32, 32);
  }
  m.P = planes_of(m.type, m.rows, m.K);
  m.expert_stride = n_expert > 0 ? one : 0;
  return m;
}

std::vector<float> load_f32(const GGUFFile& f, const std::string& name) {
  const GGUFTensor* t = f.find(name);
  if (!t || t->type != T_F32) throw std::runtime_error("missing F32 tensor " + name);
  std::vector<float> v(t->n_elements());
  std::memcpy(v.data(), f.data(*t), v.size() * 4);
  return v;
}

// ---- q8 activations: identical rounding to the GPU prologue (round half to even)
struct Q8 {
  std::vector<int8_t> q;   // [T][K]
  std::vector<float> d;    // [T][K/32]
  std::vector<int> s16;    // [T][K/16] sums of q over 16
  int K = 0;
};

void quantize_rows(const float* x, int T, int ldx, int K, const std::vector<float>* norm, float eps, Q8& o) {
  o.K = K;
  o.q.resize((size_t)T * K);
  o.d.resize((size_t)T * K / 32);
  o.s16.resize((size_t)T * K / 16);
  for (int t = 0; t < T; ++t) {
    const float* xr = x + (size_t)t * ldx;
    float scale = 1.f;
    if (norm) {
      double ss = 0;
      for (int i = 0; i < K; ++i) ss += (double)xr[i] * xr[i];
      scale = 1.f / std::sqrt((float)(ss / K) + eps);
    }
    for (int b = 0; b < K / 32; ++b) {
      float v[32], amax = 0.f;
      for (int i = 0; i < 32; ++i) {
        v[i] = norm ? xr[32 * b + i] * scale * (*norm)[32 * b + i] : xr[32 * b + i];
        amax = std::max(amax, std::fabs(v[i]));
      }
      const float d = amax * (1.f / 127.f);
      const float id = d > 0.f ? 1.f / d : 0.f;
      int8_t* q = o.q.data() + (size_t)t * K + 32 * b;
      for (int i = 0; i < 32; ++i) q[i] = (int8_t)std::nearbyint(v[i] * id);
      o.d[(size_t)t * (K / 32) + b] = d;
      int s0 = 0, s1 = 0;
      for (int i = 0; i < 16; ++i) { s0 += q[i]; s1 += q[16 + i]; }
      o.s16[(size_t)t * (K / 16) + 2 * b] = s0;
      o.s16[(size_t)t * (K / 16) + 2 * b + 1] = s1;
    }
  }
}

// One 32-weight chunk decoded to int8 + per-half affine scales (the GPU chunk map).
struct Chunk {
  int8_t w[32];              // [0,16) lo half, [16,32) hi half
  int off_lo, off_hi;        // x offsets of the halves
  float s_lo, m_lo, s_hi, m_hi;  // sum = s*dot(w,x) - m*sum(x)   (x in q8 units, times xd)
  bool is_float = false;
  float wf[32];
};

inline void scale_min_k4(int j, const uint8_t* q, int& sc, int& m) {
  if (j < 4) { sc = q[j] & 63; m = q[j + 4] & 63; }
  else { sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4); }
}

inline float hf(const uint8_t* p) { uint16_t h; std::memcpy(&h, p, 2); return h2f(h); }

void decode_chunk(const CpuMat& W, const uint8_t* base, size_t row, int c, Chunk& ch) {
  const Planes& P = W.P;
  const int sb = c >> 3, j = c & 7;
  switch (W.type) {
    case T_Q4_K:
    case T_Q5_K: {
      const int g = j >> 1, h = j & 1;
      const uint8_t* qs = base + P.p0 + row * P.s0 + 16 * c;
      const uint8_t* meta = base + (W.type == T_Q4_K ? P.p1 + row * P.s1 : P.p2 + row * P.s2) + 16 * sb;
      const uint8_t* qh = W.type == T_Q5_K ? base + P.p1 + row * P.s1 + 32 * sb + 16 * h : nullptr;
      const float d = hf(meta), dmin = hf(meta + 2);
      int sc0, m0, sc1, m1;
      scale_min_k4(2 * g, meta + 4, sc0, m0);
      scale_min_k4(2 * g + 1, meta + 4, sc1, m1);
      for (int i = 0; i < 16; ++i) {
        int lo = qs[i] & 0xF, hi = qs[i] >> 4;
        if (qh) { lo |= ((qh[i] >> (2 * g)) & 1) << 4; hi |= ((qh[i] >> (2 * g + 1)) & 1) << 4; }
        ch.w[i] = (int8_t)lo;
        ch.w[16 + i] = (int8_t)hi;
      }
      ch.off_lo = sb * 256 + 64 * g + 16 * h;
      ch.off_hi = ch.off_lo + 32;
      ch.s_lo = d * sc0; ch.m_lo = dmin * m0;
      ch.s_hi = d * sc1; ch.m_hi = dmin * m1;
      break;
    }
    case T_Q6_K: {
      const int n = j >> 2, o = 16 * (j & 3);
      const uint8_t* ql = base + P.p0 + row * P.s0 + 16 * c;
      const uint8_t* qh = base + P.p1 + row * P.s1 + 64 * sb + 32 * n + (o & 31);
      const int8_t* sc = reinterpret_cast<const int8_t*>(base + P.p2 + row * P.s2 + 16 * sb);
      const float d = hf(base + P.p3 + row * P.s3 + 2 * sb);
      const int s = o >= 32 ? 2 : 0;
      for (int i = 0; i < 16; ++i) {
        ch.w[i] = (int8_t)((ql[i] & 0xF) | (((qh[i] >> s) & 3) << 4));
        ch.w[16 + i] = (int8_t)((ql[i] >> 4) | (((qh[i] >> (s + 4)) & 3) << 4));
      }
      const int si = 8 * n + (o >> 4);
      ch.off_lo = sb * 256 + 128 * n + o;
      ch.off_hi = ch.off_lo + 64;
      ch.s_lo = d * sc[si]; ch.m_lo = 32.f * ch.s_lo;
      ch.s_hi = d * sc[si + 4]; ch.m_hi = 32.f * ch.s_hi;
      break;
    }
    case T_Q8_0: {
      const int8_t* q = reinterpret_cast<const int8_t*>(base + P.p0 + row * P.s0 + 32 * c);
      std::memcpy(ch.w, q, 32);
      const float d = hf(base + P.p1 + row * P.s1 + 2 * c);
      ch.off_lo = 32 * c;
      ch.off_hi = 32 * c + 16;
      ch.s_lo = ch.s_hi = d;
      ch.m_lo = ch.m_hi = 0.f;
      break;
    }
    case T_F32:
    case T_F16: {
      ch.is_float = true;
      for (int i = 0; i < 32; ++i)
        ch.wf[i] = W.type == T_F32 ? reinterpret_cast<const float*>(base + row * P.s0)[32 * c + i]
                                   : h2f(reinterpret_cast<const uint16_t*>(base + row * P.s0)[32 * c + i]);
      ch.off_lo = 32 * c;
      ch.off_hi = 32 * c + 16;
      break;
    }
    default:
      throw std::runtime_error("cpu: unsupported weight type");
  }
}

// ---- AVX2 path for the block-quantised types: one 32-weight chunk is unpacked
// into a 256-bit vector (lo 16 | hi 16, unsigned for the K-quants, signed for
// Q8_0) and dotted with the q8 activations of every token on
// vpmaddubsw/vpmaddwd; per-chunk scales are applied in float lanes (lo 4 | hi 4)
// so no horizontal sum happens until the end of the row.
template <int QT>
inline __m256i chunk_w(const CpuMat& W, const uint8_t* base, size_t row, int c, float& s_lo, float& m_lo, float& s_hi,
                       float& m_hi, int& off_lo, int& off_hi) {
  const Planes& P = W.P;
  const int sb = c >> 3, j = c & 7;
  const __m128i m4 = _mm_set1_epi8(0x0F);
  if constexpr (QT == T_Q4_K || QT == T_Q5_K) {
    const int g = j >> 1, h = j & 1;
    const __m128i q = _mm_loadu_si128(reinterpret_cast<const __m128i*>(base + P.p0 + row * P.s0 + 16 * c));
    __m128i lo = _mm_and_si128(q, m4), hi = _mm_and_si128(_mm_srli_epi16(q, 4), m4);
    const uint8_t* meta = base + (QT == T_Q4_K ? P.p1 + row * P.s1 : P.p2 + row * P.s2) + 16 * sb;
    if constexpr (QT == T_Q5_K) {
      const __m128i qh = _mm_loadu_si128(reinterpret_cast<const __m128i*>(base + P.p1 + row * P.s1 + 32 * sb + 16 * h));
      const __m128i one = _mm_set1_epi8(1);
      lo = _mm_or_si128(lo, _mm_slli_epi16(_mm_and_si128(_mm_srl_epi16(qh, _mm_cvtsi32_si128(2 * g)), one), 4));
      hi = _mm_or_si128(hi, _mm_slli_epi16(_mm_and_si128(_mm_srl_epi16(qh, _mm_cvtsi32_si128(2 * g + 1)), one), 4));
    }
    const float d = hf(meta), dmin = hf(meta + 2);
    int sc0, mm0, sc1, mm1;
    scale_min_k4(2 * g, meta + 4, sc0, mm0);
    scale_min_k4(2 * g + 1, meta + 4, sc1, mm1);
    s_lo = d * sc0; m_lo = dmin * mm0; s_hi = d * sc1; m_hi = dmin * mm1;
    off_lo = sb * 256 + 64 * g + 16 * h;
    off_hi = off_lo + 32;
    return _mm256_set_m128i(hi, lo);
  } else if constexpr (QT == T_Q6_K) {
    const int n = j >> 2, o = 16 * (j & 3);
    const __m128i ql = _mm_loadu_si128(reinterpret_cast<const __m128i*>(base + P.p0 + row * P.s0 + 16 * c));
    const __m128i qh =
        _mm_loadu_si128(reinterpret_cast<const __m128i*>(base + P.p1 + row * P.s1 + 64 * sb + 32 * n + (o & 31)));
    const int sh = o >= 32 ? 2 : 0;
    const __m128i m3 = _mm_set1_epi8(3);
    const __m128i lo = _mm_or_si128(_mm_and_si128(ql, m4),
                                    _mm_slli_epi16(_mm_and_si128(_mm_srl_epi16(qh, _mm_cvtsi32_si128(sh)), m3), 4));
    const __m128i hi = _mm_or_si128(_mm_and_si128(_mm_srli_epi16(ql, 4), m4),
                                    _mm_slli_epi16(_mm_and_si128(_mm_srl_epi16(qh, _mm_cvtsi32_si128(sh + 4)), m3), 4));
    const int8_t* sc = reinterpret_cast<const int8_t*>(base + P.p2 + row * P.s2 + 16 * sb);
    const float d = hf(base + P.p3 + row * P.s3 + 2 * sb);
    const int si = 8 * n + (o >> 4);
    s_lo = d * sc[si]; m_lo = 32.f * s_lo;
    s_hi = d * sc[si + 4]; m_hi = 32.f * s_hi;
    off_lo = sb * 256 + 128 * n + o;
    off_hi = off_lo + 64;
    return _mm256_set_m128i(hi, lo);
  } else {  // Q8_0 (signed)
    const float d = hf(base + P.p1 + row * P.s1 + 2 * c);
    s_lo = s_hi = d;
    m_lo = m_hi = 0.f;
    off_lo = 32 * c;
    off_hi = 32 * c + 16;
    return _mm256_loadu_si256(reinterpret_cast<const __m256i*>(base + P.p0 + row * P.s0 + 32 * c));
  }
}

template <int QT>
void gemm_rows_avx2(const CpuMat& W, const uint8_t* base, const Q8& xq, int T, float* y, int ldy, bool add) {
  const int K = W.K, nchunks = K / 32, nb = K / 32, n16 = K / 16;
  const __m256i ones = _mm256_set1_epi16(1);
#pragma omp parallel for schedule(static)
  for (int r = 0; r < W.rows; ++r) {
    __m256 acc[128];
    float mterm[128];
    for (int t = 0; t < T; ++t) { acc[t] = _mm256_setzero_ps(); mterm[t] = 0.f; }
    for (int c = 0; c < nchunks; ++c) {
      float s_lo, m_lo, s_hi, m_hi;
      int off_lo, off_hi;
      __m256i w = chunk_w<QT>(W, base, (size_t)r, c, s_lo, m_lo, s_hi, m_hi, off_lo, off_hi);
      __m256i wa = w;
      if constexpr (QT == T_Q8_0) wa = _mm256_sign_epi8(w, w);  // |w| (unsigned operand of vpmaddubsw)
      const int blo = off_lo >> 5, bhi = off_hi >> 5;
      for (int t = 0; t < T; ++t) {
        const int8_t* x = xq.q.data() + (size_t)t * K;
        __m256i xv = _mm256_set_m128i(_mm_loadu_si128(reinterpret_cast<const __m128i*>(x + off_hi)),
                                      _mm_loadu_si128(reinterpret_cast<const __m128i*>(x + off_lo)));
        if constexpr (QT == T_Q8_0) xv = _mm256_sign_epi8(xv, w);
        const __m256i p = _mm256_madd_epi16(_mm256_maddubs_epi16(wa, xv), ones);
        const float* xd = xq.d.data() + (size_t)t * nb;
        const float xl = xd[blo], xh = xd[bhi];
        const __m256 sv = _mm256_set_m128(_mm_set1_ps(s_hi * xh), _mm_set1_ps(s_lo * xl));
        acc[t] = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p), sv, acc[t]);
        if constexpr (QT != T_Q8_0) {
          const int* s16 = xq.s16.data() + (size_t)t * n16;
          mterm[t] += m_lo * xl * (float)s16[off_lo >> 4] + m_hi * xh * (float)s16[off_hi >> 4];
        }
      }
    }
    for (int t = 0; t < T; ++t) {
      const __m128 h = _mm_add_ps(_mm256_castps256_ps128(acc[t]), _mm256_extractf128_ps(acc[t], 1));
      const __m128 h2 = _mm_add_ps(h, _mm_movehl_ps(h, h));
      const float v = _mm_cvtss_f32(_mm_add_ss(h2, _mm_shuffle_ps(h2, h2, 1))) - mterm[t];
      float* o = y + (size_t)t * ldy + r;
      *o = add ? *o + v : v;
    }
  }
}

void gemm_rows_scalar(const CpuMat& W, const uint8_t* base, const Q8& xq, int T, float* y, int ldy, bool add);

// y[t][r] (+)= W[r] . x_t for rows r of a (possibly expert-offset) matrix
void gemm_rows(const CpuMat& W, const uint8_t* base, const Q8& xq, int T, float* y, int ldy, bool add) {
  if (T > 128) throw std::runtime_error("cpu gemm: at most 128 tokens per call");
  switch (W.type) {
    case T_Q4_K: return gemm_rows_avx2<T_Q4_K>(W, base, xq, T, y, ldy, add);
    case T_Q5_K: return gemm_rows_avx2<T_Q5_K>(W, base, xq, T, y, ldy, add);
    case T_Q6_K: return gemm_rows_avx2<T_Q6_K>(W, base, xq, T, y, ldy, add);
    case T_Q8_0: return gemm_rows_avx2<T_Q8_0>(W, base, xq, T, y, ldy, add);
    default: return gemm_rows_scalar(W, base, xq, T, y, ldy, add);
  }
}

// portable path (F16/F32 and the numerics reference of the AVX2 path)
void gemm_rows_scalar(const CpuMat& W, const uint8_t* base, const Q8& xq, int T, float* y, int ldy, bool add) {
  const int K = W.K, nchunks = K / 32, nb = K / 32, n16 = K / 16;
#pragma omp parallel for schedule(static)
  for (int r = 0; r < W.rows; ++r) {
    float acc[128];
    for (int t = 0; t < T; ++t) acc[t] = 0.f;
    Chunk ch;
    for (int c = 0; c < nchunks; ++c) {
      decode_chunk(W, base, (size_t)r, c, ch);
      const int blo = ch.off_lo >> 5, bhi = ch.off_hi >> 5;
      for (int t = 0; t < T; ++t) {
        const int8_t* x = xq.q.data() + (size_t)t * K;
        const float* xd = xq.d.data() + (size_t)t * nb;
        if (ch.is_float) {
          float s = 0.f;
          for (int i = 0; i < 16; ++i) s += ch.wf[i] * x[ch.off_lo + i] * xd[blo];
          for (int i = 0; i < 16; ++i) s += ch.wf[16 + i] * x[ch.off_hi + i] * xd[bhi];
          acc[t] += s;
          continue;
        }
        int dl = 0, dh = 0;
        for (int i = 0; i < 16; ++i) dl += (int)ch.w[i] * x[ch.off_lo + i];
        for (int i = 0; i < 16; ++i) dh += (int)ch.w[16 + i] * x[ch.off_hi + i];
        const int* s16 = xq.s16.data() + (size_t)t * n16;
        acc[t] += xd[blo] * (ch.s_lo * (float)dl - ch.m_lo * (float)s16[ch.off_lo >> 4]) +
                  xd[bhi] * (ch.s_hi * (float)dh - ch.m_hi * (float)s16[ch.off_hi >> 4]);
      }
    }
    for (int t = 0; t < T; ++t) {
      float* o = y + (size_t)t * ldy + r;
      *o = add ? *o + acc[t] : acc[t];
    }
  }
}

inline float silu(float g) { return g / (1.f + std::exp(-g)); }

}  // namespace

float splitmix_uniform(uint64_t seed, uint64_t step) {
  uint64_t x = seed ^ (step * 0xD1B54A32D192ED03ull);
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.f / 16777216.f);
}

int cpu_sample(std::vector<float> l, const std::vector<int>& window, const CpuSampling& sp, int step) {
  const int V = (int)l.size();
  // penalties (first occurrence applies, count = occurrences in the window)
  if (sp.last_n > 0 && !window.empty()) {
    const int n = (int)window.size(), w0 = std::max(0, n - sp.last_n);
    for (int i = w0; i < n; ++i) {
      const int t = window[i];
      if (t < 0 || t >= V) continue;
      bool first = true;
      int cnt = 0;
      for (int j = w0; j < n; ++j) {
        if (window[j] == t) { ++cnt; if (j < i) first = false; }
      }
      if (!first) continue;
      float v = l[t];
      v = v <= 0.f ? v * sp.repeat_penalty : v / sp.repeat_penalty;
      v -= (float)cnt * sp.freq_penalty + sp.presence_penalty;
      l[t] = v;
    }
  }
  if (sp.temp <= 0.f) return (int)(std::max_element(l.begin(), l.end()) - l.begin());
  const int k = (sp.top_k > 0 && sp.top_k < V) ? sp.top_k : V;
  std::vector<int> ids(V);
  std::iota(ids.begin(), ids.end(), 0);
  auto better = [&](int a, int b) { return l[a] > l[b] || (l[a] == l[b] && a < b); };
  std::partial_sort(ids.begin(), ids.begin() + k, ids.end(), better);
  ids.resize(k);
  int n = k;
  const double v0 = l[ids[0]];
  if (sp.top_p < 1.f) {
    double tot = 0;
    for (int i = 0; i < n; ++i) tot += std::exp((double)l[ids[i]] - v0);
    double cum = 0;
    for (int i = 0; i < n; ++i) {
      cum += std::exp((double)l[ids[i]] - v0) / tot;
      if (cum >= sp.top_p) { n = i + 1; break; }
    }
  }
  if (sp.min_p > 0.f) {
    const double thr = v0 + std::log((double)sp.min_p);
    int keep = 0;
    for (int i = 0; i < n; ++i) keep += (double)l[ids[i]] >= thr;
    n = std::max(1, keep);
  }
  std::vector<double> cw(n);
  double acc = 0;
  for (int i = 0; i < n; ++i) {
    acc += std::exp(((double)l[ids[i]] - v0) / sp.temp);
    cw[i] = acc;
  }
  const double u = splitmix_uniform(sp.seed, (uint64_t)step) * acc;
  for (int i = 0; i < n; ++i)
    if (cw[i] > u) return ids[i];
  return ids[n - 1];
}

CpuEngine::CpuEngine(const std::string& path, const CpuOptions& o)
    : opt_(o), n_ctx_(o.n_ctx), n_threads_(o.n_threads > 0 ? o.n_threads : omp_get_max_threads()),
      n_batch_(std::max(1, std::min(o.n_batch, 128))) {
  omp_set_num_threads(n_threads_);
  GGUFFile f(path);
  std::string arch = f.get_str("general.architecture", "llama");
  auto gi = [&](const char* k, int64_t d) { return (int)f.get_int(arch + "." + k, d); };
  n_embd_ = gi("embedding_length", 0);
  n_layer_ = gi("block_count", 0);
  n_head_ = gi("attention.head_count", 0);
  n_head_kv_ = gi("attention.head_count_kv", n_head_);
  head_dim_ = gi("rope.dimension_count", n_embd_ / n_head_);
  n_ff_ = gi("feed_forward_length", 0);
  n_expert_ = gi("expert_count", 0);
  n_expert_used_ = gi("expert_used_count", 0);
  eps_ = (float)f.get_float(arch + ".attention.layer_norm_rms_epsilon", 1e-5);
  rope_base_ = (float)f.get_float(arch + ".rope.freq_base", 10000.0);
  if (n_ctx_ <= 0) n_ctx_ = gi("context_length", 2048);
  const GGUFTensor* emb = f.find("token_embd.weight");
  if (!emb) throw std::runtime_error("missing token_embd.weight");
  n_vocab_ = (int)emb->ne[1];
  if (head_dim_ % 32) throw std::runtime_error("cpu backend: head_dim must be a multiple of 32");
  sp_ = make_shard_plan(n_head_, n_head_kv_, head_dim_, n_ff_, n_vocab_, o.tp_size, o.tp_rank, o.tensor_split);
  layer_end_ = o.layer_end < 0 ? n_layer_ : std::min(o.layer_end, n_layer_);
  tok_embd_ = load_mat(f, "token_embd.weight");
  if (o.load_head) {
    out_norm_ = load_f32(f, "output_norm.weight");
    const std::string on = f.find("output.weight") ? "output.weight" : "token_embd.weight";
    output_ = load_mat(f, on, 0, sp_.v_row0(), sp_.V_l);
  }
  layers_.resize(n_layer_);
  for (int l = 0; l < layer_end_; ++l) {
    const std::string p = "blk." + std::to_string(l) + ".";
    CpuLayer& L = layers_[l];
    L.attn_norm = load_f32(f, p + "attn_norm.weight");
    L.ffn_norm = load_f32(f, p + "ffn_norm.weight");
    L.wq = load_mat(f, p + "attn_q.weight", 0, sp_.q_row0(), sp_.nq);
    L.wk = load_mat(f, p + "attn_k.weight", 0, sp_.kv_row0(), sp_.nkvd);
    L.wv = load_mat(f, p + "attn_v.weight", 0, sp_.kv_row0(), sp_.nkvd);
    L.wo = load_mat(f, p + "attn_output.weight", 0, 0, -1, sp_.q_row0(), sp_.nq);
    if (n_expert_ > 0) {
      L.router = load_mat(f, p + "ffn_gate_inp.weight");
      L.gu_exps = load_gate_up(f, p + "ffn_gate_exps.weight", p + "ffn_up_exps.weight", n_expert_, sp_.f0(), sp_.F_l);
      L.down_exps = load_mat(f, p + "ffn_down_exps.weight", n_expert_, 0, -1, sp_.f0(), sp_.F_l);
    } else {
      L.w_gu = load_gate_up(f, p + "ffn_gate.weight", p + "ffn_up.weight", 0, sp_.f0(), sp_.F_l);
      L.w_down = load_mat(f, p + "ffn_down.weight", 0, 0, -1, sp_.f0(), sp_.F_l);
    }
  }
  const size_t kv = (size_t)layer_end_ * sp_.nkv_l * n_ctx_ * head_dim_;
  kc_.assign(kv, 0);
  vc_.assign(kv, 0);
  rope_cos_.resize((size_t)n_ctx_ * head_dim_ / 2);
  rope_sin_.resize(rope_cos_.size());
  for (int p = 0; p < n_ctx_; ++p)
    for (int i = 0; i < head_dim_ / 2; ++i) {
      const double a = p * std::pow((double)rope_base_, -2.0 * i / head_dim_);
      rope_cos_[(size_t)p * head_dim_ / 2 + i] = (float)std::cos(a);
      rope_sin_[(size_t)p * head_dim_ / 2 + i] = (float)std::sin(a);
    }
}

void CpuEngine::set_comm(std::function<void(float*, size_t)> allreduce,
                         std::function<void(const float*, float*, size_t)> allgather) {
  allreduce_ = std::move(allreduce);
  allgather_ = std::move(allgather);
}

void CpuEngine::reduce(float* y, size_t n) {
  if (sp_.tp == 1) return;
  if (!allreduce_) throw std::runtime_error("tensor parallel CPU engine: set_comm() was not called");
  allreduce_(y, n);
}

void CpuEngine::matmul(const CpuMat& W, const float* x, int T, int ldx, float* y, int ldy,
                       const std::vector<float>* norm, bool add) const {
  Q8 q;
  quantize_rows(x, T, ldx, W.K, norm, eps_, q);
  gemm_rows(W, W.data.data(), q, T, y, ldy, add);
}

void CpuEngine::embed(const int* tokens, int T, float* x) const {
  const int d = n_embd_;
  for (int t = 0; t < T; ++t) {
    if (tokens[t] < 0 || tokens[t] >= n_vocab_) throw std::runtime_error("token id out of range");
    Chunk ch;
    for (int c = 0; c < d / 32; ++c) {
      decode_chunk(tok_embd_, tok_embd_.data.data(), (size_t)tokens[t], c, ch);
      float* xr = x + (size_t)t * d;
      for (int i = 0; i < 16; ++i) {
        xr[ch.off_lo + i] = ch.is_float ? ch.wf[i] : ch.s_lo * ch.w[i] - ch.m_lo;
        xr[ch.off_hi + i] = ch.is_float ? ch.wf[16 + i] : ch.s_hi * ch.w[16 + i] - ch.m_hi;
      }
    }
  }
}

void CpuEngine::attention(int l, const float* q, int T, int pos0, float* out) const {
  const int hd = head_dim_, nh = sp_.nh_l, nkv = sp_.nkv_l, G = nh / nkv;
  const float scale = 1.f / std::sqrt((float)hd);
  const uint16_t* kc = kc_.data() + (size_t)l * nkv * n_ctx_ * hd;
  const uint16_t* vc = vc_.data() + (size_t)l * nkv * n_ctx_ * hd;
  // f16 rows are widened 8 at a time (F16C) and dotted / accumulated on FMA
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
  for (int t = 0; t < T; ++t)
    for (int h = 0; h < nh; ++h) {
      const int L = pos0 + t + 1, kvh = h / G;
      const float* qh = q + ((size_t)t * nh + h) * hd;
      std::vector<float> s(L);
      float m = -INFINITY;
      for (int j = 0; j < L; ++j) {
        const uint16_t* kr = kc + ((size_t)kvh * n_ctx_ + j) * hd;
        __m256 a = _mm256_setzero_ps();
        for (int i = 0; i < hd; i += 8) {
          const __m256 kf = _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i*>(kr + i)));
          a = _mm256_fmadd_ps(_mm256_loadu_ps(qh + i), kf, a);
        }
        const __m128 h4 = _mm_add_ps(_mm256_castps256_ps128(a), _mm256_extractf128_ps(a, 1));
        const __m128 h2 = _mm_add_ps(h4, _mm_movehl_ps(h4, h4));
        s[j] = _mm_cvtss_f32(_mm_add_ss(h2, _mm_shuffle_ps(h2, h2, 1))) * scale;
        m = std::max(m, s[j]);
      }
      float den = 0.f;
      for (int j = 0; j < L; ++j) { s[j] = std::exp(s[j] - m); den += s[j]; }
      const float inv = 1.f / den;
      float* o = out + ((size_t)t * nh + h) * hd;
      for (int i0 = 0; i0 < hd; i0 += 32) {  // 4 accumulators of 8 dims
        __m256 o0 = _mm256_setzero_ps(), o1 = o0, o2 = o0, o3 = o0;
        for (int j = 0; j < L; ++j) {
          const uint16_t* vr = vc + ((size_t)kvh * n_ctx_ + j) * hd + i0;
          const __m256 p = _mm256_set1_ps(s[j] * inv);
          o0 = _mm256_fmadd_ps(p, _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i*>(vr))), o0);
          o1 = _mm256_fmadd_ps(p, _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i*>(vr + 8))), o1);
          o2 = _mm256_fmadd_ps(p, _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i*>(vr + 16))), o2);
          o3 = _mm256_fmadd_ps(p, _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i*>(vr + 24))), o3);
        }
        _mm256_storeu_ps(o + i0, o0);
        _mm256_storeu_ps(o + i0 + 8, o1);
        _mm256_storeu_ps(o + i0 + 16, o2);
        _mm256_storeu_ps(o + i0 + 24, o3);
      }
    }
}

void CpuEngine::ffn(const CpuLayer& L, float* x, int T) {
  const int d = n_embd_, F = sp_.F_l;
  std::vector<float> part((size_t)T * d, 0.f);
  if (n_expert_ == 0) {
    std::vector<float> gu((size_t)T * 2 * F), h((size_t)T * F);
    matmul(L.w_gu, x, T, d, gu.data(), 2 * F, &L.ffn_norm, false);
    for (int t = 0; t < T; ++t)
      for (int f = 0; f < F; ++f) {
        const int r = (f >> 5) * 64 + (f & 31);
        h[(size_t)t * F + f] = silu(gu[(size_t)t * 2 * F + r]) * gu[(size_t)t * 2 * F + r + 32];
      }
    matmul(L.w_down, h.data(), T, F, part.data(), d, nullptr, false);
  } else {
    const int E = n_expert_;
    std::vector<float> rl((size_t)T * E);
    matmul(L.router, x, T, d, rl.data(), E, &L.ffn_norm, false);
    Q8 xq;
    quantize_rows(x, T, d, d, &L.ffn_norm, eps_, xq);
    for (int t = 0; t < T; ++t) {
      std::vector<double> p(E);
      double mx = -1e300, sum = 0;
      for (int e = 0; e < E; ++e) mx = std::max(mx, (double)rl[(size_t)t * E + e]);
      for (int e = 0; e < E; ++e) { p[e] = std::exp(rl[(size_t)t * E + e] - mx); sum += p[e]; }
      std::vector<int> ids(E);
      std::iota(ids.begin(), ids.end(), 0);
      std::stable_sort(ids.begin(), ids.end(), [&](int a, int b) { return p[a] > p[b]; });
      double wsum = 0;
      for (int j = 0; j < n_expert_used_; ++j) wsum += p[ids[j]] / sum;
      Q8 one;
      one.K = d;
      one.q.assign(xq.q.begin() + (size_t)t * d, xq.q.begin() + (size_t)(t + 1) * d);
      one.d.assign(xq.d.begin() + (size_t)t * d / 32, xq.d.begin() + (size_t)(t + 1) * d / 32);
      one.s16.assign(xq.s16.begin() + (size_t)t * d / 16, xq.s16.begin() + (size_t)(t + 1) * d / 16);
      for (int j = 0; j < n_expert_used_; ++j) {
        const int e = ids[j];
        const float w = (float)(p[e] / sum / wsum);
        std::vector<float> gu(2 * F), h(F), y(d);
        gemm_rows(L.gu_exps, L.gu_exps.data.data() + L.gu_exps.expert_stride * e, one, 1, gu.data(), 2 * F, false);
        for (int f = 0; f < F; ++f) {
          const int r = (f >> 5) * 64 + (f & 31);
          h[f] = silu(gu[r]) * gu[r + 32];
        }
        Q8 hq;
        quantize_rows(h.data(), 1, F, F, nullptr, eps_, hq);
        gemm_rows(L.down_exps, L.down_exps.data.data() + L.down_exps.expert_stride * e, hq, 1, y.data(), d, false);
        for (int i = 0; i < d; ++i) part[(size_t)t * d + i] += w * y[i];
      }
    }
  }
  reduce(part.data(), part.size());
  for (size_t i = 0; i < part.size(); ++i) x[i] += part[i];
}

void CpuEngine::run_layers(float* x, int T, int pos0, int l0, int l1) {
  if (l1 > layer_end_) throw std::runtime_error("run_layers: layer range not resident on the CPU");
  if (pos0 + T > n_ctx_) throw std::runtime_error("run_layers: exceeds n_ctx");
  const int d = n_embd_, hd = head_dim_;
  const int nq = sp_.nq, nkv = sp_.nkvd, nkvh = sp_.nkv_l;
  std::vector<float> q((size_t)T * nq), k((size_t)T * nkv), v((size_t)T * nkv), att((size_t)T * nq);
  std::vector<float> part((size_t)T * d);
  for (int l = l0; l < l1; ++l) {
    const CpuLayer& L = layers_[l];
    Q8 xq;
    quantize_rows(x, T, d, d, &L.attn_norm, eps_, xq);
    gemm_rows(L.wq, L.wq.data.data(), xq, T, q.data(), nq, false);
    gemm_rows(L.wk, L.wk.data.data(), xq, T, k.data(), nkv, false);
    gemm_rows(L.wv, L.wv.data.data(), xq, T, v.data(), nkv, false);
    for (int t = 0; t < T; ++t) {
      const int pos = pos0 + t;
      auto rope = [&](float* r, int n) {
        for (int i = 0; i < n; i += 2) {
          const int dd = i % hd;
          const float c = rope_cos_[(size_t)pos * hd / 2 + dd / 2], sn = rope_sin_[(size_t)pos * hd / 2 + dd / 2];
          const float a0 = r[i], a1 = r[i + 1];
          r[i] = a0 * c - a1 * sn;
          r[i + 1] = a0 * sn + a1 * c;
        }
      };
      rope(q.data() + (size_t)t * nq, nq);
      rope(k.data() + (size_t)t * nkv, nkv);
      for (int i = 0; i < nkv; ++i) {
        const size_t ci = (((size_t)l * nkvh + i / hd) * n_ctx_ + pos) * hd + i % hd;
        kc_[ci] = f2h(k[(size_t)t * nkv + i]);
        vc_[ci] = f2h(v[(size_t)t * nkv + i]);
      }
    }
    attention(l, q.data(), T, pos0, att.data());
    matmul(L.wo, att.data(), T, nq, part.data(), d, nullptr, false);
    reduce(part.data(), part.size());
    for (size_t i = 0; i < part.size(); ++i) x[i] += part[i];
    ffn(L, x, T);
  }
}

void CpuEngine::head(const float* xrow, float* logits) {
  if (!opt_.load_head) throw std::runtime_error("head: output layer not resident on the CPU");
  if (sp_.tp == 1) {
    matmul(output_, xrow, 1, n_embd_, logits, n_vocab_, &out_norm_, false);
    return;
  }
  std::vector<float> loc(sp_.V_l), all(sp_.V_pad);
  matmul(output_, xrow, 1, n_embd_, loc.data(), sp_.V_l, &out_norm_, false);
  if (!allgather_) throw std::runtime_error("tensor parallel CPU engine: set_comm() was not called");
  allgather_(loc.data(), all.data(), (size_t)sp_.V_l);
  std::memcpy(logits, all.data(), sizeof(float) * n_vocab_);
}

std::vector<float> CpuEngine::eval_logits(const std::vector<int>& tokens, int pos0) {
  const int T = (int)tokens.size();
  if (T <= 0 || pos0 + T > n_ctx_) throw std::runtime_error("eval_logits: bad range");
  std::vector<float> x;
  for (int p = 0; p < T; p += n_batch_) {
    const int n = std::min(n_batch_, T - p);
    x.assign((size_t)n * n_embd_, 0.f);
    embed(tokens.data() + p, n, x.data());
    run_layers(x.data(), n, pos0 + p, 0, n_layer_);
  }
  std::vector<float> logits(n_vocab_);
  const int last = (T - 1) % n_batch_;
  head(x.data() + (size_t)last * n_embd_, logits.data());
  return logits;
}

void CpuEngine::kv_transfer(void* buf, int n, bool load) {
  if (n < 0 || n > n_ctx_) throw std::runtime_error("kv_transfer: n out of range");
  const size_t hd = head_dim_, rows = kc_.size() / ((size_t)n_ctx_ * hd);
  uint16_t* b = static_cast<uint16_t*>(buf);
  for (int which = 0; which < 2; ++which) {
    std::vector<uint16_t>& cache = which == 0 ? kc_ : vc_;
    uint16_t* packed = b + (size_t)which * rows * n * hd;
    for (size_t r = 0; r < rows; ++r) {
      uint16_t* c = cache.data() + r * n_ctx_ * hd;
      uint16_t* p = packed + r * n * hd;
      if (load) std::memcpy(c, p, (size_t)n * hd * 2);
      else std::memcpy(p, c, (size_t)n * hd * 2);
    }
  }
}

std::vector<float> CpuEngine::eval_hidden(const std::vector<int>& tokens, int pos0) {
  const int T = (int)tokens.size();
  if (T <= 0 || pos0 + T > n_ctx_) throw std::runtime_error("eval_hidden: bad range");
  std::vector<float> out((size_t)T * n_embd_);
  for (int p = 0; p < T; p += n_batch_) {
    const int n = std::min(n_batch_, T - p);
    float* x = out.data() + (size_t)p * n_embd_;
    embed(tokens.data() + p, n, x);
    run_layers(x, n, pos0 + p, 0, layer_end_);
  }
  return out;
}

CpuGenOut CpuEngine::generate(const std::vector<int>& prompt, int n_keep, int max_new, const CpuSampling& sp,
                              const std::vector<int>& stop, const std::function<bool()>& poll,
                              const std::function<void(int)>& on_token) {
  CpuGenOut out;
  const int n_prompt = (int)prompt.size();
  if (n_prompt >= n_ctx_) throw std::runtime_error("prompt exceeds context window");
  if (n_keep < 0 || n_keep >= n_prompt) n_keep = 0;
  const double t0 = now_s();
  std::vector<int> suffix(prompt.begin() + n_keep, prompt.end());
  std::vector<float> logits = eval_logits(suffix, n_keep);
  const double t1 = now_s();
  out.prefill_s = t1 - t0;
  out.n_prefilled = n_prompt - n_keep;
  std::vector<int> hist(prompt);
  out.finish = "length";
  std::vector<float> x(n_embd_);
  for (int step = 0; step < max_new; ++step) {
    if (poll && poll()) { out.finish = "cancelled"; break; }
    const int w0 = std::max(0, (int)hist.size() - std::max(sp.last_n, 0));
    std::vector<int> window(hist.begin() + w0, hist.end());
    const int tok = cpu_sample(logits, window, sp, step);
    out.tokens.push_back(tok);
    hist.push_back(tok);
    if (on_token) on_token(tok);
    if (std::find(stop.begin(), stop.end(), tok) != stop.end()) { out.finish = "stop"; break; }
    const int pos = (int)hist.size() - 1;
    if (step + 1 == max_new || pos >= n_ctx_) break;
    embed(&tok, 1, x.data());
    run_layers(x.data(), 1, pos, 0, n_layer_);
    head(x.data(), logits.data());
  }
  out.decode_s = now_s() - t1;
  out.n_evaluated = n_prompt + std::max(0, (int)out.tokens.size() - 1);
  return out;
}

}  // namespace lfk
