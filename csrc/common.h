// Shared definitions for the MI355X (gfx950) runtime and kernels.
//
// Weight layout on the GPU ("row-planar" repack, done once at load time):
// every quantised matrix with R rows (output features) and K columns is split
// into per-field planes so each plane row is contiguous and 16-B aligned - the
// GGUF block layout (Q6_K 210 B, Q8_0 34 B) is not, which would break wide
// coalesced loads (SURVEY §2.3 "Row bytes are 16-B aligned ... blocks are not").
//
//   Q4_K : qs[R][K/256][128] | meta[R][K/256][16]   (meta = d, dmin, scales[12])
//   Q5_K : qs[R][K/256][128] | qh[R][K/256][32] | meta[R][K/256][16]
//   Q6_K : ql[R][K/256][128] | qh[R][K/256][64] | sc[R][K/256][16] | d[R][K/256] (f16)
//   Q8_0 : qs[R][K/32][32]   | d[R][K/32] (f16)
//   F16 / F32 : [R][K] unchanged
//
// Total bytes are identical to the GGUF tensor (no padding), so 4.6 GB of
// Llama-3-8B Q4_K_M weights stay 4.6 GB on HBM.
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace lfk {

enum QType : int {
  T_F32 = 0,
  T_F16 = 1,
  T_Q8_0 = 8,
  T_Q4_K = 12,
  T_Q5_K = 13,
  T_Q6_K = 14,
  T_BF16 = 30,
};

struct TypeInfo {
  int block;   // weights per block
  int bytes;   // bytes per block
};

inline TypeInfo type_info(int t) {
  switch (t) {
    case T_F32: return {1, 4};
    case T_F16: return {1, 2};
    case T_BF16: return {1, 2};
    case T_Q8_0: return {32, 34};
    case T_Q4_K: return {256, 144};
    case T_Q5_K: return {256, 176};
    case T_Q6_K: return {256, 210};
  }
  throw std::runtime_error("unsupported ggml type " + std::to_string(t));
}

inline size_t qbytes(int t, size_t rows, size_t K) {
  TypeInfo ti = type_info(t);
  return rows * (K / ti.block) * ti.bytes;
}

// Plane offsets (bytes from the matrix base) for the planar layout. Usable on host and device.
struct Planes {
  size_t p0, p1, p2, p3;  // start of plane 0..3
  size_t s0, s1, s2, s3;  // per-row stride of plane 0..3
};

#if defined(__HIPCC__)
#define LFK_HD __host__ __device__ __forceinline__
#else
#define LFK_HD inline
#endif

LFK_HD Planes planes_of(int t, size_t R, size_t K) {
  Planes p{0, 0, 0, 0, 0, 0, 0, 0};
  size_t nsb = K / 256, nb = K / 32;
  switch (t) {
    case T_Q4_K:
      p.s0 = nsb * 128; p.s1 = nsb * 16;
      p.p0 = 0; p.p1 = R * p.s0;
      break;
    case T_Q5_K:
      p.s0 = nsb * 128; p.s1 = nsb * 32; p.s2 = nsb * 16;
      p.p0 = 0; p.p1 = R * p.s0; p.p2 = p.p1 + R * p.s1;
      break;
    case T_Q6_K:
      p.s0 = nsb * 128; p.s1 = nsb * 64; p.s2 = nsb * 16; p.s3 = nsb * 2;
      p.p0 = 0; p.p1 = R * p.s0; p.p2 = p.p1 + R * p.s1; p.p3 = p.p2 + R * p.s2;
      break;
    case T_Q8_0:
      p.s0 = nb * 32; p.s1 = nb * 2;
      p.p0 = 0; p.p1 = R * p.s0;
      break;
    case T_F16: case T_BF16:
      p.s0 = K * 2; break;
    case T_F32:
      p.s0 = K * 4; break;
    default: break;
  }
  return p;
}

}  // namespace lfk
