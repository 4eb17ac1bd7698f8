#include "repack.h"

#include <cstring>
#include <stdexcept>

#include "../common.h"

namespace lfk {

void repack_planar(int type, const uint8_t* src, size_t K_src, size_t r0, size_t R, size_t c0, size_t K,
                   uint8_t* dst, size_t R_dst, int G, int off) {
  const TypeInfo ti = type_info(type);
  if (K % ti.block || c0 % ti.block || K_src % ti.block) throw std::runtime_error("repack: unaligned column slice");
  const size_t nb_src = K_src / ti.block, nb = K / ti.block, b0 = c0 / ti.block;
  const Planes P = planes_of(type, R_dst, K);
  switch (type) {
    case T_Q4_K: case T_Q5_K: case T_Q6_K: case T_Q8_0: case T_F16: case T_BF16: case T_F32: break;
    default: throw std::runtime_error("repack: unsupported type");
  }
#pragma omp parallel for schedule(static)
  for (long long ii = 0; ii < (long long)R; ++ii) {
    const size_t i = (size_t)ii;
    const size_t dr = G > 0 ? (i / G) * 2 * G + off + i % G : off + i;
    const uint8_t* srow = src + ((r0 + i) * nb_src + b0) * ti.bytes;
    switch (type) {
      case T_Q4_K:
        for (size_t b = 0; b < nb; ++b) {
          const uint8_t* blk = srow + b * 144;
          std::memcpy(dst + P.p1 + dr * P.s1 + b * 16, blk, 16);
          std::memcpy(dst + P.p0 + dr * P.s0 + b * 128, blk + 16, 128);
        }
        break;
      case T_Q5_K:
        for (size_t b = 0; b < nb; ++b) {
          const uint8_t* blk = srow + b * 176;
          std::memcpy(dst + P.p2 + dr * P.s2 + b * 16, blk, 16);
          std::memcpy(dst + P.p1 + dr * P.s1 + b * 32, blk + 16, 32);
          std::memcpy(dst + P.p0 + dr * P.s0 + b * 128, blk + 48, 128);
        }
        break;
      case T_Q6_K:
        for (size_t b = 0; b < nb; ++b) {
          const uint8_t* blk = srow + b * 210;
          std::memcpy(dst + P.p0 + dr * P.s0 + b * 128, blk, 128);
          std::memcpy(dst + P.p1 + dr * P.s1 + b * 64, blk + 128, 64);
          std::memcpy(dst + P.p2 + dr * P.s2 + b * 16, blk + 192, 16);
          std::memcpy(dst + P.p3 + dr * P.s3 + b * 2, blk + 208, 2);
        }
        break;
      case T_Q8_0:
        for (size_t b = 0; b < nb; ++b) {
          const uint8_t* blk = srow + b * 34;
          std::memcpy(dst + P.p1 + dr * P.s1 + b * 2, blk, 2);
          std::memcpy(dst + P.p0 + dr * P.s0 + b * 32, blk + 2, 32);
        }
        break;
      case T_F16:
      case T_BF16:
        std::memcpy(dst + dr * P.s0, srow, K * 2);
        break;
      case T_F32:
        std::memcpy(dst + dr * P.s0, srow, K * 4);
        break;
      default:
        break;
    }
  }
}

}  // namespace lfk
