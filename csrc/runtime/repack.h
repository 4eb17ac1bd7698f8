// GGUF block layout -> planar layout (../common.h), with row/column slicing for
// tensor-parallel shards and gate/up row interleaving.
#pragma once
#include <cstddef>
#include <cstdint>

namespace lfk {

// Copy rows [r0, r0+R) x columns [c0, c0+K) of a ggml matrix whose rows hold
// K_src weights into the planar matrix `dst` (R_dst rows, K columns).
// Source row i lands on destination row  G>0 ? (i/G)*2G + off + i%G : off + i
// (G>0 interleaves two matrices in G-row groups: gate rows at off=0, up at off=G).
// c0 and K must be multiples of the type's block size. Multi-threaded (OpenMP).
void repack_planar(int type, const uint8_t* src, size_t K_src, size_t r0, size_t R, size_t c0, size_t K,
                   uint8_t* dst, size_t R_dst, int G, int off);

}  // namespace lfk
