// Prefill GEMM on MFMA with LDS-staged, dequantised weight tiles:
//   Y[T][N] = X[T][K] (bf16) . W[N][K]^T (Q4_K/Q5_K/Q6_K/Q8_0/F16/F32, planar)
//
// Replaces upstream's "dequantise to f16 + cublasGemmEx" / MMQ with one kernel
// and no vendor BLAS: each 256-thread block owns a 64 (tokens) x 128 (weight
// rows) tile (split over K when the tile grid is too small to fill the chip);
// per 64-deep K step the block
//   1. stages X (bf16) into LDS and
//   2. decodes 128 x 64 quantised weights straight into a bf16 LDS tile
//      (2 threads per weight row, 32 contiguous weights each),
//   3. runs v_mfma_f32_32x32x16_bf16: wave w owns weight rows 32w..32w+31 and
//      both 32-token halves (2 accumulators x 16 f32 per lane).
// LDS rows are padded by 16 B (row pitch 144 B) to spread ds_read_b128 banks.
// Epilogues: f32 store (optionally + residual for the TP rank that owns it),
// in-place residual add, or SwiGLU over gate/up rows interleaved in 32-row
// groups (the pair lives in adjacent waves; exchanged through LDS), bf16 out.
#include <hip/hip_bf16.h>

#include <algorithm>

#include "kernels.h"
#include "qdot.h"

namespace lfk {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

static constexpr int BM = 64, BN = 128, BK = 64, PITCH = BK + 8;  // bf16 elements

__device__ __forceinline__ uint4 pack_bf16x8(const float* w) {
  uint4 p;
  p.x = pk_bf16_pair(w[0], w[1]);
  p.y = pk_bf16_pair(w[2], w[3]);
  p.z = pk_bf16_pair(w[4], w[5]);
  p.w = pk_bf16_pair(w[6], w[7]);
  return p;
}

// Software pipeline (double-buffered LDS, one barrier per K step): the global
// loads of step k+1 (X tile + raw quantised weights) are issued before step
// k's MFMAs and decoded into the other LDS buffer after them. Split-K
// (gridDim.z > 1) partitions the K steps; partial tiles are atomically added.
// DB: double-buffered LDS (55 KB, 2 blocks/CU) for grids that fit the chip;
// single-buffered (27 KB, up to 5 blocks/CU, one extra barrier per step) for
// large grids where more resident blocks hide more latency.
// BMT: tokens per tile (64, or 128 for longer prompts: twice the MFMA work per
// decoded weight tile - the PMC profile showed 27 VALU instructions per MFMA at 64,
// the kernel VALU-bound on the weight decode).
template <int QT, int EPI, bool DB, int D = 3, int BMT = BM, int BNT = BN>
__global__ __launch_bounds__(2 * BNT) void gemm_dq_kernel(GemmArgs a) {
  constexpr int NT = 2 * BNT;  // threads: 2 per weight row of the tile, wave w owns rows 32w..32w+31
  constexpr int NBUF = DB ? 2 : 1, MT = BMT / 32, XL = BMT * 8 / NT;  // XL: 16-B X loads per thread per step
  // one LDS array (Xs buffers, then Ws buffers): the SwiGLU epilogue reuses it whole
  __shared__ __attribute__((aligned(16))) unsigned short lds[NBUF * (BMT + BNT) * PITCH];
  auto Xs = [&](int b) { return lds + b * BMT * PITCH; };
  auto Ws = [&](int b) { return lds + NBUF * BMT * PITCH + b * BNT * PITCH; };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * BNT, m0 = blockIdx.y * BMT;
  if (a.seg_dev) {  // grouped form: this expert's rows of the gathered buffers
    const int r0 = a.seg_dev[0];
    a.T = a.seg_dev[1] - r0;
    if (m0 >= a.T) return;  // whole block, before any barrier
    a.x += (size_t)r0 * a.w.K;
    if (a.out) a.out += (size_t)r0 * a.ldo;
    if (a.out_bf16) a.out_bf16 += (size_t)r0 * (a.w.rows >> 1);
  }
  const int N = a.w.rows, K = a.w.K, T = a.T;
  const int nk = K / BK, ks = (nk + gridDim.z - 1) / gridDim.z;
  const int kb = blockIdx.z * ks, ke = min(nk, kb + ks);
  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;

  const int wrow = tid >> 1, whalf = tid & 1;
  const unsigned wmask = n0 + wrow < N ? ~0u : 0u;
  const size_t wr = (size_t)min(n0 + wrow, N - 1);
  const unsigned short* xg = reinterpret_cast<const unsigned short*>(a.x);
  // D-deep register prefetch ring: the global loads of step k+D go out at the start
  // of step k, so one step's load latency (~1-2 us under load) is spread over D
  // steps of MFMA work (with one stage in flight every K step was latency-bound).
  // Every load is unconditional (step and token row clamped, rows past T zeroed by
  // a select after the load): a load under a runtime branch makes hipcc drain vmcnt
  // at the join, which would serialise the ring.
  uint4 xr[D][XL];
  DqRaw<QT> raw[D];
  auto load_step = [&](int k, int st) {
    const int k0 = min(k, ke - 1) * BK;
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + NT * i;
      const int r = idx >> 3, c = idx & 7;
      xr[st][i] = *reinterpret_cast<const uint4*>(xg + (size_t)min(m0 + r, T - 1) * K + k0 + 8 * c);
    }
    dq_load<QT>(raw[st], a.w.base, a.w.P, wr, (k0 >> 5) + whalf);
  };
  auto store_step = [&](int k, int st, int buf) {
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + NT * i;
      const int r = idx >> 3, c = idx & 7;
      *reinterpret_cast<uint4*>(Xs(buf) + r * PITCH + 8 * c) = (m0 + r < T) ? xr[st][i] : make_uint4(0, 0, 0, 0);
    }
    float w[32];
    dq_decode<QT>(raw[st], ((k * BK) >> 5) + whalf, w);
    uint4* dst = reinterpret_cast<uint4*>(Ws(buf) + wrow * PITCH + 32 * whalf);
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // rows past N: AND with 0 (a select here compiles to a branch)
      const uint4 p = pack_bf16x8(w + 8 * i);
      dst[i] = make_uint4(p.x & wmask, p.y & wmask, p.z & wmask, p.w & wmask);
    }
  };
  if (kb < ke) {
#pragma unroll
    for (int j = 0; j < D; ++j) load_step(kb + j, j);
    store_step(kb, 0, 0);
  }
  __syncthreads();
  const int lr = lane & 31, lk = 8 * (lane >> 5);
  for (int k0 = kb; k0 < ke; k0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int k = k0 + j;
      load_step(k + D, j);  // stage j held step k, already in LDS: refill it (clamped past ke)
      if (k < ke) {
        const int buf = DB ? ((k - kb) & 1) : 0;
        const bool more = k + 1 < ke;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 16) {
          const bf16x8 bw = *reinterpret_cast<const bf16x8*>(Ws(buf) + (32 * wave + lr) * PITCH + kk + lk);
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8*>(Xs(buf) + (32 * m + lr) * PITCH + kk + lk);
            acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xv, bw, acc[m], 0, 0, 0);
          }
        }
        if constexpr (DB) {
          if (more) store_step(k + 1, (j + 1) % D, buf ^ 1);
          __syncthreads();
        } else {
          __syncthreads();  // every wave is done reading the single buffer
          if (more) store_step(k + 1, (j + 1) % D, 0);
          __syncthreads();
        }
      }
    }
  }

  // ---- epilogue. acc[m][r]: token = 32m + (r&3) + 8(r>>2) + 4(lane>>5), col = 32*wave + (lane&31)
  const int col = n0 + 32 * wave + (lane & 31);
  if constexpr (EPI == GEMM_SWIGLU) {
    // BNT/64 odd waves x MT x 16 x 64 floats (16 KiB at 128 x 64, 64 KiB at 256 x 128) in the whole LDS array
    static_assert((BNT / 64) * MT * 16 * 64 * 4 <= NBUF * (BMT + BNT) * PITCH * 2, "SwiGLU exchange does not fit");
    float* ex = reinterpret_cast<float*>(lds);
    __syncthreads();  // the last K step's MFMA reads of the tiles are done
    if (wave & 1) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) ex[(((wave >> 1) * MT + m) * 16 + r) * 64 + lane] = acc[m][r];
    }
    __syncthreads();
    if (!(wave & 1)) {
      const int feat = ((n0 + 32 * wave) >> 6) * 32 + (lane & 31);
      const int F = N >> 1;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int t = m0 + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (t < T && feat < F) {
            const float g = acc[m][r];
            const float u = ex[(((wave >> 1) * MT + m) * 16 + r) * 64 + lane];
            a.out_bf16[(size_t)t * F + feat] = __float2bfloat16(g / (1.f + __expf(-g)) * u);
          }
        }
    }
  } else {
    if (col < N) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int t = m0 + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (t < T) {
            float* o = a.out + (size_t)t * a.ldo + col;
            if (gridDim.z > 1) {  // split-K: partial tiles meet by atomic add (STORE outputs pre-zeroed)
              float v = acc[m][r];
              if (EPI == GEMM_STORE && a.resid && blockIdx.z == 0) v += a.resid[(size_t)t * a.ldo + col];
              atomicAdd(o, v);
            } else if constexpr (EPI == GEMM_ADD) {
              *o += acc[m][r];
            } else {
              *o = a.resid ? acc[m][r] + a.resid[(size_t)t * a.ldo + col] : acc[m][r];
            }
          }
        }
    }
  }
}

template <int QT, int BMT, int BNT>
static void launch_gemm_t(const GemmArgs& a, int epi, hipStream_t s) {
  const int rows = a.seg_dev ? std::max(1, std::min(a.T, a.rows_hint > 0 ? a.rows_hint : a.T)) : a.T;
  const int tiles = ((a.w.rows + BNT - 1) / BNT) * ((rows + BMT - 1) / BMT);
  const int nk = a.w.K / BK;
  // split K until ~2 blocks per CU are busy, keeping >= 8 K steps per split
  const int target = BNT == 256 ? 256 : 512;
  int split = 1;
  if (epi != GEMM_SWIGLU) {
    while (tiles * split < target && nk / (split * 2) >= 8) split *= 2;
  }
  if (split > 1 && epi == GEMM_STORE && !a.seg_dev && !a.out_zeroed) {
    const hipError_t e = hipMemset2DAsync(a.out, sizeof(float) * a.ldo, 0, sizeof(float) * a.w.rows, a.T, s);
    if (e != hipSuccess) throw std::runtime_error("gemm_dq: memset failed");
  }
  dim3 grid((a.w.rows + BNT - 1) / BNT, (a.T + BMT - 1) / BMT, split), block(2 * BNT);
  // 256-token or 256-row tiles are always double-buffered (110 KB of LDS, one block per CU)
  constexpr bool big = BMT == 256 || BNT == 256;
  const bool db = big || tiles * split <= 512;
  if (a.seg_dev && split > 1 && epi != GEMM_STORE) throw std::runtime_error("gemm_dq: grouped split-K needs STORE");
#define LFK_GEMM_LAUNCH(E)                                                                        \
  do {                                                                                             \
    if (db) hipLaunchKernelGGL((gemm_dq_kernel<QT, E, true, 3, BMT, BNT>), grid, block, 0, s, a);  \
    else if constexpr (!big)                                                                       \
      hipLaunchKernelGGL((gemm_dq_kernel<QT, E, false, 3, BMT, BNT>), grid, block, 0, s, a);       \
  } while (0)
  switch (epi) {
    case GEMM_STORE: LFK_GEMM_LAUNCH(GEMM_STORE); break;
    case GEMM_ADD: LFK_GEMM_LAUNCH(GEMM_ADD); break;
    case GEMM_SWIGLU: LFK_GEMM_LAUNCH(GEMM_SWIGLU); break;
    default: throw std::runtime_error("gemm_dq: bad epilogue");
  }
#undef LFK_GEMM_LAUNCH
}

// 128-token tiles once a prompt chunk (or an expert's expected rows) exceeds 64 tokens;
template <int QT>
static void launch_gemm(const GemmArgs& a, int epi, hipStream_t s) {
  const int rows = a.seg_dev ? (a.rows_hint > 0 ? a.rows_hint : a.T) : a.T;
  const int bm = rows > 64 ? 128 : 64;
  // 256-row tiles for the gate/up GEMM (measured: 124.6 -> 112.6 us at 256 tokens, 242 -> 239 at
  // 512); the split-K residual projections stay on 128-row tiles (Q6_K down is slower at 256)
  const bool wide = epi == GEMM_SWIGLU;
  if (bm >= 256) launch_gemm_t<QT, 256, 128>(a, epi, s);
  else if (bm >= 128) {
    if (wide) launch_gemm_t<QT, 128, 256>(a, epi, s);
    else launch_gemm_t<QT, 128, 128>(a, epi, s);
  } else launch_gemm_t<QT, 64, 128>(a, epi, s);
}

void gemm_dq(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.T <= 0) return;
  if (a.w.K % BK) throw std::runtime_error("gemm_dq: K must be a multiple of 64");
  if (epi == GEMM_SWIGLU && (a.w.rows % 64)) throw std::runtime_error("gemm_dq: swiglu needs 64-row groups");
  switch (a.w.type) {
    case T_Q4_K: launch_gemm<T_Q4_K>(a, epi, s); break;
    case T_Q5_K: launch_gemm<T_Q5_K>(a, epi, s); break;
    case T_Q6_K: launch_gemm<T_Q6_K>(a, epi, s); break;
    case T_Q8_0: launch_gemm<T_Q8_0>(a, epi, s); break;
    case T_F16: launch_gemm<T_F16>(a, epi, s); break;
    case T_F32: launch_gemm<T_F32>(a, epi, s); break;
    default: throw std::runtime_error("gemm_dq: unsupported weight type");
  }
}

}  // namespace lfk
