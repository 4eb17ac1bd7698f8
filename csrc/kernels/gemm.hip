// Prefill GEMM on MFMA with LDS-staged, dequantised weight tiles:
//   Y[T][N] = X[T][K] (bf16) . W[N][K]^T (Q4_K/Q5_K/Q6_K/Q8_0/F16/F32, planar)
//
// Replaces upstream's "dequantise to f16 + cublasGemmEx" / MMQ with one kernel
// and no vendor BLAS: each 256-thread block owns a 64 (tokens) x 128 (weight
// rows) tile; per 64-deep K step the block
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

#include "kernels.h"
#include "qdot.h"

namespace lfk {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

static constexpr int BM = 64, BN = 128, BK = 64, PITCH = BK + 8;  // bf16 elements

__device__ __forceinline__ unsigned short f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<unsigned short*>(&b);
}

template <int QT, int EPI>
__global__ __launch_bounds__(256) void gemm_dq_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Xs[BM * PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short Ws[BN * PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int N = a.w.rows, K = a.w.K, T = a.T;
  f32x16 acc[2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;

  const int wrow = tid >> 1, whalf = tid & 1;
  const unsigned short* xg = reinterpret_cast<const unsigned short*>(a.x);
  for (int k0 = 0; k0 < K; k0 += BK) {
    // ---- stage X: 64 rows x 64 bf16 = 512 x 16 B
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i;
      const int r = idx >> 3, c = idx & 7;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m0 + r < T) v = *reinterpret_cast<const uint4*>(xg + (size_t)(m0 + r) * K + k0 + 8 * c);
      *reinterpret_cast<uint4*>(&Xs[r * PITCH + 8 * c]) = v;
    }
    // ---- stage W: decode 32 weights per thread into bf16
    {
      float w[32];
      if (n0 + wrow < N) {
        dequant32<QT>(a.w.base, a.w.P, (size_t)(n0 + wrow), (k0 >> 5) + whalf, w);
      } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) w[i] = 0.f;
      }
      uint4* dst = reinterpret_cast<uint4*>(&Ws[wrow * PITCH + 32 * whalf]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint4 p;
        p.x = f2bf(w[8 * i + 0]) | ((unsigned)f2bf(w[8 * i + 1]) << 16);
        p.y = f2bf(w[8 * i + 2]) | ((unsigned)f2bf(w[8 * i + 3]) << 16);
        p.z = f2bf(w[8 * i + 4]) | ((unsigned)f2bf(w[8 * i + 5]) << 16);
        p.w = f2bf(w[8 * i + 6]) | ((unsigned)f2bf(w[8 * i + 7]) << 16);
        dst[i] = p;
      }
    }
    __syncthreads();
    // ---- MFMA: 4 k-steps of 16
    const int lr = lane & 31, lk = 8 * (lane >> 5);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 16) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Ws[(32 * wave + lr) * PITCH + kk + lk]);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(&Xs[(32 * m + lr) * PITCH + kk + lk]);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, b, acc[m], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- epilogue. acc[m][r]: token = 32m + (r&3) + 8(r>>2) + 4(lane>>5), col = 32*wave + (lane&31)
  const int col = n0 + 32 * wave + (lane & 31);
  if constexpr (EPI == GEMM_SWIGLU) {
    float* ex = reinterpret_cast<float*>(Ws);  // 2 odd waves x 2 x 16 x 64 floats = 16 KiB (fits Ws)
    if (wave & 1) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) ex[(((wave >> 1) * 2 + m) * 16 + r) * 64 + lane] = acc[m][r];
    }
    __syncthreads();
    if (!(wave & 1)) {
      const int feat = ((n0 + 32 * wave) >> 6) * 32 + (lane & 31);
      const int F = N >> 1;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int t = m0 + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (t < T && feat < F) {
            const float g = acc[m][r];
            const float u = ex[(((wave >> 1) * 2 + m) * 16 + r) * 64 + lane];
            a.out_bf16[(size_t)t * F + feat] = __float2bfloat16(g / (1.f + __expf(-g)) * u);
          }
        }
    }
  } else {
    if (col < N) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int t = m0 + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (t < T) {
            float* o = a.out + (size_t)t * a.ldo + col;
            if constexpr (EPI == GEMM_ADD) *o += acc[m][r];
            else *o = a.resid ? acc[m][r] + a.resid[(size_t)t * a.ldo + col] : acc[m][r];
          }
        }
    }
  }
}

template <int QT>
static void launch_gemm(const GemmArgs& a, int epi, hipStream_t s) {
  dim3 grid((a.w.rows + BN - 1) / BN, (a.T + BM - 1) / BM), block(256);
  switch (epi) {
    case GEMM_STORE: hipLaunchKernelGGL((gemm_dq_kernel<QT, GEMM_STORE>), grid, block, 0, s, a); break;
    case GEMM_ADD: hipLaunchKernelGGL((gemm_dq_kernel<QT, GEMM_ADD>), grid, block, 0, s, a); break;
    case GEMM_SWIGLU: hipLaunchKernelGGL((gemm_dq_kernel<QT, GEMM_SWIGLU>), grid, block, 0, s, a); break;
    default: throw std::runtime_error("gemm_dq: bad epilogue");
  }
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
