// Exact-fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32): the MatMul of
// the reference's fp32 MNIST MLP (/root/reference/distribute_training.py:54,61 — tf.layers.dense
// in float32 — forward F1/F5 and backward G3/G4 of SURVEY.md §2.6) and ttd.nn.dense on fp32
// tensors. gfx950 has no xf32/TF32 mode; the f32 MFMA is a k-ordered fmaf chain, so results
// match a CPU fp32 GEMM to rounding-order level (cdna_hip_programming.md §3 "FP32-input MFMA").
//
// C[M,N] = op(A) . op(B) (+ bias[N]) (+ C when beta), op = optional transpose (the NN / TN / NT
// products of a dense layer's forward, weight gradient and data gradient). 64 x 64 output tile,
// 4 waves (2 x 2, 32 x 32 each), K-steps of 16 staged through LDS as [k][m] / [k][n] so every
// lane's MFMA operand is one float at a fixed stride; loads are coalesced along whichever
// dimension is contiguous in memory. The MLP's GEMMs are tiny (<= 128 x 784 x 200): this kernel
// is sized for exactness and few launches, not for the large-GEMM roofline.
#include "common.h"

namespace ttdk {
namespace {

constexpr int F_BM = 64, F_BN = 64, F_BK = 16, F_THR = 256;

typedef __attribute__((ext_vector_type(16))) float f32x16_v;

// element (row, k) of op(X) where X is row-major with leading dimension ld:
// not transposed: X[row][k] = p[row*ld + k]; transposed: X^T[row][k] = p[k*ld + row]
__device__ __forceinline__ float ld_op(const float* __restrict__ p, long long ld, bool tr, int row, int k, int rows,
                                       int K) {
  if (row >= rows || k >= K) return 0.f;
  return tr ? p[static_cast<long long>(k) * ld + row] : p[static_cast<long long>(row) * ld + k];
}

__global__ __launch_bounds__(F_THR) void gemm_f32_kernel(const float* __restrict__ A, long long lda, int ta,
                                                          const float* __restrict__ B, long long ldb, int tb,
                                                          float* __restrict__ C, long long ldc, const float* __restrict__ bias,
                                                          int beta, int M, int N, int K, long long sa = 0,
                                                          long long sb = 0, long long sc = 0) {
  // strided batch (tf.matmul on rank > 2 operands): entry blockIdx.z at element offsets z * s*
  A += blockIdx.z * sa;
  B += blockIdx.z * sb;
  C += blockIdx.z * sc;
  __shared__ float sA[F_BK][F_BM + 1];
  __shared__ float sB[F_BK][F_BN + 1];
  const int m0 = blockIdx.y * F_BM, n0 = blockIdx.x * F_BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  f32x16_v acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  // op(A) is M x K, op(B) is K x N: B element (k, n) = op(B)[k][n]; with tb the stored matrix is
  // [N][K] (B^T row-major), else [K][N]
  for (int k0 = 0; k0 < K; k0 += F_BK) {
#pragma unroll
    for (int e = 0; e < (F_BM * F_BK) / F_THR; ++e) {
      const int q = e * F_THR + tid;
      // coalesce along the contiguous dimension: A not transposed -> k fastest; transposed -> m fastest
      int mm, kk;
      if (ta) { mm = q % F_BM; kk = q / F_BM; } else { kk = q % F_BK; mm = q / F_BK; }
      sA[kk][mm] = ld_op(A, lda, ta != 0, m0 + mm, k0 + kk, M, K);
      int nn, kb;
      if (tb) { kb = q % F_BK; nn = q / F_BK; } else { nn = q % F_BN; kb = q / F_BN; }
      // op(B)[k][n]: stored [K][N] (tb = 0) or [N][K] (tb = 1)
      float v = 0.f;
      if (n0 + nn < N && k0 + kb < K)
        v = tb ? B[static_cast<long long>(n0 + nn) * ldb + k0 + kb] : B[static_cast<long long>(k0 + kb) * ldb + n0 + nn];
      sB[kb][nn] = v;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < F_BK; ks += 2) {
      // v_mfma_f32_32x32x2_f32: lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]
      const float a = sA[ks + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = sB[ks + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // D layout (dtype independent on gfx950): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= N) return;
  const float bv = bias ? bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < M) {
      float* o = C + static_cast<long long>(m) * ldc + n;
      *o = acc[r] + bv + (beta ? *o : 0.f);
    }
  }
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

// C[M,N] (row stride ldc) = op(A) . op(B) (+ bias) (+ C if beta); ta/tb: A stored [K][M] / B
// stored [N][K]. All fp32, exact f32 products (f32 MFMA).
TTDK_EXPORT int ttdk_gemm_f32(const float* A, long long lda, int ta, const float* B, long long ldb, int tb, float* C,
                              long long ldc, const float* bias, int beta, int M, int N, int K, hipStream_t st) {
  if (M <= 0 || N <= 0 || K < 0) return hipErrorInvalidValue;
  dim3 grid(ceil_div(N, F_BN), ceil_div(M, F_BM));
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(F_THR), 0, st, A, lda, ta, B, ldb, tb, C, ldc, bias, beta, M, N, K);
  return hipGetLastError();
}

// Strided-batched form: `batch` GEMMs in one launch (entry z reads A + z*sa, B + z*sb, writes
// C + z*sc; element strides). The batched MatMul of ttd.nn.matmul on rank > 2 fp32 operands.
TTDK_EXPORT int ttdk_gemm_f32_batched(const float* A, long long lda, long long sa, int ta, const float* B, long long ldb,
                                      long long sb, int tb, float* C, long long ldc, long long sc, int M, int N, int K,
                                      int batch, hipStream_t st) {
  if (M <= 0 || N <= 0 || K < 0 || batch <= 0 || batch > 65535) return hipErrorInvalidValue;
  dim3 grid(ceil_div(N, F_BN), ceil_div(M, F_BM), batch);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(F_THR), 0, st, A, lda, ta, B, ldb, tb, C, ldc, nullptr, 0, M, N, K, sa,
                     sb, sc);
  return hipGetLastError();
}
