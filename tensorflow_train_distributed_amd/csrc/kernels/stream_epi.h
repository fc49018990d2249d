// Epilogue pieces shared by the persistent streaming conv kernels (pw_gemm.hip, conv3_halo.hip):
// accumulators of v_mfma_f32_16x16x32_bf16 with swapped operands (D = B.A^T, so each lane holds
// 4 consecutive output columns of one row) staged to LDS as bf16 rows, and the per-tile
// reduction of the BatchNorm partial statistics gathered by epi_rows (gemm_conv.h).
#pragma once

#include "gemm_conv.h"

namespace ttdk {
namespace {
namespace sepi {

// acc[a][c] is the 16x16 block (rows wm*WR + a*16.., cols wn*WC + c*16..) of the tile
template <int TM, int TN, int WR, int WC, int PITCH>
__device__ __forceinline__ void stage_acc(char* sS, const f32x4_t (&acc)[TM][TN], int wm, int wn, int lane,
                                          float alpha) {
  const int gq4 = lane >> 4, i16 = lane & 15;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int c = 0; c < TN; ++c) {
      const int r = wm * WR + a * 16 + i16, cc = wn * WC + c * 16 + 4 * gq4;
      const f32x4_t v = acc[a][c] * alpha;
      *reinterpret_cast<uint2*>(sS + r * PITCH + cc * 2) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
}

// Fold the per-thread column sums (thread owns 16-B chunk c of every RPP-th row) into one
// [2][N] row of E.stat (and E.stat2) for tile t. `red` needs NW*3*BN floats of LDS. Ends with
// the block synchronised.
template <int BN, int NW, int THR, int ECPR>
__device__ __forceinline__ void tile_stats(const EpiParams& E, float* red, float (&s8)[8], float (&q8)[8],
                                           float (&r8)[8], int c, int lane, int wave, int tid, int n0, int N, long long t) {
  static_assert(ECPR <= 64, "one chunk column per lane group");
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int o = ECPR; o < 64; o <<= 1) {
      s8[j] += __shfl_xor(s8[j], o, 64);
      q8[j] += __shfl_xor(q8[j], o, 64);
      if (E.stat2) r8[j] += __shfl_xor(r8[j], o, 64);
    }
  }
  if (lane < ECPR) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wave * 3 + 0) * BN + c * 8 + j] = s8[j];
      red[(wave * 3 + 1) * BN + c * 8 + j] = q8[j];
      red[(wave * 3 + 2) * BN + c * 8 + j] = r8[j];
    }
  }
  __syncthreads();
  for (int t2 = tid; t2 < BN; t2 += THR) {
    if (n0 + t2 < N) {
      float ss = 0.f, qq = 0.f, rr = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        ss += red[(k * 3 + 0) * BN + t2];
        qq += red[(k * 3 + 1) * BN + t2];
        rr += red[(k * 3 + 2) * BN + t2];
      }
      E.stat[(t * 2 + 0) * N + n0 + t2] = ss;
      E.stat[(t * 2 + 1) * N + n0 + t2] = qq;
      if (E.stat2) {
        E.stat2[(t * 2 + 0) * N + n0 + t2] = ss;
        E.stat2[(t * 2 + 1) * N + n0 + t2] = rr;
      }
    }
  }
  __syncthreads();
}

}  // namespace sepi
}  // namespace
}  // namespace ttdk
