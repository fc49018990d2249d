// Forward convolution (bf16 and fp8 block-scaled MFMA) and the fp8 GEMM; kernels in gemm_conv.h.
#include "gemm_conv.h"

// bm == 256 requests the LDS-DMA kernel (bn = its tile width 256 or 128; the caller sized
// `stat` for 256-row tiles); the request fails loudly when the conv is not eligible.
TTDK_EXPORT int ttdk_conv_fwd(const bf16_t* x, const bf16_t* w, const TtdkConv* g, int bm, int bn,
                              const TtdkEpilogue* epi, hipStream_t st) {
  if (g->C % 8) return hipErrorInvalidValue;
  EpiParams pe = to_epi(epi);
  const int M = g->N * g->P * g->Q, N = g->K, K = g->R * g->S * g->C;
  if (bm == 256) {
    const int bbn = big_bn(M, N, K);
    if (!bbn || bbn != bn || pe.remap || g->C % 64) return hipErrorInvalidValue;
    if (is_pointwise(g)) return bbn == 256 ? big::dense<256>(x, g->C, true, w, K, true, pe, M, N, K, 1, st)
                                           : big::dense<128>(x, g->C, true, w, K, true, pe, M, N, K, 1, st);
    const big::ConvP pa = conv_params(x, g->H, g->W, g->C, g->P, g->Q, g, M);
    const big::DenseP pb{w, K, N};
    if (bbn == 256)
      return big::launch<256, big::OpConvK<128, 2, false>, big::OpDenseK<128, 2>>(pa, pb, pe, M, N, K, 1, st);
    return big::launch<128, big::OpConvK<128, 2, false>, big::OpDenseK<64, 2>>(pa, pb, pe, M, N, K, 1, st);
  }
  if (bm == 0 || bn == 0) pick_tile(M, N, &bm, &bn);
  DenseParams pb{w, K, N, K};
  if (is_pointwise(g)) {
    DenseParams pa{x, g->C, M, K};
    return dispatch<KDense, KDense>(&pa, &pb, pe, M, N, K, 1, bm, bn, st);
  }
  GatherParams pa{x, g->H, g->W, g->C, g->P, g->Q, g->R, g->S, g->sh, g->sw, g->ph, g->pw, g->dh, g->dw, M, K};
  return dispatch<KConvFwd, KDense>(&pa, &pb, pe, M, N, K, 1, bm, bn, st);
}

// Pointwise (1x1, stride 1) forward conv whose input is the RAW conv output y3 of the previous
// conv+BN+residual+ReLU unit: the 256-row kernel forms that unit's output
// h = relu(sc*y3 + sh + r) (r = the residual, or rsc*r + rsh with `proj`) in LDS as its operand
// and stores h + its ReLU bits (tile column 0) — the unit's BN apply pass disappears.
// coef = [sc | sh (| rsc | rsh)] fp32 [2 or 4][C]. hipErrorNotSupported when the shape is not on
// the 256-row kernel (the caller keeps the pass). `stat` rows are 256-row tiles.
TTDK_EXPORT int ttdk_conv_fwd_bnpro(const bf16_t* y3, const bf16_t* w, const TtdkConv* g, const bf16_t* res,
                                    const float* coef, int proj, bf16_t* h_out, uint8_t* mask_out,
                                    const TtdkEpilogue* epi, hipStream_t st) {
  if (!is_pointwise(g) || !res || !h_out || !mask_out) return hipErrorNotSupported;
  EpiParams pe = to_epi(epi);
  const int M = g->N * g->P * g->Q, N = g->K, K = g->C;
  const int bbn = big_bn(M, N, K);
  if (!bbn || K % 64 || pe.remap || pe.mode != 0) return hipErrorNotSupported;
  pe.py = res;
  pe.pcoef = coef;
  pe.pdz = h_out;
  pe.pmask = mask_out;
  pe.pld = K;
  const big::DenseP pa{y3, K, M}, pb{w, K, N};
  if (proj) {
    if (bbn == 256)
      return big::launch<256, big::OpDenseKBN<128, 2, big::THR, 3>, big::OpDenseK<128, 2>, 0, 0>(pa, pb, pe, M, N, K, 1, st);
    return big::launch<128, big::OpDenseKBN<128, 2, big::THR, 3>, big::OpDenseK<64, 2>, 0, 0>(pa, pb, pe, M, N, K, 1, st);
  }
  if (bbn == 256)
    return big::launch<256, big::OpDenseKBN<128, 2, big::THR, 2>, big::OpDenseK<128, 2>, 0, 0>(pa, pb, pe, M, N, K, 1, st);
  return big::launch<128, big::OpDenseKBN<128, 2, big::THR, 2>, big::OpDenseK<64, 2>, 0, 0>(pa, pb, pe, M, N, K, 1, st);
}

// fp8 forward conv / GEMM on the block-scaled MFMA: x8 [N,H,W,C] and w8 [K][R][S][C] in fp8
// e4m3 (per-tensor scales folded into epi->alpha by the caller). C % 128 == 0, 256-row tiles.
TTDK_EXPORT int ttdk_conv_fwd_fp8(const uint8_t* x8, const uint8_t* w8, const TtdkConv* g, int bn,
                                  const TtdkEpilogue* epi, hipStream_t st) {
  EpiParams pe = to_epi(epi);
  const int M = g->N * g->P * g->Q, N = g->K, K = g->R * g->S * g->C;
  const int bbn = N >= 256 ? 256 : 128;  // fp8 always runs the LDS-DMA kernel (edges are clamped)
  if (bbn != bn || g->C % 128 || pe.remap || M < 1) return hipErrorInvalidValue;
  const big::DenseP pb{w8, K, N};
  if (is_pointwise(g)) {
    const big::DenseP pa{x8, g->C, M};
    if (bbn == 256) return big::launch<256, big::OpDenseK<128, 1>, big::OpDenseK<128, 1>, 1>(pa, pb, pe, M, N, K, 1, st);
    return big::launch<128, big::OpDenseK<128, 1>, big::OpDenseK<64, 1>, 1>(pa, pb, pe, M, N, K, 1, st);
  }
  const big::ConvP pa = conv_params(x8, g->H, g->W, g->C, g->P, g->Q, g, M);
  if (bbn == 256) return big::launch<256, big::OpConvK<128, 1, false>, big::OpDenseK<128, 1>, 1>(pa, pb, pe, M, N, K, 1, st);
  return big::launch<128, big::OpConvK<128, 1, false>, big::OpDenseK<64, 1>, 1>(pa, pb, pe, M, N, K, 1, st);
}

// fp8 GEMM C[M,N] = A[M,K] . B[N,K]^T (both K-major fp8; a_fmt 0 = e4m3, 1 = e5m2; B e4m3),
// K % 128 == 0, fused bf16 epilogue or fp32 (split-K slab) output like ttdk_gemm_bf16.
TTDK_EXPORT int ttdk_gemm_fp8(const uint8_t* A, long long lda, const uint8_t* B, long long ldb, int a_fmt, int M,
                              int N, int K, int splits, const TtdkEpilogue* epi, hipStream_t st) {
  EpiParams pe = to_epi(epi);
  const int bbn = N >= 256 ? 256 : 128;  // fp8 always runs the LDS-DMA kernel (edges are clamped)
  if (M < 1 || N < 1 || K % 128 || lda % 16 || ldb % 16 || pe.remap) return hipErrorInvalidValue;
  const big::DenseP pa{A, lda, M}, pb{B, ldb, N};
#define TTDK_F8(BN_, BH_, F_) \
  return big::launch<BN_, big::OpDenseK<128, 1>, big::OpDenseK<BH_, 1>, F_>(pa, pb, pe, M, N, K, splits, st)
  if (bbn == 256) {
    if (a_fmt) TTDK_F8(256, 128, 2);
    TTDK_F8(256, 128, 1);
  }
  if (a_fmt) TTDK_F8(128, 64, 2);
  TTDK_F8(128, 64, 1);
#undef TTDK_F8
}

// fp8 data gradient of a unit-stride conv on the block-scaled MFMA: dy8 [N,P,Q,K] in OCP e5m2
// (gradients), wt8 = the filter transposed to [C][R][S][K] in e4m3; dx = dequant (epi.ascale0 x
// epi.ascale1) of the implicit-GEMM gather, with the bf16 path's epilogues (accumulate, next BN's
// masked gradient + backward statistics on 256-row tiles). K % 128 == 0 (one 128-element K-tile
// inside one tap).
TTDK_EXPORT int ttdk_conv_dgrad_fp8(const uint8_t* dy8, const uint8_t* wt8, const TtdkConv* g, const TtdkEpilogue* epi,
                                    hipStream_t st) {
  if (g->sh != 1 || g->sw != 1 || g->dh != 1 || g->dw != 1 || g->K % 128 || g->C % 8) return hipErrorInvalidValue;
  EpiParams pe = to_epi(epi);
  if (pe.remap || pe.residual || pe.bH || pe.by2 || pe.mode != 0) return hipErrorInvalidValue;
  if (pe.by && (pe.stat == nullptr || pe.ldo % 8 || pe.act)) return hipErrorInvalidValue;
  const int N = g->C, K = g->R * g->S * g->K;
  const int M = g->N * g->H * g->W;
  const big::DenseP pb{wt8, K, N};
  if (is_pointwise(g)) {
    // 1x1: dy8 is the dense K-major A operand (no per-row gather addressing)
    const big::DenseP pd{dy8, g->K, M};
    if (N >= 256) return big::launch<256, big::OpDenseK<128, 1>, big::OpDenseK<128, 1>, 2>(pd, pb, pe, M, N, K, 1, st);
    return big::launch<128, big::OpDenseK<128, 1>, big::OpDenseK<64, 1>, 2>(pd, pb, pe, M, N, K, 1, st);
  }
  const big::ConvP pa = conv_params(dy8, g->P, g->Q, g->K, g->H, g->W, g, M);
  if (N >= 256) return big::launch<256, big::OpConvK<128, 1, true, true>, big::OpDenseK<128, 1>, 2>(pa, pb, pe, M, N, K, 1, st);
  return big::launch<128, big::OpConvK<128, 1, true, true>, big::OpDenseK<64, 1>, 2>(pa, pb, pe, M, N, K, 1, st);
}
