// Convolution weight gradient (split-K); kernels in gemm_conv.h.
#include "gemm_conv.h"

extern "C" int ttdk_gemm4t_wgrad(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                 int splits, float* ws, float* out, int beta, float alpha, float* rowsum,
                                 hipStream_t st);
extern "C" long long ttdk_gemm4t_ws(int M, int N, int K, int splits);

// dw[K,R,S,C] (fp32) = sum over pixels of dy ⊗ im2col(x). `ws` is a split-K workspace of
// splits*K*R*S*C floats (may be null when splits == 1, then dw is written directly).
TTDK_EXPORT int ttdk_conv_wgrad(const bf16_t* x, const bf16_t* dy, const TtdkConv* g, float* dw, float* ws,
                                int splits, int beta, int bm, int bn, hipStream_t st) {
  const int M = g->K, N = g->R * g->S * g->C, K = g->N * g->P * g->Q;
  if (g->C % 8 || g->K % 8) return hipErrorInvalidValue;
  const int bbn = (bm == 0 || bm == 256) ? big_bn_wgrad(M, N, K) : 0;
  if (bm == 0 || bn == 0 || bm == 256) pick_tile(M, N, &bm, &bn);
  const int ktiles = ceil_div(K, BK);
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  if (splits > 1 && !ws) return hipErrorInvalidValue;
  // unit-stride 1x1 convs with >= 256 output and input channels: the 4-wave transposed-read
  // kernel (gemm4t.hip), split-K summed by the last split of each tile
  if (bbn && is_pointwise(g) && M >= 256 && N >= 256 &&
      (splits == 1 || ttdk_gemm4t_ws(M, N, K, splits) <= static_cast<long long>(splits) * M * N)) {
    const int rc = ttdk_gemm4t_wgrad(dy, g->K, x, g->C, M, N, K, splits, ws, dw, beta, 1.f, nullptr, st);
    if (rc != hipErrorInvalidValue) return rc;
  }
  EpiParams pe{};
  pe.alpha = 1.f;
  pe.ldo = N;
  if (splits > 1) {
    pe.mode = 1;
    pe.out = ws;
    pe.slab_stride = static_cast<long long>(M) * N;
  } else {
    pe.mode = 2;
    pe.out = dw;
    pe.beta = beta;
  }
  DenseParams pa{dy, g->K, M, K};
  hipError_t e;
  bool folded = false;
  if (bbn && splits > 1 && big::inkernel_fold()) {
    // the 256-row kernel folds its own slabs (the last split of each tile sums them into dw)
    int* ctr = big::tile_counters(st, ceil_div(M, big::BM) * ceil_div(N, bbn));
    if (ctr) {
      pe.mode = 3;
      pe.kout = dw;
      pe.kctr = ctr;
      pe.beta = beta;
      folded = true;
    }
  }
  if (bbn && is_pointwise(g)) {
    e = bbn == 256 ? big::dense<256>(dy, g->K, false, x, g->C, false, pe, M, N, K, splits, st)
                   : big::dense<128>(dy, g->K, false, x, g->C, false, pe, M, N, K, splits, st);
  } else if (bbn) {
    const big::DenseP pa2{dy, g->K, M};
    const big::ConvP pb2 = conv_params(x, g->H, g->W, g->C, g->P, g->Q, g, N);
    e = bbn == 256 ? big::launch<256, big::OpDenseMN<128>, big::OpWgradMN<128>>(pa2, pb2, pe, M, N, K, splits, st)
                   : big::launch<128, big::OpDenseMN<128>, big::OpWgradMN<64>>(pa2, pb2, pe, M, N, K, splits, st);
  } else if (is_pointwise(g)) {
    DenseParams pb{x, g->C, N, K};
    e = dispatch<MNDense, MNDense>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  } else {
    GatherParams pb{x, g->H, g->W, g->C, g->P, g->Q, g->R, g->S, g->sh, g->sw, g->ph, g->pw, g->dh, g->dw, N, K};
    e = dispatch<MNDense, MNConvGather>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  }
  if (e != hipSuccess || splits == 1 || folded) return e;
  return splitk_reduce(ws, splits, static_cast<long long>(M) * N, dw, beta, st);
}

// Weight gradient whose dy is the output of a BatchNorm backward applied on the fly:
// dy = coef[0]*g + coef[1]*y + coef[2] per output channel (see MNDenseBN). Only the 4-wave
// im2col-gather path (non-pointwise convs too small for the 256-row kernel, e.g. the stem);
// returns hipErrorInvalidValue where ttdk_conv_wgrad would pick another kernel.
TTDK_EXPORT int ttdk_conv_wgrad_bn(const bf16_t* x, const bf16_t* g, const bf16_t* y, const float* coef,
                                   const TtdkConv* gm, float* dw, float* ws, int splits, int beta, int bm, int bn,
                                   hipStream_t st) {
  const int M = gm->K, N = gm->R * gm->S * gm->C, K = gm->N * gm->P * gm->Q;
  if (gm->C % 8 || gm->K % 8 || is_pointwise(gm) || big_bn_wgrad(M, N, K)) return hipErrorInvalidValue;
  if (bm == 0 || bn == 0 || bm == 256) pick_tile(M, N, &bm, &bn);
  const int ktiles = ceil_div(K, BK);
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  if (splits > 1 && !ws) return hipErrorInvalidValue;
  EpiParams pe{};
  pe.alpha = 1.f;
  pe.ldo = N;
  if (splits > 1) {
    pe.mode = 1;
    pe.out = ws;
    pe.slab_stride = static_cast<long long>(M) * N;
  } else {
    pe.mode = 2;
    pe.out = dw;
    pe.beta = beta;
  }
  DenseBNParams pa{g, gm->K, M, K, y, coef};
  GatherParams pb{x, gm->H, gm->W, gm->C, gm->P, gm->Q, gm->R, gm->S, gm->sh, gm->sw, gm->ph, gm->pw, gm->dh, gm->dw, N, K};
  hipError_t e = dispatch<MNDenseBN, MNConvGather>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  if (e != hipSuccess || splits == 1) return e;
  return splitk_reduce(ws, splits, static_cast<long long>(M) * N, dw, beta, st);
}

// fp8 weight gradient: dw[K,R,S,C] (fp32) = sum over pixels of dy8 (x) im2col(x8), dy8 OCP e5m2 and
// x8 e4m3 (both NHWC bytes: the e5m2 copy of the BN-backward output that the fp8 data gradient
// already consumes, and the e4m3 copy of the conv input that the fp8 forward consumed), both
// MN-major in the 256-row kernel (OpDenseMN8 / OpWgradMN8, ds_read_b64_tr_b8 fragments) on the
// block-scaled fp8 MFMA at twice the bf16 rate; ascale_dy / ascale_x: the inverse quantisation
// scales (device fp32), folded into the fp32 output. Requires C, K % 16 == 0, pixels % 128 == 0,
// 9C >= 256 (K < 256 output channels leave part of the 256-row tile idle).
TTDK_EXPORT int ttdk_conv_wgrad_fp8(const uint8_t* x8, const uint8_t* dy8, const TtdkConv* g, float* dw, float* ws,
                                    int splits, int beta, const float* ascale_dy, const float* ascale_x,
                                    hipStream_t st) {
  const int M = g->K, N = g->R * g->S * g->C, K = g->N * g->P * g->Q;
  if (g->C % 16 || g->K % 16 || K % 128 || N < 256 || M < 16 || !ascale_dy || !ascale_x ||
      static_cast<long long>(g->N) * g->H * g->W * g->C >= (1LL << 32) ||  // 32-bit im2col offsets
      (reinterpret_cast<uintptr_t>(x8) & 15) || (reinterpret_cast<uintptr_t>(dy8) & 15))
    return hipErrorInvalidValue;
  const int ktiles = K / 128;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  if (splits > 1 && !ws) return hipErrorInvalidValue;
  EpiParams pe{};
  pe.alpha = 1.f;
  pe.ascale0 = ascale_dy;
  pe.ascale1 = ascale_x;
  pe.ldo = N;
  if (splits > 1) {
    pe.mode = 1;
    pe.out = ws;
    pe.slab_stride = static_cast<long long>(M) * N;
  } else {
    pe.mode = 2;
    pe.out = dw;
    pe.beta = beta;
  }
  const big::DenseP pa{dy8, g->K, M};
  const big::ConvP pb = conv_params(x8, g->H, g->W, g->C, g->P, g->Q, g, N);
  // 256 x 128 tiles: with 256-wide tiles the i32x8 fragments and 128 accumulators held the whole
  // register file and the loader state spilled inside the main loop (each reload a vmcnt(0)
  // drain of the LDS-DMA pipeline)
  hipError_t e = big::launch<128, big::OpDenseMN8<128>, big::OpWgradMN8<64>, 2>(pa, pb, pe, M, N, K, splits, st);
  if (e != hipSuccess || splits == 1) return e;
  return splitk_reduce(ws, splits, static_cast<long long>(M) * N, dw, beta, st);
}
