// Convolution data gradient (direct gathers and sub-pixel phases); kernels in gemm_conv.h.
#include "gemm_conv.h"

// dx[N,H,W,C] = conv_transpose(dy[N,P,Q,K], w): wt must hold w transposed to [C][R][S][K]
// (ttdk_conv_weight_transpose). Rows of the GEMM are the pixels of dx.
// Strided 1x1 (no padding) convs compute only the rows that receive a gradient and use the
// epilogue's row remap; the caller zero-fills or pre-loads (beta=1) the other pixels.
TTDK_EXPORT int ttdk_conv_dgrad(const bf16_t* dy, const bf16_t* wt, const TtdkConv* g, int bm, int bn,
                                const TtdkEpilogue* epi, hipStream_t st) {
  if (g->K % 8) return hipErrorInvalidValue;
  EpiParams pe = to_epi(epi);
  if (pe.by && (pe.stat == nullptr || pe.mode != 0 || g->C % 8 || pe.ldo % 8 || pe.residual || pe.act))
    return hipErrorInvalidValue;
  if ((pe.by2 || pe.stat2) && !(pe.by && pe.by2 && pe.stat2)) return hipErrorInvalidValue;
  const int N = g->C, K = g->R * g->S * g->K;
  DenseParams pb{wt, K, N, K};
  if (g->R == 1 && g->S == 1 && g->ph == 0 && g->pw == 0) {
    const int M = g->N * g->P * g->Q;
    DenseParams pa{dy, g->K, M, K};
    if (g->sh != 1 || g->sw != 1) {
      // the stride-2-sampled beta (bH) tests the GEMM row, which a remap no longer equals
      if (g->sh != g->sw || pe.bH) return hipErrorInvalidValue;
      pe.remap = 1;
      pe.rP = g->P;
      pe.rQ = g->Q;
      pe.rOH = g->H;
      pe.rOW = g->W;
      pe.rs = g->sh;
    }
    const int bbn = big_bn(M, N, K);
    // per-tile statistics need the caller to know the tile height: with `stat` the 256-row
    // kernel runs only on an explicit bm == 256 request (and must then be eligible)
    if (((bm == 0 && pe.stat == nullptr) || bm == 256) && bbn && (bm != 256 || bn == bbn))
      return bbn == 256 ? big::dense<256>(dy, g->K, true, wt, K, true, pe, M, N, K, 1, st)
                        : big::dense<128>(dy, g->K, true, wt, K, true, pe, M, N, K, 1, st);
    if (bm == 256 && pe.stat) return hipErrorInvalidValue;
    if (bm == 0 || bn == 0 || bm == 256) pick_tile(M, N, &bm, &bn);
    return dispatch<KDense, KDense>(&pa, &pb, pe, M, N, K, 1, bm, bn, st);
  }
  const int M = g->N * g->H * g->W;
  const int bbn = big_bn(M, N, K);
  // unit-stride dgrad gathers on the LDS-DMA kernel (strided ones keep the 4-wave kernel: the
  // divisibility test costs registers the 256-row tile does not have)
  static const bool strided_big = [] {
    const char* e = getenv("TTD_BIG_STRIDED_DGRAD");
    return e != nullptr && e[0] == '1';
  }();
  const bool unit = g->sh == 1 && g->sw == 1;
  if (((bm == 0 && pe.stat == nullptr) || bm == 256) && bbn && (bm != 256 || bn == bbn) && g->K % 64 == 0 &&
      !pe.remap && (unit || strided_big)) {
    const big::ConvP pa = conv_params(dy, g->P, g->Q, g->K, g->H, g->W, g, M);
    const big::DenseP pb2{wt, K, N};
    if (unit) {
      if (bbn == 256)
        return big::launch<256, big::OpConvK<128, 2, true, true>, big::OpDenseK<128, 2>>(pa, pb2, pe, M, N, K, 1, st);
      return big::launch<128, big::OpConvK<128, 2, true, true>, big::OpDenseK<64, 2>>(pa, pb2, pe, M, N, K, 1, st);
    }
    if (bbn == 256)
      return big::launch<256, big::OpConvK<128, 2, true>, big::OpDenseK<128, 2>>(pa, pb2, pe, M, N, K, 1, st);
    return big::launch<128, big::OpConvK<128, 2, true>, big::OpDenseK<64, 2>>(pa, pb2, pe, M, N, K, 1, st);
  }
  if (bm == 256 && pe.stat) return hipErrorInvalidValue;
  if (bm == 0 || bn == 0 || bm == 256) pick_tile(M, N, &bm, &bn);
  GatherParams pa{dy, g->P, g->Q, g->K, g->H, g->W, g->R, g->S, g->sh, g->sw, g->ph, g->pw, g->dh, g->dw, M, K};
  return dispatch<KConvDgrad, KDense>(&pa, &pb, pe, M, N, K, 1, bm, bn, st);
}

// Pointwise (1x1, stride 1) data gradient whose operand is the BN backward of the unit's output
// gradient, formed in the 256-row kernel's LDS (EpiParams::py / pcoef / pdz):
//   dz = coef[0][k]*g + coef[1][k]*y + coef[2][k]  (g: the masked output gradient, y: the unit's conv output)
//   dx = dz . W  (+ the usual epilogue: accumulate, feeding-BN statistics)
// dz is also stored (by the workgroups of tile column 0) for the weight gradient. Returns
// hipErrorNotSupported when the shape is not on the 256-row kernel (the caller keeps the pass).
TTDK_EXPORT int ttdk_conv_dgrad_bnpro(const bf16_t* g_in, const bf16_t* wt, const TtdkConv* g, const bf16_t* y,
                                      const float* coef, bf16_t* dz, const TtdkEpilogue* epi, hipStream_t st) {
  if (!(g->R == 1 && g->S == 1 && g->ph == 0 && g->pw == 0 && g->sh == 1 && g->sw == 1)) return hipErrorNotSupported;
  EpiParams pe = to_epi(epi);
  if (pe.by && (pe.stat == nullptr || pe.mode != 0 || g->C % 8 || pe.ldo % 8 || pe.residual || pe.act))
    return hipErrorInvalidValue;
  if ((pe.by2 || pe.stat2) && !(pe.by && pe.by2 && pe.stat2)) return hipErrorInvalidValue;
  const int N = g->C, K = g->K;
  const int M = g->N * g->P * g->Q;
  const int bbn = big_bn(M, N, K);
  if (!bbn || K % 64 || pe.mode != 0 || pe.remap) return hipErrorNotSupported;
  pe.py = y;
  pe.pcoef = coef;
  pe.pdz = dz;
  pe.pld = K;
  const big::DenseP pa{g_in, K, M}, pb{wt, K, N};
  if (bbn == 256)
    return big::launch<256, big::OpDenseKBN<128, 2>, big::OpDenseK<128, 2>, 0, 0>(pa, pb, pe, M, N, K, 1, st);
  return big::launch<128, big::OpDenseKBN<128, 2>, big::OpDenseK<64, 2>, 0, 0>(pa, pb, pe, M, N, K, 1, st);
}

// Whether ttdk_conv_dgrad_bnpro runs this shape (its BN statistics rows are 256-row tiles).
TTDK_EXPORT int ttdk_conv_dgrad_bnpro_ok(const TtdkConv* g) {
  const int M = g->N * g->P * g->Q;
  return g->R == 1 && g->S == 1 && g->ph == 0 && g->pw == 0 && g->sh == 1 && g->sw == 1 && g->K % 64 == 0 &&
         big_bn(M, g->C, g->K) != 0;
}

// ---- strided dgrad by sub-pixel (phase) decomposition
// For stride s, the input pixels h = s*i + a of one phase a only receive taps r ≡ (a + ph)
// (mod s), so dx restricted to that phase is a UNIT-stride dgrad over dy with the tap subset
// r = r0 + t*s (t < T_a) and padding off_a = (a + ph - r0)/s:
//     dx[s*i + a] = sum_t dy[i + off_a - t] * w[r0 + t*s]
// The s*s phases partition dx exactly; each is a gather GEMM of K = T_a*T_b*Kout written
// through the epilogue's strided row remap (base pointer shifted to pixel (a, b)). Versus
// the direct strided gather this skips the (s*s-1)/(s*s) zero taps — 4x fewer MFMA ops for
// ResNet's 3x3 stride-2 convs — and every phase runs on the unit-stride LDS-DMA path.
__global__ __launch_bounds__(256) void subpixel_weights_kernel(const bf16_t* __restrict__ wt, bf16_t* __restrict__ ws,
                                                               int C, int R, int S, int Kc, int s, int r0, int Tr,
                                                               int s0, int Ts) {
  const int k8n = Kc >> 3;
  const long long total = static_cast<long long>(C) * Tr * Ts * k8n;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += static_cast<long long>(gridDim.x) * 256) {
    const int k8 = static_cast<int>(idx % k8n);
    long long rest = idx / k8n;
    const int ts = static_cast<int>(rest % Ts);
    rest /= Ts;
    const int tr = static_cast<int>(rest % Tr);
    const long long c = rest / Tr;
    const bf16_t* src = wt + c * (static_cast<long long>(R) * S * Kc) +
                        (static_cast<long long>(r0 + tr * s) * S + (s0 + ts * s)) * Kc + k8 * 8;
    reinterpret_cast<uint4*>(ws)[idx] = *reinterpret_cast<const uint4*>(src);
  }
}

// Phase geometry along one axis: first tap, tap count, padding offset, phase extent.
struct Phase {
  int r0, T, off, n;
};
static Phase phase_of(int a, int s, int pad, int R, int H) {
  Phase ph;
  ph.r0 = (a + pad) % s;
  ph.T = ph.r0 < R ? (R - ph.r0 + s - 1) / s : 0;
  ph.off = (a + pad - ph.r0) / s;
  ph.n = a < H ? (H - a + s - 1) / s : 0;
  return ph;
}

// dx[N,H,W,C] of a strided conv (dilation 1, every phase has >= 1 tap) by phases. `ws`:
// scratch for the phase sub-kernels, C*R*S*Kout bf16 (the size of wt); ws_ready != 0: ws
// already holds the phase filters in this launcher's phase order (ttdk_wprep, once per step),
// wt is not read.
TTDK_EXPORT int ttdk_conv_dgrad_subpixel(const bf16_t* dy, const bf16_t* wt, const TtdkConv* g, bf16_t* ws,
                                         int ws_ready, const TtdkEpilogue* epi, hipStream_t st) {
  const int s = g->sh;
  if (g->sw != s || s < 2 || g->dh != 1 || g->dw != 1 || g->R < s || g->S < s || g->K % 8 || g->C % 8)
    return hipErrorInvalidValue;
  EpiParams pe = to_epi(epi);
  if (pe.remap || pe.residual || pe.aux || pe.mode == 1 || pe.by2 || pe.stat2 || pe.bH) return hipErrorInvalidValue;
  if ((pe.stat != nullptr) != (pe.by != nullptr) || (pe.by && (pe.mode != 0 || g->C % 8 || pe.ldo % 8)))
    return hipErrorInvalidValue;
  const int N = g->C, Kc = g->K;
  const size_t esz = pe.mode == 0 ? sizeof(bf16_t) : sizeof(float);
  bf16_t* wsp = ws;
  long long stat_row = 0;  // BN-backward statistics: each phase GEMM owns its own block of tile rows
  for (int a = 0; a < s; ++a) {
    const Phase pr = phase_of(a, s, g->ph, g->R, g->H);
    for (int b = 0; b < s; ++b) {
      const Phase pc = phase_of(b, s, g->pw, g->S, g->W);
      if (pr.n == 0 || pc.n == 0) continue;
      const int M = g->N * pr.n * pc.n, K = pr.T * pc.T * Kc;
      const long long wn = static_cast<long long>(N) * K;
      int grid = static_cast<int>(std::min<long long>((wn / 8 + 255) / 256, 4096));
      if (!ws_ready)
        hipLaunchKernelGGL(subpixel_weights_kernel, dim3(grid), dim3(256), 0, st, wt, wsp, N, g->R, g->S, Kc, s,
                           pr.r0, pr.T, pc.r0, pc.T);
      EpiParams e = pe;
      e.remap = 1;
      e.rP = pr.n;
      e.rQ = pc.n;
      e.rOH = g->H;
      e.rOW = g->W;
      e.rs = s;
      const long long base = (static_cast<long long>(a) * g->W + b) * pe.ldo;  // phase origin (elements)
      e.out = static_cast<char*>(pe.out) + base * esz;
      hipError_t err;
      const int bbn = big_bn(M, N, K);
      if (pe.by) {
        e.by = pe.by + base;
        e.bmask = pe.bmask ? pe.bmask + base / 8 : nullptr;
        e.stat = pe.stat + stat_row * 2 * N;
        int pbm = 0, pbn = 0;
        pick_tile(M, N, &pbm, &pbn);
        stat_row += ceil_div(M, (bbn && Kc % 64 == 0) ? 256 : pbm);
      }
      if (bbn && Kc % 64 == 0) {
        const big::ConvP pa{dy, g->P, g->Q, Kc, pr.n, pc.n, pr.T, pc.T, 1, 1, pr.off, pc.off, 1, 1, M};
        const big::DenseP pb{wsp, K, N};
        err = bbn == 256
                  ? big::launch<256, big::OpConvK<128, 2, true, true>, big::OpDenseK<128, 2>>(pa, pb, e, M, N, K, 1, st)
                  : big::launch<128, big::OpConvK<128, 2, true, true>, big::OpDenseK<64, 2>>(pa, pb, e, M, N, K, 1, st);
      } else {
        int bm = 0, bn = 0;
        pick_tile(M, N, &bm, &bn);
        GatherParams pa{dy, g->P, g->Q, Kc, pr.n, pc.n, pr.T, pc.T, 1, 1, pr.off, pc.off, 1, 1, M, K};
        DenseParams pb{wsp, K, N, K};
        err = dispatch<KConvDgrad, KDense>(&pa, &pb, e, M, N, K, 1, bm, bn, st);
      }
      if (err != hipSuccess) return err;
      wsp += wn;
    }
  }
  return hipGetLastError();
}

// Tile rows of the BN-backward partial-sum buffer ttdk_conv_dgrad_subpixel fills when its
// epilogue carries statistics (sum over phases of each phase GEMM's row tiles).
TTDK_EXPORT long long ttdk_conv_dgrad_subpixel_stat_rows(const TtdkConv* g) {
  const int s = g->sh;
  if (g->sw != s || s < 2) return -1;
  const int N = g->C;
  long long rows = 0;
  for (int a = 0; a < s; ++a) {
    const Phase pr = phase_of(a, s, g->ph, g->R, g->H);
    for (int b = 0; b < s; ++b) {
      const Phase pc = phase_of(b, s, g->pw, g->S, g->W);
      if (pr.n == 0 || pc.n == 0) continue;
      const int M = g->N * pr.n * pc.n, K = pr.T * pc.T * g->K;
      int pbm = 0, pbn = 0;
      pick_tile(M, N, &pbm, &pbn);
      rows += ceil_div(M, (big_bn(M, N, K) && g->K % 64 == 0) ? 256 : pbm);
    }
  }
  return rows;
}
