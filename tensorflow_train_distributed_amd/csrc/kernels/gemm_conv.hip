// Dense bf16 GEMM entry point (+ split-K reduce); kernels in gemm_conv.h.
#include "gemm_conv.h"

extern "C" int ttdk_gemm4t_wgrad(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                 int splits, float* ws, float* out, int beta, float alpha, float* rowsum,
                                 hipStream_t st);
extern "C" long long ttdk_gemm4t_ws(int M, int N, int K, int splits);
extern "C" int ttdk_gemm4w_bf16(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                const TtdkEpilogue* epi, hipStream_t st);

// General GEMM: C[M,N] = alpha * A·B with A either K-major (a_kmajor=1: A[m*lda + k]) or
// MN-major (A[k*lda + m]); B either K-major (B[n*ldb + k]) or MN-major (B[k*ldb + n]).
TTDK_EXPORT int ttdk_gemm_bf16(const bf16_t* A, long long lda, int a_kmajor, const bf16_t* B, long long ldb,
                               int b_kmajor, int M, int N, int K, int splits, int bm, int bn,
                               const TtdkEpilogue* epi, hipStream_t st) {
  EpiParams pe = to_epi(epi);
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // 16-B vector operand loads need the contiguous dim and the leading dim to be multiples
  // of 8 elements and 16-B aligned bases; otherwise both operands use the masked scalar path.
  const bool vec = al(A) && al(B) && lda % 8 == 0 && ldb % 8 == 0 && (a_kmajor ? K % 8 == 0 : M % 8 == 0) &&
                   (b_kmajor ? K % 8 == 0 : N % 8 == 0);
  DenseParams pa{A, lda, M, K};
  DenseParams pb{B, ldb, N, K};
  // K-major x K-major GEMMs with an elementwise epilogue: the 4-wave AGPR-accumulator kernel
  // (gemm4w.hip; persistent, ~5-15 % ahead of the 8-wave 256-row kernel at every BERT-Large
  // shape, tools/g4_bench.py). It refuses what it does not take (hipErrorInvalidValue) and the
  // 256-row path below runs instead. TTD_G4=0: off.
  static const int g4_on = getenv_int("TTD_G4", 1);
  if (g4_on && a_kmajor && b_kmajor && vec && bm == 0 && bn == 0 && pe.mode == 0 && M >= 256 && N >= 256 &&
      K >= 128 && K % 128 == 0) {
    const int rc = ttdk_gemm4w_bf16(A, lda, B, ldb, M, N, K, epi, st);
    if (rc != hipErrorInvalidValue) return rc;
  }
  // 256-row LDS-DMA path for big GEMMs (explicit tile 256 forces it; 128/64 force the 4-wave kernel)
  const int bbn = big_bn(M, N, K);
  // per-tile statistics rows follow the kernel's tile height: with `stat` the 256-row kernel runs
  // only on an explicit bm == 256 request (the caller sized `stat` for 256-row tiles)
  const bool big_ok = vec && bbn && pe.remap == 0 && (pe.stat == nullptr || bm == 256) && (a_kmajor || M % 8 == 0);
  if (big_ok && (bm == 256 || bm == 0)) {
    if (bbn == 256) return big::dense<256>(A, lda, a_kmajor, B, ldb, b_kmajor, pe, M, N, K, splits, st);
    return big::dense<128>(A, lda, a_kmajor, B, ldb, b_kmajor, pe, M, N, K, splits, st);
  }
  if (bm == 256 && pe.stat) return hipErrorInvalidValue;  // asked for 256-row statistics rows, kernel not eligible
  if (bm == 256) bm = 0;
  if (bm == 0 || bn == 0) pick_tile(M, N, &bm, &bn);
  if (vec) {
    if (a_kmajor && b_kmajor) return dispatch<KDense, KDense>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
    if (a_kmajor) return dispatch<KDense, MNDense>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
    if (b_kmajor) return dispatch<MNDense, KDense>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
    return dispatch<MNDense, MNDense>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  }
  if (a_kmajor && b_kmajor) return dispatch<KDenseS, KDenseS>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  if (a_kmajor) return dispatch<KDenseS, MNDenseS>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  if (b_kmajor) return dispatch<MNDenseS, KDenseS>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
  return dispatch<MNDenseS, MNDenseS>(&pa, &pb, pe, M, N, K, splits, bm, bn, st);
}

// Strided-batched GEMM: C_z[M,N] = alpha * op(A_z) . op(B_z) for z < batch in ONE launch (batch on
// grid z; A_z = A + z*sa, B_z = B + z*sb, C_z = out + z*so, element strides), bf16 operands in
// either layout, bf16 (out_fp32 = 0) or fp32 output. The batched MatMul of ttd.nn.matmul
// (tf.matmul on rank > 2 operands; per-entry launches before).
TTDK_EXPORT int ttdk_gemm_bf16_batched(const bf16_t* A, long long lda, long long sa, int a_kmajor, const bf16_t* B,
                                       long long ldb, long long sb, int b_kmajor, void* out, long long ldo,
                                       long long so, int out_fp32, int M, int N, int K, int batch, hipStream_t st) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return hipErrorInvalidValue;
  const bool vec = al(A) && al(B) && lda % 8 == 0 && ldb % 8 == 0 && sa % 8 == 0 && sb % 8 == 0 &&
                   (a_kmajor ? K % 8 == 0 : M % 8 == 0) && (b_kmajor ? K % 8 == 0 : N % 8 == 0);
  TtdkEpilogue te{};
  te.mode = out_fp32 ? 2 : 0;
  te.out = out;
  te.ldo = ldo;
  EpiParams pe = to_epi(&te);
  DenseParams pa{A, lda, M, K};
  DenseParams pb{B, ldb, N, K};
  int bm = 0, bn = 0;
  pick_tile(M, N, &bm, &bn);
#define TTDK_BCASE(BM_, BN_, LA_, LB_)                                                                            \
  if (bm == BM_ && bn == BN_) return launch_batched<BM_, BN_, LA_<BM_>, LB_<BN_>>(pa, pb, pe, M, N, K, batch, sa, sb, so, st);
#define TTDK_BLAYOUT(LA_, LB_) \
  {                            \
    TTDK_BCASE(128, 128, LA_, LB_) \
    TTDK_BCASE(128, 64, LA_, LB_)  \
    TTDK_BCASE(64, 128, LA_, LB_)  \
    TTDK_BCASE(64, 64, LA_, LB_)   \
  }
  if (vec) {
    if (a_kmajor && b_kmajor) TTDK_BLAYOUT(KDense, KDense)
    if (a_kmajor && !b_kmajor) TTDK_BLAYOUT(KDense, MNDense)
    if (!a_kmajor && b_kmajor) TTDK_BLAYOUT(MNDense, KDense)
    if (!a_kmajor && !b_kmajor) TTDK_BLAYOUT(MNDense, MNDense)
  } else {
    if (a_kmajor && b_kmajor) TTDK_BLAYOUT(KDenseS, KDenseS)
    if (a_kmajor && !b_kmajor) TTDK_BLAYOUT(KDenseS, MNDenseS)
    if (!a_kmajor && b_kmajor) TTDK_BLAYOUT(MNDenseS, KDenseS)
    if (!a_kmajor && !b_kmajor) TTDK_BLAYOUT(MNDenseS, MNDenseS)
  }
#undef TTDK_BLAYOUT
#undef TTDK_BCASE
  return hipErrorInvalidValue;
}

// Split-K GEMM into an fp32 output: C (+)= alpha * A.B over `splits` K-slices with fp32 slabs in
// `ws` [splits][M][N]. On the 256-row kernel the launch folds its own slabs (EpiParams mode 3);
// elsewhere a fold pass follows.
TTDK_EXPORT int ttdk_gemm_bf16_splitk(const bf16_t* A, long long lda, int a_kmajor, const bf16_t* B, long long ldb,
                                      int b_kmajor, int M, int N, int K, int splits, float* ws, float* out, int beta,
                                      float alpha, int tile_m, int tile_n, hipStream_t st) {
  TtdkEpilogue te{};
  te.mode = 1;
  te.out = ws;
  te.ldo = N;
  te.slab_stride = static_cast<long long>(M) * N;
  te.alpha = alpha;
  EpiParams pe = to_epi(&te);
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool vec = al(A) && al(B) && lda % 8 == 0 && ldb % 8 == 0 && (a_kmajor ? K % 8 == 0 : M % 8 == 0) &&
                   (b_kmajor ? K % 8 == 0 : N % 8 == 0);
  const int bbn = big_bn(M, N, K);
  const int ktiles = K / 64;
  // a forced tile (tile_m / tile_n != 0, tests and benches) always takes the slab + fold path,
  // which honours it; the in-kernel fold exists for the 256-row kernel at its own BN only
  const bool forced = tile_m != 0 || tile_n != 0;
  // MN-major operands (weight gradients): the 4-wave transposed-read kernel (gemm4t.hip), its
  // split-K summed by the last split of each tile
  if (!forced && !a_kmajor && !b_kmajor && ttdk_gemm4t_ws(M, N, K, splits) <= static_cast<long long>(splits) * M * N) {
    const int rc = ttdk_gemm4t_wgrad(A, lda, B, ldb, M, N, K, splits, ws, out, beta, alpha, nullptr, st);
    if (rc != hipErrorInvalidValue) return rc;
  }
  if (!forced && splits > 1 && vec && bbn && (a_kmajor || M % 8 == 0) && big::inkernel_fold() && ktiles >= splits) {
    int* ctr = big::tile_counters(st, ceil_div(M, big::BM) * ceil_div(N, bbn));
    if (ctr) {
      pe.mode = 3;
      pe.kout = out;
      pe.kctr = ctr;
      pe.beta = beta;
      return bbn == 256 ? big::dense<256>(A, lda, a_kmajor, B, ldb, b_kmajor, pe, M, N, K, splits, st)
                        : big::dense<128>(A, lda, a_kmajor, B, ldb, b_kmajor, pe, M, N, K, splits, st);
    }
  }
  const int rc = ttdk_gemm_bf16(A, lda, a_kmajor, B, ldb, b_kmajor, M, N, K, splits, tile_m, tile_n, &te, st);
  if (rc != hipSuccess) return rc;
  return splitk_reduce(ws, splits, static_cast<long long>(M) * N, out, beta, st);
}

// Weight gradient + bias gradient in one pass over dY: out[M,N] (+)= alpha * A.B with A = dY^T
// MN-major (A[k*lda + m], k = token) and B MN-major, and rowsum[M] = sum_k A[k][m] (the bias
// gradient, written) formed from the A tiles already in LDS (gemm256_kernel RS): the separate
// column-sum pass over dY disappears. ws: splits * M * N floats (split-K slabs) followed by
// splits * ceil(N / 256) * M floats (row-sum partials). Returns hipErrorInvalidValue when the
// shape does not take the 256-row ping-pong kernel (the caller keeps its column-sum pass).
TTDK_EXPORT long long ttdk_gemm_wgrad_bias_ws(int M, int N, int K, int splits) {
  // -1 (no fused path: the caller keeps its column-sum pass) unless gemm4t or the 256-row
  // kernel admits the shape
  const long long w4 = ttdk_gemm4t_ws(M, N, K, splits);
  if (big_bn(M, N, K) != 256 || M % 8 || N % 8 || K % 64) return w4;
  const int ktiles = K / 64;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  splits = ceil_div(ktiles, ceil_div(ktiles, splits));
  return std::max(w4, static_cast<long long>(splits) * M * N + static_cast<long long>(splits) * ceil_div(N, 256) * M);
}

TTDK_EXPORT int ttdk_gemm_wgrad_bias(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                     int splits, float* ws, float* out, int beta, float alpha, float* rowsum,
                                     hipStream_t st) {
  {
    const int rc = ttdk_gemm4t_wgrad(A, lda, B, ldb, M, N, K, splits, ws, out, beta, alpha, rowsum, st);
    if (rc != hipErrorInvalidValue) return rc;
  }
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al(A) || !al(B) || lda % 8 || ldb % 8 || M % 8 || N % 8 || K % 64 || big_bn(M, N, K) != 256 || !rowsum)
    return hipErrorInvalidValue;
  const int ktiles = K / 64;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  splits = ceil_div(ktiles, ceil_div(ktiles, splits));
  if (ceil_div(ktiles, splits) < 16) return hipErrorInvalidValue;  // the ping-pong schedule's K-tile floor
  TtdkEpilogue te{};
  te.mode = 1;
  te.out = ws;
  te.ldo = N;
  te.slab_stride = static_cast<long long>(M) * N;
  te.alpha = alpha;
  EpiParams pe = to_epi(&te);
  float* rs = ws + static_cast<long long>(splits) * M * N;
  pe.rsum = rs;
  const int rc = big::dense_rowsum(A, lda, B, ldb, pe, M, N, K, splits, st);
  if (rc != hipSuccess) return rc;
  const int r2 = splitk_reduce(ws, splits, static_cast<long long>(M) * N, out, beta, st);
  if (r2 != hipSuccess) return r2;
  return splitk_reduce(rs, splits * ceil_div(N, 256), M, rowsum, 0, st);
}

TTDK_EXPORT int ttdk_splitk_reduce(const float* ws, int splits, long long n, float* out, int beta, hipStream_t st) {
  return splitk_reduce(ws, splits, n, out, beta, st);
}

// process-wide runtime switches (declared in gemm_conv.h)
namespace ttdk_rt {
int& pers_flag() {
  static int on = getenv_int("TTD_BIG_PERS", 1);
  return on;
}
int& reserved_cus() {
  static int n = getenv_int("TTD_RESERVED_CUS", 0);
  return n;
}
int& fold_flag() {
  static int on = getenv_int("TTD_SPLITK_FOLD_INKERNEL", 0);
  return on;
}
}  // namespace ttdk_rt

// Runtime switch of the in-kernel split-K fold (gemm_conv.h inkernel_fold); returns the previous
// setting.
TTDK_EXPORT int ttdk_set_inkernel_fold(int on) {
  const int old = ttdk_rt::fold_flag();
  ttdk_rt::fold_flag() = on;
  return old;
}

// CUs kept free of persistent grids for the collective engine's CTAs (see device_cus in
// gemm_conv.h); returns the previous setting.
TTDK_EXPORT int ttdk_set_reserved_cus(int n) {
  const int old = ttdk_rt::reserved_cus();
  ttdk_rt::reserved_cus() = n < 0 ? 0 : n;
  return old;
}

// CUs the persistent kernels currently size their grids to.
TTDK_EXPORT int ttdk_persistent_cus() { return big::device_cus(); }


// Runtime switch of the persistent register-epilogue 256-row GEMM (gemm256p_kernel); returns
// the previous setting.
TTDK_EXPORT int ttdk_set_big_pers(int on) {
  const int old = ttdk_rt::pers_flag();
  ttdk_rt::pers_flag() = on;
  return old;
}
