// 4-wave 256 x 256 weight-gradient GEMM on MN-major operands: dW[M,N] (+)= alpha * A^T . B with
// A [K][M] (row stride lda) and B [K][N] (ldb), K = tokens / pixels, both operands read in their
// stored layout — the reduction runs down the rows, so neither operand is K-contiguous.
//
// Reference op: the kernel gradients of tf.layers.dense (/root/reference/distribute_training.py:54,61,
// taken by the optimizer's compute_gradients at :152).
//
// Why a second 4-wave kernel (gemm4w.hip is the K-major one): the 8-wave 256-row loop ran BERT's
// weight gradients at 29-32 % MFMA utilisation with 41-43 % of wave cycles waiting
// (profiles/r4_bert_wgrad_pmc_s2.txt), plus a split-K fold pass over fp32 slabs (~17-22 ms per
// BERT-Large step). Here:
//  * operand tiles [64 k-rows][256 columns] reach LDS by LDS-DMA (16 B per lane) in their HBM
//    layout; the MFMA fragments (8 consecutive k of one column per lane) come out of LDS with the
//    CDNA4 transposing read ds_read_b64_tr_b16 (4 k-rows x 16 columns per 16-lane group, two
//    reads per 16x32 fragment) — no transpose pass, no VALU shuffles;
//  * LDS rows are 512 B; the 32-B slot of columns 16j..16j+15 in k-row r sits at slot
//    j ^ f(r), f(r) = (r & 3) | ((r >> 3) & 1) << 2: the 8 k-rows one half-wave's transposed
//    read touches (rows 8g + q, g = the half's two groups, q = 0..3) land on 8 different bank
//    groups (conflict-free); the DMA applies the same XOR when choosing which global chunk each
//    lane fetches, so the LDS side stays lane-linear;
//  * accumulators: 64 AGPR tiles per wave (inline-asm MFMA, "+a"), the schedule of gemm4w's
//    SCHED 2 (two barriers per K-tile, DMA of K-tile kt + 2 under K-step 1's MFMAs);
//  * split-K without a fold pass: every split stores its fp32 partial tile lane-linear (1 KB per
//    store instruction), the LAST split of a tile to arrive (per-tile counter) sums the tile's
//    partials in split order (deterministic) and writes dW (+= with beta);
//  * GB: B read as the im2col of a convolution input x [N][H][W][C] (the weight gradient of a
//    strided / 3x3 conv: k-row = output pixel, column = filter tap (r, s, c)): each lane's 16-B
//    DMA chunk has its own source offset per k-row, formed for K-tile kt + 2 between the MFMAs
//    of K-tile kt (pixel -> (n, p, q) by multiply-high divisions, tap validity against the
//    padding); a tap in the padding gets an offset past the buffer's end, which the buffer load
//    returns as zeros — no branch, no zero fill;
//  * RS: the bias gradient rowsum(A^T) = column sums of dY from the A fragments already in
//    registers, as an MFMA against a ones operand (D = 1 . A): 4 extra MFMAs per K-step and wave
//    on 1 / tiles_n of the K-tiles (spread over the tile columns); the last workgroup of a tile
//    row to finish sums the row's partials (no separate reduce launch: on the side stream of the
//    BERT step a tiny reduce kernel waited ~200 us per call for a free CU).
#include "gemm_conv.h"

#include <type_traits>

typedef __attribute__((ext_vector_type(4))) int ttd_i32x4_t;
typedef __attribute__((ext_vector_type(4))) short ttd_s16x4_t;

namespace ttdk {
namespace {
namespace g4t {

constexpr int T = 256;
constexpr int OPB = 64 * 512;    // the B operand's K-tile image: 64 k-rows x 256 bf16 columns
constexpr int kLgkm0 = 0xC07F;   // s_waitcnt encoding: lgkmcnt(0), vmcnt / expcnt not waited

typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) ttd_s16x4_t lds_s4_t;

__device__ __forceinline__ ttd_i32x4_t make_srd(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  ttd_i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane(static_cast<int>((a >> 32) & 0xffffu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA piece with M0 already holding its LDS base; sets M0 for the next piece right after
// issuing (MFMAs separate it from the next piece: no s_nop for the M0 hazard). Nothing else
// writes M0 in this kernel (ds_* need no M0 on gfx950; every LDS-DMA is this asm).
__device__ __forceinline__ void dma_chain(uint32_t voff, const ttd_i32x4_t& srd, int soff, uint32_t next_m0) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds\n\ts_mov_b32 m0, %3"
               :
               : "v"(voff), "s"(srd), "s"(soff), "s"(next_m0)
               : "memory");
}
__device__ __forceinline__ void m0_init(uint32_t v) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(v) : "memory");
}

template <int N, class F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

// MN-major operand loader: K-tile image [64 k-rows][512 B]; piece i (0..7) of thread tid fills
// LDS chunk i * 256 + tid = k-row i * 8 + tid / 32, physical 16-B chunk tid % 32, i.e. 32-B slot
// (tid % 32) / 2, which holds logical slot ((tid % 32) / 2) ^ f(row). f depends on the piece only
// through i & 1, so two per-lane offsets cover the 8 pieces; the k-row step (i * 8 rows) and the
// K-tile offset are scalar (soffset). Columns past the operand's end are clamped to its last 8
// (their outputs are never stored).
struct LoadMN {
  ttd_i32x4_t srd;
  uint32_t voff[2];
  int row8;  // bytes of 8 k-rows
  __device__ __forceinline__ void init(const bf16_t* p, long long ld, int K, int cols, int col0, int tid) {
    srd = make_srd(p, static_cast<uint32_t>(static_cast<long long>(K) * ld * 2));
    row8 = static_cast<int>(ld * 16);
    const int pc = tid & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = ((tid >> 5) & 3) | (i << 2);
      const int col = min(col0 + (((pc >> 1) ^ f) << 4) + (pc & 1) * 8, cols - 8);
      voff[i] = static_cast<uint32_t>((static_cast<long long>(tid >> 5) * ld + col) * 2);
    }
  }
};

// im2col geometry of a gathered B operand: conv input x [N][H][W][C], k-row = output pixel
// (n, p, q) of a P x Q map, column = (r, s, c) of an R x S filter. Divisions by P*Q and Q are
// multiply-high + shift (magic numbers from the host, exact for k < 2^31).
struct Gather {
  int H, W, C, Q, PQ, S, sh, sw, ph, pw;
  unsigned pq_m, q_m;
  int pq_s, q_s;
};

constexpr uint32_t kOob = 0x80000000u;  // past the end of every gathered buffer (< 2 GiB): reads 0

// per-lane column decode of a gathered operand (once per kernel): tap (r, s) and the element
// offset of (r, s, c) relative to the pixel's (h0, w0) corner
struct GCol {
  int r[2], s[2], toff[2];
};

__device__ __forceinline__ uint32_t gather_voff(const Gather& G, const GCol& gc, int j, int k) {
  const int n = static_cast<int>(__umulhi(static_cast<unsigned>(k), G.pq_m) >> G.pq_s);
  const int rem = k - n * G.PQ;
  const int p = static_cast<int>(__umulhi(static_cast<unsigned>(rem), G.q_m) >> G.q_s);
  const int q = rem - p * G.Q;
  const int hb = p * G.sh - G.ph, wb = q * G.sw - G.pw;
  const bool ok = static_cast<unsigned>(hb + gc.r[j]) < static_cast<unsigned>(G.H) &&
                  static_cast<unsigned>(wb + gc.s[j]) < static_cast<unsigned>(G.W);
  return ok ? static_cast<uint32_t>((((n * G.H + hb) * G.W + wb) * G.C + gc.toff[j]) * 2) : kOob;
}

__device__ __forceinline__ ttd_s16x4_t trd(const lds_char_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)p);
}

__device__ __forceinline__ bf16x8_t cat(const ttd_s16x4_t& lo, const ttd_s16x4_t& hi) {
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// acc (+)= x . y^T, accumulator an AGPR operand (FIRST: C = 0). "memory": keeps the compiler's
// LDS reads where the schedule puts them (between MFMAs) instead of hoisting / sinking them.
template <bool FIRST>
__device__ __forceinline__ void mfma_acc(f32x4_t& c, const bf16x8_t& x, const bf16x8_t& y) {
  if constexpr (FIRST)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(y), "v"(x) : "memory");
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(y), "v"(x) : "memory");
}
// column sums of a fragment: c[.][col] += sum_k x[k][col] (D = ones . x). Wait states hipcc does
// not insert around asm: the leading s_nop 1 (hipcc may rematerialise `ones` or zero `c` — VALU
// writes — right before; a VALU-written MFMA operand needs 2), and after the LAST of a group
// (TAIL) s_nop 11: the VGPR result may be read or moved by compiler code next, and an 8-pass
// MFMA's D needs 12 states before any reader but a chained MFMA (a missing tail read stale sums
// of the group's last block).
template <bool TAIL>
__device__ __forceinline__ void mfma_rs(f32x4_t& c, const bf16x8_t& ones, const bf16x8_t& x) {
  if constexpr (TAIL)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\ts_nop 11" : "+v"(c) : "v"(ones), "v"(x)
                 : "memory");
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(ones), "v"(x) : "memory");
}

__device__ __forceinline__ void tile_of(int t, int tiles_m, int tiles_n, int group, int& tm, int& tn) {
  const int per = group * tiles_n;
  const int g0 = (t / per) * group;
  const int gm = min(tiles_m - g0, group);
  const int r = t - (t / per) * per;
  tm = g0 + r % gm;
  tn = r / gm;
}

// Tile geometry: BM x 256 output tiles, BM = 256 (2 x 2 waves of 128 x 128) or 128 (2 x 2 waves of
// 64 x 128: the weight gradients with 128 output rows — ResNet stage-3 c1 / 3x3 convs — no longer
// pay a half-empty 256-row tile). A image: 64 k-rows x BM columns (rows of 2 BM bytes, the 32-B
// slot XOR of the B image), B image: 64 k-rows x 256 columns.
template <int BM>
struct Geo {
  static_assert(BM == 256 || BM == 128, "256- or 128-row tiles");
  static constexpr int NA = BM / 32;        // A fragments (16-row blocks) per wave
  static constexpr int NB = 8;              // B fragments per wave
  static constexpr int NF = NA + NB;
  static constexpr int AROW = BM * 2;       // bytes per A k-row
  static constexpr int ACPR = AROW / 16;    // 16-B chunks per A k-row
  static constexpr int ARPP = 256 / ACPR;   // A k-rows per DMA piece (one 16-B chunk per lane)
  static constexpr int PA = 64 / ARPP;      // A DMA pieces per K-tile
  static constexpr int OPA = 64 * AROW;     // A image bytes
  static constexpr int SB = 2 * OPA;        // B stages at SB / SB + OPB
  static constexpr int SMEMB = SB + 2 * OPB;
  static constexpr int SLABB = BM * 256;    // floats of one split's partial tile
  static constexpr int NMF = NA * NB;       // MFMAs per K-step and wave
  static constexpr int NQ = PA + 8;         // DMA pieces per K-tile
};

// fragment read order of a K-step (first use in the a-major MFMA sweep): 0: A0, 1..NB: B0..B(NB-1),
// NB+1..: A1..; two transposed reads (k-rows +0..3, +4..7 of each lane group) per fragment
template <int NA, int NB>
constexpr bool fr_is_a(int r) { return r == 0 || r > NB; }
template <int NA, int NB>
constexpr int fr_blk(int r) { return r == 0 ? 0 : (r <= NB ? r - 1 : r - NB); }

template <bool RS, bool GB, int BM = 256>
__global__ __launch_bounds__(T, 1) void gemm4t_kernel(const bf16_t* __restrict__ A, long long lda,
                                                     const bf16_t* __restrict__ B, long long ldb, int M, int N, int K,
                                                     int tiles_m, int tiles_n, int splits, int kt_per,
                                                     float* __restrict__ ws, float* __restrict__ out, int beta,
                                                     float alpha, int* __restrict__ ctr, float* __restrict__ rsw,
                                                     float* __restrict__ rowsum, Gather G, long long b_bytes) {
  using Gm = Geo<BM>;
  constexpr int NA = Gm::NA, NB = Gm::NB, NF = Gm::NF, OPA = Gm::OPA, SBO = Gm::SB;
  static_assert(!RS || BM == 256, "bias row sums on the 256-row tile");
  // 1 KB aligned: the read bases' bits 5..9 are the lane's own, so a column block is one XOR
  __shared__ __attribute__((aligned(1024))) char smem[Gm::SMEMB + 16];
  // the epilogue's arguments into SGPRs now: loaded lazily behind the main loop's first K-tile,
  // a pending scalar load at the loop header makes hipcc's LDS-read waits there lgkmcnt(0)
  // (scalar loads complete out of order)
  asm volatile("" : "+s"(out), "+s"(ws), "+s"(ctr), "+s"(rsw), "+s"(rowsum), "+s"(beta), "+s"(alpha));
  const int tiles = tiles_m * tiles_n;
  // XCD-contiguous work index, split-major: the ~32 workgroups of one XCD share a K range and a
  // block of 8 tile rows (tile_of), so their A / B panels are read once into that XCD's L2
  const int w = xcd_remap(blockIdx.x, tiles * splits);
  const int split = w / tiles, t = w - split * tiles;
  int tm, tn;
  tile_of(t, tiles_m, tiles_n, 8, tm, tn);
  const int m0 = tm * BM, n0 = tn * 256;
  const int kt0 = split * kt_per;
  const int nk = min(kt_per, K / 64 - kt0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int i16 = lane & 15, g = lane >> 4, q = i16 >> 2, p = i16 & 3;
  const int f = q | ((g & 1) << 2);

  lds_char_t* const lds = (lds_char_t*)smem;
  // per-lane read base of column block 0 of the wave's A / B columns per stage; block j is
  // base ^ (32 j): the wave's first 32-B slot s0 is a multiple of its block count, so the
  // physical slot (s0 + j) ^ f = (s0 ^ f) ^ j; K-step and half are immediates
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds));
  const uint32_t krow = static_cast<uint32_t>(8 * g + q);
  const uint32_t bA0 = sb + krow * Gm::AROW + 8 * p + 32 * ((wm * NA) ^ f);
  const uint32_t bB0 = sb + SBO + krow * 512 + 8 * p + 32 * ((wn * 8) ^ f);
  const uint32_t ldsw = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sb + wave * 1024)));
  // A loader: piece i of thread tid = A k-row i * ARPP + tid / ACPR, physical chunk tid % ACPR
  ttd_i32x4_t srd_a = make_srd(A, static_cast<uint32_t>(static_cast<long long>(K) * lda * 2));
  uint32_t voff_a[2];
  {
    const int pc = tid % Gm::ACPR, r0 = tid / Gm::ACPR;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = i * Gm::ARPP + r0;
      const int fr = (r & 3) | (((r >> 3) & 1) << 2);
      const int col = min(m0 + (((pc >> 1) ^ fr) << 4) + (pc & 1) * 8, M - 8);
      voff_a[i] = static_cast<uint32_t>((static_cast<long long>(r0) * lda + col) * 2);
    }
  }
  const int arow_step = static_cast<int>(lda * 2 * Gm::ARPP);  // bytes per A piece's k-rows
  LoadMN lb;
  GCol gc;
  uint32_t gv[8];  // GB: this lane's source offsets of the 8 B pieces of the next K-tile to load
  if constexpr (GB) {
    lb.srd = make_srd(B, static_cast<uint32_t>(b_bytes));
    const int pc = tid & 31;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int f = ((tid >> 5) & 3) | (j << 2);
      const int col = min(n0 + (((pc >> 1) ^ f) << 4) + (pc & 1) * 8, N - 8);
      const int tap = col / G.C, c = col - tap * G.C;
      gc.r[j] = tap / G.S;
      gc.s[j] = tap - gc.r[j] * G.S;
      gc.toff[j] = (gc.r[j] * G.W + gc.s[j]) * G.C + c;
    }
  } else {
    lb.init(B, ldb, K, N, n0, tid);
  }
  // GB: offsets of K-tile kt's 8 B pieces (piece i: k-row i * 8 + tid / 32)
  auto gather_piece = [&](int kt, int i) {
    if constexpr (GB) gv[i] = gather_voff(G, gc, i & 1, (kt0 + kt) * 64 + i * 8 + (tid >> 5));
  };
  const int kstride_a = static_cast<int>(lda * 128), kstride_b = static_cast<int>(ldb * 128);  // bytes per K-tile

  f32x4_t acc[NA][NB];
  ttd_s16x4_t fl[2][NF], fh[2][NF];  // [set][fragment: 0..NA-1 A, NA.. B] low / high k halves
  f32x4_t rsacc[4];
  bf16x8_t ones;
  if constexpr (RS) {
#pragma unroll
    for (int j = 0; j < 4; ++j) rsacc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    ones = __builtin_bit_cast(bf16x8_t, ttd_i32x4_t{0x3F803F80, 0x3F803F80, 0x3F803F80, 0x3F803F80});
  }

  // read r (0 .. 2 NF - 1) of K-step S of the image in stage st into fragment set SET
  auto rd1 = [&](auto R, auto S, int st, auto SET) {
    constexpr int r = decltype(R)::value, s = decltype(S)::value, set = decltype(SET)::value;
    constexpr int fr = r / 2, h = r % 2, blk = fr_blk<NA, NB>(fr);
    constexpr bool isa = fr_is_a<NA, NB>(fr);
    constexpr int imm = isa ? s * 32 * Gm::AROW + h * 4 * Gm::AROW : s * 16384 + h * 2048;
    const uint32_t base = isa ? bA0 + st * OPA : bB0 + st * OPB;
    const ttd_s16x4_t v = trd((const lds_char_t*)(uintptr_t)((blk ? (base ^ (32u * blk)) : base) + imm));
    constexpr int slot = isa ? blk : NA + blk;
    if constexpr (h == 0) fl[set][slot] = v;
    else fh[set][slot] = v;
  };
  // LDS base of piece q (0..PA-1 A, PA.. B) in stage st; pieces go out in the order (stage st:
  // all), (stage st ^ 1: all), ..., each setting M0 for its successor
  auto m0_of = [&](int qq, int st) {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(
        ldsw + (qq < Gm::PA ? st * OPA + qq * 4096 : SBO + st * OPB + (qq - Gm::PA) * 4096))));
  };
  auto dma1 = [&](auto Q, int st, int kt) {  // piece q of K-tile kt into stage st (M0 = its base)
    constexpr int qq = decltype(Q)::value;
    const uint32_t next = qq < Gm::NQ - 1 ? m0_of(qq + 1, st) : m0_of(0, st ^ 1);
    if constexpr (qq < Gm::PA) {
      dma_chain(voff_a[qq & 1], srd_a, (kt0 + kt) * kstride_a + qq * arow_step, next);
    } else {
      constexpr int i = qq - Gm::PA;
      if constexpr (GB) dma_chain(gv[i], lb.srd, 0, next);
      else dma_chain(lb.voff[i & 1], lb.srd, (kt0 + kt) * kstride_b + i * lb.row8, next);
    }
  };
  auto fa = [&](int set, int a) { return cat(fl[set][a], fh[set][a]); };
  auto fb = [&](int set, int b) { return cat(fl[set][NA + b], fh[set][NA + b]); };

  // HAS2 (K-tile kt + 2 exists) is compile-time: no branch around the DMA pieces in the
  // steady-state loop. Phases (MFMA counts for BM = 256 / 128):
  //   0  (64 / 32, K-step 0)       | the 2 NF reads of K-step 1, spread evenly
  //   1a (32 / 16, K-step 1 first half) | the A pieces of K-tile kt + 2 into the freed stage
  //   1b (32 / 16, second half)   | the B pieces of kt + 2 | the 2 NF reads of K-tile kt + 1, K-step 0
  constexpr int NR = 2 * NF, H0 = Gm::NMF, H1 = Gm::NMF / 2;
  auto ktile = [&](int kt, auto first, auto has2c) {
    constexpr bool FIRST = decltype(first)::value;
    constexpr bool has2 = decltype(has2c)::value;
    const int st = kt & 1;
    const bool rs_on = RS && ((kt0 + kt) % tiles_n == tn);
    // phase 0: K-step 0 (set 0) | reads of K-step 1 into set 1 (read j before MFMA j * H0 / NR)
    static_for<H0>([&](auto I) {
      constexpr int i = decltype(I)::value;
      static_for<NR>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if constexpr (j * H0 / NR == i) rd1(J, std::integral_constant<int, 1>{}, st, std::integral_constant<int, 1>{});
      });
      mfma_acc<FIRST>(acc[i / NB][i % NB], fa(0, i / NB), fb(0, i % NB));
      // GB: the gathered B offsets of K-tile kt + 2 (DMA'd in phase 1b), between the MFMAs
      if constexpr (GB && has2 && i % (H0 / 8) == (H0 / 8) - 3) gather_piece(kt + 2, i / (H0 / 8));
    });
    if constexpr (RS) {
      if (rs_on) {  // (wave-uniform branches: no VALU-selected operand)
        if (wn == 0) {
          static_for<4>([&](auto J) {
            constexpr int j = decltype(J)::value;
            mfma_rs<j == 3>(rsacc[j], ones, fa(0, j));
          });
        } else {
          static_for<4>([&](auto J) {
            constexpr int j = decltype(J)::value;
            mfma_rs<j == 3>(rsacc[j], ones, fa(0, 4 + j));
          });
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);  // (a real s_waitcnt: hipcc's own wait tracking sees it)
    asm volatile("s_barrier" ::: "memory");
    // phase 1a: first half of K-step 1 | A pieces of K-tile kt + 2 into the freed stage
    static_for<H1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i % (H1 / Gm::PA) == 0)
        if constexpr (has2) dma1(std::integral_constant<int, i / (H1 / Gm::PA)>{}, st, kt + 2);
      mfma_acc<false>(acc[i / NB][i % NB], fa(1, i / NB), fb(1, i % NB));
    });
    if constexpr (RS) {
      if (rs_on) {  // (wave-uniform branches: no VALU-selected operand)
        if (wn == 0) {
          static_for<4>([&](auto J) {
            constexpr int j = decltype(J)::value;
            mfma_rs<j == 3>(rsacc[j], ones, fa(1, j));
          });
        } else {
          static_for<4>([&](auto J) {
            constexpr int j = decltype(J)::value;
            mfma_rs<j == 3>(rsacc[j], ones, fa(1, 4 + j));
          });
        }
      }
    }
    if constexpr (has2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Gm::PA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    // phase 1b: second half of K-step 1 | B pieces of kt + 2 | reads of K-tile kt + 1, K-step 0
    static_for<H1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i % (H1 / 8) == (H1 / 8 > 1 ? 1 : 0))
        if constexpr (has2) dma1(std::integral_constant<int, Gm::PA + i / (H1 / 8)>{}, st, kt + 2);
      static_for<NR>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if constexpr (j * H1 / NR == i) rd1(J, std::integral_constant<int, 0>{}, st ^ 1, std::integral_constant<int, 0>{});
      });
      mfma_acc<false>(acc[NA / 2 + i / NB][i % NB], fa(1, NA / 2 + i / NB), fb(1, i % NB));
    });
  };

  // prologue: K-tiles 0 and 1 into stages 0 and 1, K-step 0 fragments of K-tile 0
  m0_init(m0_of(0, 0));
  if constexpr (GB)
    for (int i = 0; i < 8; ++i) gather_piece(0, i);
  static_for<Gm::NQ>([&](auto Q) { dma1(Q, 0, 0); });
  if constexpr (GB)
    if (nk > 1)
      for (int i = 0; i < 8; ++i) gather_piece(1, i);
  static_for<Gm::NQ>([&](auto Q) { dma1(Q, 1, 1); });
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(Gm::NQ) : "memory");
  static_for<NR>([&](auto R) { rd1(R, std::integral_constant<int, 0>{}, 0, std::integral_constant<int, 0>{}); });
  if (nk >= 3) {
    ktile(0, std::true_type{}, std::true_type{});
    for (int kt = 1; kt < nk - 2; ++kt) ktile(kt, std::false_type{}, std::true_type{});
    ktile(nk - 2, std::false_type{}, std::false_type{});
    ktile(nk - 1, std::false_type{}, std::false_type{});
  } else {
    ktile(0, std::true_type{}, std::false_type{});
    if (nk == 2) ktile(1, std::false_type{}, std::false_type{});
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) asm volatile("" : "+a"(acc[a][b]));

  // bias-gradient partials: rsw[(split * tiles_n + tn) * M + m], summed below by the last of the
  // splits * tiles_n workgroups of tile row tm to arrive
  if constexpr (RS) {
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 128 + (wn * 4 + j) * 16 + i16;
        if (m < M) rsw[static_cast<long long>(split * tiles_n + tn) * M + m] = rsacc[j][0];
      }
    }
  }
  // acc[a][b] = C[m0 + wm*(BM/2) + a*16 + i16][n0 + wn*128 + b*16 + 4g .. +3]
  const bool whole = m0 + BM <= M && n0 + 256 <= N;
  auto store = [&](int a, int b, f32x4_t v) {
    const int m = m0 + wm * (BM / 2) + a * 16 + i16, n = n0 + wn * 128 + b * 16 + 4 * g;
    if (whole || (m < M && n < N)) {
      f32x4_t* o = reinterpret_cast<f32x4_t*>(out + static_cast<long long>(m) * N + n);
      if (beta) v += *o;
      *o = v;
    }
  };
  // rows a..NA-1 re-pinned before row a is read: hipcc would otherwise move all accumulator
  // reads to the top (VGPR spills)
  auto pin_from = [&](int a0) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if (a >= a0)
#pragma unroll
        for (int b = 0; b < NB; ++b) asm volatile("" : "+a"(acc[a][b]));
  };
  const long long lin = static_cast<long long>(wave) * NA * NB * 256 + lane * 4;  // + (a * NB + b) * 256
  if (splits == 1) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      pin_from(a);
#pragma unroll
      for (int b = 0; b < NB; ++b) store(a, b, acc[a][b] * alpha);
    }
    if constexpr (!RS) return;
  } else {
    // split-K: partial tile lane-linear into this split's slab (stored straight from the AGPRs)
    float* slab = ws + static_cast<long long>(split * tiles + t) * Gm::SLABB + lin;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(slab + (a * NB + b) * 256), "a"(acc[a][b])
                     : "memory");
  }
  // release the partials, count arrivals: per tile (ctr[t], splits) and per tile row for the
  // bias gradient (ctr[tiles + tm], splits * tiles_n)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __threadfence();
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + Gm::SMEMB);
  if (tid == 0) {
    flag[0] = splits > 1 && atomicAdd(ctr + t, 1) == splits - 1;
    flag[1] = RS && atomicAdd(ctr + tiles + tm, 1) == splits * tiles_n - 1;
  }
  __syncthreads();
  const bool last_tile = flag[0], last_row = flag[1];
  if (!last_tile && !last_row) return;
  __threadfence();  // acquire: the other workgroups' partials
  if constexpr (RS) {
    if (last_row) {
      const int m = m0 + tid;
      if (m < M) {
        float sum = 0.f;  // fixed order (deterministic whoever is last)
        for (int q = 0; q < splits * tiles_n; ++q) sum += rsw[static_cast<long long>(q) * M + m];
        rowsum[m] = sum;
      }
      if (tid == 0) ctr[tiles + tm] = 0;
    }
  }
  if (!last_tile) return;
  // last split of this tile: sum the partials in split order, its own re-read from the slab it
  // just wrote (deterministic whoever is last; no accumulator stays live through the fold)
  const float* src0 = ws + static_cast<long long>(t) * Gm::SLABB + lin;
  const long long sstride = static_cast<long long>(tiles) * Gm::SLABB;
  // (one workgroup streams splits x 128 / 256 KB: the loads of 4 splits are issued before their
  // adds — 32 x 16 B in flight per lane instead of 8 — the adds stay in split order)
#pragma unroll 1
  for (int a = 0; a < NA; ++a) {
    f32x4_t v[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) v[b] = *reinterpret_cast<const f32x4_t*>(src0 + (a * NB + b) * 256);
    int s = 1;
    for (; s + 4 <= splits; s += 4) {
      f32x4_t x[4][NB];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* src = src0 + (s + u) * sstride + a * NB * 256;
#pragma unroll
        for (int b = 0; b < NB; ++b) x[u][b] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(src + b * 256));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int b = 0; b < NB; ++b) v[b] += x[u][b];
    }
    for (; s < splits; ++s) {
      const float* src = src0 + s * sstride + a * NB * 256;
#pragma unroll
      for (int b = 0; b < NB; ++b) v[b] += *reinterpret_cast<const f32x4_t*>(src + b * 256);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) store(a, b, v[b] * alpha);
  }
  if (tid == 0) ctr[t] = 0;  // ready for the next launch on this counter block
}

// ------------------------------------------------------------------------------ fp8 form
// dW[M,N] (+)= sa * sb * A8^T . B8: A8 = dy in OCP e5m2 [K][M] (K = pixels), B8 = x in e4m3 —
// dense [K][N] or the im2col gather of x [N][H][W][C] — on v_mfma_scale_f32_32x32x64_f8f6f4 (fp8
// at twice the bf16 rate; block scales fixed at 2^0, the per-tensor inverse scales sa / sb are
// device scalars applied in the epilogue). The weight gradients of the fp8 convolutions
// (precision="fp8"; the 8-wave conv_wgrad_fp8 kernel is the fallback): same K-tile footprint and
// the same phase schedule as the bf16 kernel above:
//  * K-tile = 128 k-rows x 256 B per operand (32 KB), two K-steps of 64 k;
//  * 32 x 32 fragments: lane l holds column l & 31, k = 32 (l >> 5) .. +31 of the K-step (32 B),
//    four ds_read_b64_tr_b8 (lane i of a 16-lane group addresses k-row k0 + i / 2 at column
//    byte 8 (i & 1) of its 16-column half and receives 8 consecutive k of its own column); per
//    K-step 4 A + 4 B fragments = 64 VGPRs, two sets double-buffered across the K-steps; 16
//    MFMAs of 32 passes per K-step into 4 x 4 accumulators of 16 AGPRs;
//  * LDS rows of 256 B: the 16-B chunk c of k-row r sits at c ^ ((r & 7) << 1), so the 8 k-rows
//    x 2 column halves of one half-wave's transposed read fall on 16 different chunks (each of
//    the 64 banks once); the DMA fetches, per lane, the global chunk that lands in its
//    lane-linear LDS slot (the XOR depends only on the lane: one offset per operand);
//  * output lane l, item v of accumulator (a, b): row m0 + 128 wm + 32 a + (l & 31), column
//    n0 + 128 wn + 32 b + 8 (v / 4) + 4 (l >> 5) + v % 4 (4 consecutive columns per 16-B store).
namespace f8 {
constexpr int OP = 128 * 256;     // operand K-tile image bytes
constexpr int NA = 4, NB = 4, NF = NA + NB, NMF = NA * NB, PA = 8, NQ = 16;
constexpr int SB = 2 * OP;        // B stages at SB, SB + OP
constexpr int SMEMB = 4 * OP;
constexpr int SLABB = 256 * 256;  // floats of one split's partial tile
}  // namespace f8

typedef __attribute__((ext_vector_type(2))) int ttd_i32x2_t;
typedef __attribute__((ext_vector_type(8))) int ttd_i32x8_t;
typedef __attribute__((ext_vector_type(16))) float ttd_f32x16_t;
typedef __attribute__((address_space(3))) ttd_i32x2_t lds_i2_t;

__device__ __forceinline__ ttd_i32x2_t trd8(const lds_char_t* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i2_t*)p);
}

// acc (+)= x8 . dy8 products: src0 = the B fragment (x, e4m3: cbsz 0), src1 = the A fragment (dy,
// e5m2: blgp 1), block scales `one` = 127 (2^0 in E8M0). The leading s_nop 1: hipcc may
// rematerialise `one` (a VALU write) right before the asm, and a VALU-written MFMA operand needs 2
// wait states.
template <bool FIRST>
__device__ __forceinline__ void mfma8(ttd_f32x16_t& c, const ttd_i32x8_t& a, const ttd_i32x8_t& b, int one) {
  if constexpr (FIRST)
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] blgp:1"
                 : "=a"(c)
                 : "v"(b), "v"(a), "v"(one)
                 : "memory");
  else
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] blgp:1"
                 : "+a"(c)
                 : "v"(b), "v"(a), "v"(one)
                 : "memory");
}

__device__ __forceinline__ uint32_t gather_voff8(const Gather& G, const GCol& gc, int k) {
  const int n = static_cast<int>(__umulhi(static_cast<unsigned>(k), G.pq_m) >> G.pq_s);
  const int rem = k - n * G.PQ;
  const int p = static_cast<int>(__umulhi(static_cast<unsigned>(rem), G.q_m) >> G.q_s);
  const int q = rem - p * G.Q;
  const int hb = p * G.sh - G.ph, wb = q * G.sw - G.pw;
  const bool ok = static_cast<unsigned>(hb + gc.r[0]) < static_cast<unsigned>(G.H) &&
                  static_cast<unsigned>(wb + gc.s[0]) < static_cast<unsigned>(G.W);
  return ok ? static_cast<uint32_t>(((n * G.H + hb) * G.W + wb) * G.C + gc.toff[0]) : kOob;
}

template <bool GB>
__global__ __launch_bounds__(T, 1) void gemm4t8_kernel(const uint8_t* __restrict__ A, long long lda,
                                                      const uint8_t* __restrict__ B, long long ldb, int M, int N,
                                                      int K, int tiles_m, int tiles_n, int splits, int kt_per,
                                                      float* __restrict__ ws, float* __restrict__ out, int beta,
                                                      const float* __restrict__ sa, const float* __restrict__ sbv,
                                                      int* __restrict__ ctr, Gather G, long long b_bytes) {
  using namespace f8;
  __shared__ __attribute__((aligned(1024))) char smem[SMEMB + 16];
  asm volatile("" : "+s"(out), "+s"(ws), "+s"(ctr), "+s"(beta), "+s"(sa), "+s"(sbv));
  const int tiles = tiles_m * tiles_n;
  const int w = xcd_remap(blockIdx.x, tiles * splits);
  const int split = w / tiles, t = w - split * tiles;
  int tm, tn;
  tile_of(t, tiles_m, tiles_n, 8, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int kt0 = split * kt_per;
  const int nk = min(kt_per, K / 128 - kt0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  lds_char_t* const lds = (lds_char_t*)smem;
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds));
  // fragment read base (K-step 0, read 0, fragment 0): k-row 32 (l >> 5) + (l & 15) / 2, chunk
  // (8 w | h) ^ (l & 14) with h = the lane's 16-column half; fragment j is base ^ (32 j), K-step
  // and read q are immediates (16 KB, 2 KB)
  const uint32_t rrow = static_cast<uint32_t>(32 * (lane >> 5) + ((lane & 15) >> 1));
  const uint32_t hx = static_cast<uint32_t>((lane >> 4) & 1), fx = static_cast<uint32_t>(lane & 14);
  const uint32_t bA0 = sb + rrow * 256 + ((((wm * 8) | hx) ^ fx) << 4) + 8 * (lane & 1);
  const uint32_t bB0 = sb + SB + rrow * 256 + ((((wn * 8) | hx) ^ fx) << 4) + 8 * (lane & 1);
  const uint32_t ldsw = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sb + wave * 1024)));
  // DMA: piece i of thread tid = k-row 16 i + tid / 16, physical chunk tid % 16 = logical chunk
  // (tid % 16) ^ ((tid / 16 & 7) << 1) (columns past the operand's end clamped to its last 16)
  const int pr = tid >> 4, lcol = ((tid & 15) ^ ((pr & 7) << 1)) * 16;
  const ttd_i32x4_t srd_a = make_srd(A, static_cast<uint32_t>(static_cast<long long>(K) * lda));
  const uint32_t voff_a = static_cast<uint32_t>(static_cast<long long>(pr) * lda + min(m0 + lcol, M - 16));
  ttd_i32x4_t srd_b;
  uint32_t voff_b = 0;
  GCol gc;
  uint32_t gv[8];  // GB: this lane's source offsets of the 8 B pieces of the next K-tile to load
  if constexpr (GB) {
    srd_b = make_srd(B, static_cast<uint32_t>(b_bytes));
    const int col = min(n0 + lcol, N - 16);
    const int tap = col / G.C, c = col - tap * G.C;
    gc.r[0] = tap / G.S;
    gc.s[0] = tap - gc.r[0] * G.S;
    gc.toff[0] = (gc.r[0] * G.W + gc.s[0]) * G.C + c;
  } else {
    srd_b = make_srd(B, static_cast<uint32_t>(static_cast<long long>(K) * ldb));
    voff_b = static_cast<uint32_t>(static_cast<long long>(pr) * ldb + min(n0 + lcol, N - 16));
  }
  auto gather_piece = [&](int kt, int i) {
    if constexpr (GB) gv[i] = gather_voff8(G, gc, (kt0 + kt) * 128 + i * 16 + pr);
  };
  const int kstride_a = static_cast<int>(lda * 128), kstride_b = static_cast<int>(ldb * 128);
  const int prow_a = static_cast<int>(lda * 16), prow_b = static_cast<int>(ldb * 16);
  int one = 127;
  asm volatile("" : "+v"(one));

  ttd_f32x16_t acc[NA][NB];
  ttd_i32x2_t fr[2][NF][4];  // [set][fragment: 0..NA-1 A, NA.. B][read q]

  // read r (0 .. 4 NF - 1) of K-step S of the image in stage st into fragment set SET
  auto rd1 = [&](auto R, auto S, int st, auto SET) {
    constexpr int r = decltype(R)::value, s = decltype(S)::value, set = decltype(SET)::value;
    constexpr int fi = r / 4, q = r % 4, blk = fr_blk<NA, NB>(fi);
    constexpr bool isa = fr_is_a<NA, NB>(fi);
    constexpr int imm = s * 16384 + q * 2048;
    const uint32_t base = (isa ? bA0 : bB0) + st * OP;
    fr[set][isa ? blk : NA + blk][q] = trd8((const lds_char_t*)(uintptr_t)((blk ? (base ^ (32u * blk)) : base) + imm));
  };
  auto frag = [&](int set, int slot) {
    const ttd_i32x2_t* v = fr[set][slot];
    const auto lo = __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3);
    const auto hi = __builtin_shufflevector(v[2], v[3], 0, 1, 2, 3);
    return static_cast<ttd_i32x8_t>(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto m0_of = [&](int qq, int st) {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(
        ldsw + (qq < PA ? st * OP + qq * 4096 : SB + st * OP + (qq - PA) * 4096))));
  };
  auto dma1 = [&](auto Q, int st, int kt) {  // piece q of K-tile kt into stage st (M0 = its base)
    constexpr int qq = decltype(Q)::value;
    const uint32_t next = qq < NQ - 1 ? m0_of(qq + 1, st) : m0_of(0, st ^ 1);
    if constexpr (qq < PA) {
      dma_chain(voff_a, srd_a, (kt0 + kt) * kstride_a + qq * prow_a, next);
    } else {
      constexpr int i = qq - PA;
      if constexpr (GB) dma_chain(gv[i], srd_b, 0, next);
      else dma_chain(voff_b, srd_b, (kt0 + kt) * kstride_b + i * prow_b, next);
    }
  };

  // phases per K-tile (as the bf16 kernel): 0 = K-step 0 (16 MFMAs) | the 32 reads of K-step 1;
  // 1a = first half of K-step 1 | A pieces of K-tile kt + 2 into the freed stage; 1b = second
  // half | B pieces of kt + 2 | the 32 reads of K-tile kt + 1, K-step 0
  constexpr int NR = 4 * NF, H0 = NMF, H1 = NMF / 2;
  auto ktile = [&](int kt, auto first, auto has2c) {
    constexpr bool FIRST = decltype(first)::value;
    constexpr bool has2 = decltype(has2c)::value;
    const int st = kt & 1;
    static_for<H0>([&](auto I) {
      constexpr int i = decltype(I)::value;
      static_for<NR>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if constexpr (j * H0 / NR == i) rd1(J, std::integral_constant<int, 1>{}, st, std::integral_constant<int, 1>{});
      });
      mfma8<FIRST>(acc[i / NB][i % NB], frag(0, i / NB), frag(0, NA + i % NB), one);
      if constexpr (GB && has2 && (i & 1)) gather_piece(kt + 2, i / 2);
    });
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    asm volatile("s_barrier" ::: "memory");
    static_for<H1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (has2) dma1(std::integral_constant<int, i>{}, st, kt + 2);
      mfma8<false>(acc[i / NB][i % NB], frag(1, i / NB), frag(1, NA + i % NB), one);
    });
    if constexpr (has2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    static_for<H1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (has2) dma1(std::integral_constant<int, PA + i>{}, st, kt + 2);
      static_for<NR>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if constexpr (j * H1 / NR == i) rd1(J, std::integral_constant<int, 0>{}, st ^ 1, std::integral_constant<int, 0>{});
      });
      mfma8<false>(acc[NA / 2 + i / NB][i % NB], frag(1, NA / 2 + i / NB), frag(1, NA + i % NB), one);
    });
  };

  // prologue: K-tiles 0 and 1 into stages 0 and 1, K-step 0 fragments of K-tile 0
  m0_init(m0_of(0, 0));
  if constexpr (GB)
    for (int i = 0; i < 8; ++i) gather_piece(0, i);
  static_for<NQ>([&](auto Q) { dma1(Q, 0, 0); });
  if constexpr (GB)
    if (nk > 1)
      for (int i = 0; i < 8; ++i) gather_piece(1, i);
  static_for<NQ>([&](auto Q) { dma1(Q, 1, 1); });
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NQ) : "memory");
  static_for<NR>([&](auto R) { rd1(R, std::integral_constant<int, 0>{}, 0, std::integral_constant<int, 0>{}); });
  if (nk >= 3) {
    ktile(0, std::true_type{}, std::true_type{});
    for (int kt = 1; kt < nk - 2; ++kt) ktile(kt, std::false_type{}, std::true_type{});
    ktile(nk - 2, std::false_type{}, std::false_type{});
    ktile(nk - 1, std::false_type{}, std::false_type{});
  } else {
    ktile(0, std::true_type{}, std::false_type{});
    if (nk == 2) ktile(1, std::false_type{}, std::false_type{});
  }
  // a 32-pass MFMA's result: >= 34 wait states before a non-MFMA reader
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) asm volatile("" : "+a"(acc[a][b]));

  const float scale = sa[0] * sbv[0];
  const bool whole = m0 + 256 <= M && n0 + 256 <= N;
  auto store = [&](int a, int b, int v4, f32x4_t v) {
    const int m = m0 + wm * 128 + a * 32 + (lane & 31), n = n0 + wn * 128 + b * 32 + 8 * v4 + 4 * (lane >> 5);
    if (whole || (m < M && n < N)) {
      f32x4_t* o = reinterpret_cast<f32x4_t*>(out + static_cast<long long>(m) * N + n);
      if (beta) v += *o;
      *o = v;
    }
  };
  auto part = [&](const ttd_f32x16_t& c, int v4) {
    return f32x4_t{c[4 * v4], c[4 * v4 + 1], c[4 * v4 + 2], c[4 * v4 + 3]};
  };
  // lane-linear partial tile: accumulator (a, b), quarter v4 at ((a NB + b) 4 + v4) 256 + 4 lane
  const long long lin = static_cast<long long>(wave) * NMF * 1024 + lane * 4;
  if (splits == 1) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        asm volatile("" : "+a"(acc[a][b]));
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4) store(a, b, v4, part(acc[a][b], v4) * scale);
      }
    return;
  }
  float* slab = ws + static_cast<long long>(split * tiles + t) * SLABB + lin;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      asm volatile("" : "+a"(acc[a][b]));
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4)
        *reinterpret_cast<f32x4_t*>(slab + ((a * NB + b) * 4 + v4) * 256) = part(acc[a][b], v4);
    }
  // release the partials, count arrivals per tile
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __threadfence();
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + SMEMB);
  if (tid == 0) flag[0] = atomicAdd(ctr + t, 1) == splits - 1;
  __syncthreads();
  if (!flag[0]) return;
  __threadfence();  // acquire: the other splits' partials
  // last split of this tile: the partials summed in split order (deterministic whoever is last)
  const float* src0 = ws + static_cast<long long>(t) * SLABB + lin;
  const long long sstride = static_cast<long long>(tiles) * SLABB;
#pragma unroll 1
  for (int ab = 0; ab < NMF; ++ab) {
    f32x4_t v[4];
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4) v[v4] = *reinterpret_cast<const f32x4_t*>(src0 + (ab * 4 + v4) * 256);
    int s = 1;
    for (; s + 4 <= splits; s += 4) {
      f32x4_t x[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4)
          x[u][v4] = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4_t*>(src0 + (s + u) * sstride + (ab * 4 + v4) * 256));
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4) v[v4] += x[u][v4];
    }
    for (; s < splits; ++s)
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4)
        v[v4] += *reinterpret_cast<const f32x4_t*>(src0 + s * sstride + (ab * 4 + v4) * 256);
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4) store(ab / NB, ab % NB, v4, v[v4] * scale);
  }
  if (tid == 0) ctr[t] = 0;  // ready for the next launch on this counter block
}

}  // namespace g4t
}  // namespace
}  // namespace ttdk

static int g4t_enabled() {
  static const int v = ttdk::getenv_int("TTD_G4T", 1);
  return v;
}

// tile rows: 128 when the output has at most 128 rows (a 256-row tile would run half its MFMAs
// on padding), else 256; the bias row sums (BERT) use the 256-row form. TTD_G4T_BM128=0: always 256.
static int g4t_bm(int M, bool rowsum) {
  static const int v = ttdk::getenv_int("TTD_G4T_BM128", 1);
  return (v && !rowsum && M <= 128) ? 128 : 256;
}

// floats of workspace ttdk_gemm4t_wgrad needs: split partial tiles + bias-gradient partials;
// -1 when the kernel would refuse the shape (the same admission checks as ttdk_gemm4t_wgrad,
// except the leading dimensions / pointers, with lda = M and ldb = N)
TTDK_EXPORT long long ttdk_gemm4t_ws(int M, int N, int K, int splits) {
  using namespace ttdk;
  const long long lim = 1LL << 31;
  if (!g4t_enabled() || K % 64 || K < 128 || M < 8 || N < 8 || M % 8 || N % 8 ||
      static_cast<long long>(K) * M * 2 >= lim || static_cast<long long>(K) * N * 2 >= lim)
    return -1;
  const int ktiles = K / 64;
  splits = std::max(1, std::min(splits, ktiles / 2));
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  // (sized for 256-row tiles: at least the 128-row form's need, and the bias row-sum form's)
  const int tiles_m = ceil_div(M, 256), tiles_n = ceil_div(N, 256);
  return static_cast<long long>(splits) * tiles_m * tiles_n * 256 * 256 + static_cast<long long>(splits) * tiles_n * M;
}

// dW[M,N] (+)= alpha * A^T . B, A [K][M] (lda), B [K][N] (ldb) bf16 MN-major, out fp32 contiguous
// [M][N]; rowsum (optional): bias gradient sum_k A[k][m], written. ws: ttdk_gemm4t_ws floats.
// Returns hipErrorInvalidValue for shapes this kernel does not take (the caller keeps another path).
TTDK_EXPORT int ttdk_gemm4t_wgrad(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                  int splits, float* ws, float* out, int beta, float alpha, float* rowsum,
                                  hipStream_t st) {
  using namespace ttdk;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const long long lim = 1LL << 31;
  if (!g4t_enabled() || K % 64 || K < 128 || M < 8 || N < 8 || M % 8 || N % 8 || lda % 8 || ldb % 8 || lda < M ||
      ldb < N || !al16(A) || !al16(B) || !al16(out) || static_cast<long long>(K) * lda * 2 >= lim ||
      static_cast<long long>(K) * ldb * 2 >= lim)
    return hipErrorInvalidValue;
  const int ktiles = K / 64;
  splits = std::max(1, std::min(splits, ktiles / 2));
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  const int bm = g4t_bm(M, rowsum != nullptr);
  const int tiles_m = ceil_div(M, bm), tiles_n = ceil_div(N, 256), tiles = tiles_m * tiles_n;
  int* ctr = nullptr;
  if (splits > 1 || rowsum) {
    ctr = big::tile_counters(st, tiles + tiles_m);
    if (!ctr || !ws) return hipErrorInvalidValue;
  }
  float* rsw = rowsum ? ws + static_cast<long long>(splits) * tiles * bm * 256 : nullptr;
  const dim3 grid(tiles * splits);
  const g4t::Gather G{};
  if (rowsum)
    hipLaunchKernelGGL((g4t::gemm4t_kernel<true, false>), grid, dim3(g4t::T), 0, st, A, lda, B, ldb, M, N, K, tiles_m,
                       tiles_n, splits, per, ws, out, beta, alpha, ctr, rsw, rowsum, G, 0LL);
  else if (bm == 128)
    hipLaunchKernelGGL((g4t::gemm4t_kernel<false, false, 128>), grid, dim3(g4t::T), 0, st, A, lda, B, ldb, M, N, K,
                       tiles_m, tiles_n, splits, per, ws, out, beta, alpha, ctr, rsw, rowsum, G, 0LL);
  else
    hipLaunchKernelGGL((g4t::gemm4t_kernel<false, false>), grid, dim3(g4t::T), 0, st, A, lda, B, ldb, M, N, K, tiles_m,
                       tiles_n, splits, per, ws, out, beta, alpha, ctr, rsw, rowsum, G, 0LL);
  return hipGetLastError();
}

namespace {
// multiply-high magic for q = n / d, exact for 0 <= n < 2^31 (d >= 2): s = ceil(log2 d) - 1,
// m = floor(2^(32 + s) / d) + 1 (< 2^32); error (m d - 2^(32+s)) n / (d 2^(32+s)) < 1 / d
void magic_div(unsigned d, unsigned* m, int* s) {
  int l = 0;
  while ((1u << l) < d) ++l;
  *s = l > 0 ? l - 1 : 0;
  *m = static_cast<unsigned>(((static_cast<unsigned __int128>(1) << (32 + *s)) / d) + 1);
}
}  // namespace

// floats of workspace ttdk_conv_wgrad4t needs (-1: the kernel does not take the conv)
TTDK_EXPORT long long ttdk_conv_wgrad4t_ws(const TtdkConv* g, int splits) {
  const int M = g->K, N = g->R * g->S * g->C;
  const long long K = static_cast<long long>(g->N) * g->P * g->Q;
  const long long xb = static_cast<long long>(g->N) * g->H * g->W * g->C * 2, yb = K * g->K * 2;
  if (g->C % 8 || g->K % 8 || K % 64 || K < 128 || g->dh != 1 || g->dw != 1 || xb >= (1LL << 31) ||
      yb >= (1LL << 31) || g->P * g->Q < 2 || g->Q < 2)
    return -1;
  return ttdk_gemm4t_ws(M, N, static_cast<int>(K), splits);
}

// Convolution weight gradient dw[K][R][S][C] (+)= sum over pixels of dy (x) im2col(x) on the 4-wave
// transposed-read kernel: A = dy [pixels][K] (MN-major), B = x read through the im2col gather
// (dense [pixels][C] for unit-stride 1x1 convs); split-K summed inside the launch (no fold pass).
// ws: ttdk_conv_wgrad4t_ws floats. hipErrorInvalidValue: the kernel does not take the conv.
TTDK_EXPORT int ttdk_conv_wgrad4t(const bf16_t* x, const bf16_t* dy, const TtdkConv* g, float* dw, float* ws,
                                  int splits, int beta, hipStream_t st) {
  using namespace ttdk;
  if (ttdk_conv_wgrad4t_ws(g, splits) < 0 || !g4t_enabled()) return hipErrorInvalidValue;
  if (is_pointwise(g))
    return ttdk_gemm4t_wgrad(dy, g->K, x, g->C, g->K, g->C, g->N * g->P * g->Q, splits, ws, dw, beta, 1.f, nullptr, st);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al16(x) || !al16(dy) || !al16(dw) || !ws) return hipErrorInvalidValue;
  const int M = g->K, N = g->R * g->S * g->C, K = g->N * g->P * g->Q;
  const int ktiles = K / 64;
  splits = std::max(1, std::min(splits, ktiles / 2));
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  const int bm = g4t_bm(M, false);
  const int tiles_m = ceil_div(M, bm), tiles_n = ceil_div(N, 256), tiles = tiles_m * tiles_n;
  int* ctr = nullptr;
  if (splits > 1) {
    ctr = big::tile_counters(st, tiles);
    if (!ctr) return hipErrorInvalidValue;
  }
  g4t::Gather G{};
  G.H = g->H;
  G.W = g->W;
  G.C = g->C;
  G.Q = g->Q;
  G.PQ = g->P * g->Q;
  G.S = g->S;
  G.sh = g->sh;
  G.sw = g->sw;
  G.ph = g->ph;
  G.pw = g->pw;
  magic_div(static_cast<unsigned>(G.PQ), &G.pq_m, &G.pq_s);
  magic_div(static_cast<unsigned>(G.Q), &G.q_m, &G.q_s);
  const long long xb = static_cast<long long>(g->N) * g->H * g->W * g->C * 2;
  if (bm == 128)
    hipLaunchKernelGGL((g4t::gemm4t_kernel<false, true, 128>), dim3(tiles * splits), dim3(g4t::T), 0, st, dy,
                       static_cast<long long>(g->K), x, 0LL, M, N, K, tiles_m, tiles_n, splits, per, ws, dw, beta, 1.f,
                       ctr, nullptr, nullptr, G, xb);
  else
    hipLaunchKernelGGL((g4t::gemm4t_kernel<false, true>), dim3(tiles * splits), dim3(g4t::T), 0, st, dy,
                       static_cast<long long>(g->K), x, 0LL, M, N, K, tiles_m, tiles_n, splits, per, ws, dw, beta, 1.f,
                       ctr, nullptr, nullptr, G, xb);
  return hipGetLastError();
}

// floats of workspace ttdk_conv_wgrad4t8 needs (-1: the fp8 kernel does not take the conv): C and
// K multiples of 16 (16-B DMA chunks of 16 channels), >= 16 output rows / columns, pixels a
// multiple of 128 (whole K-tiles), operands under 2 GiB (the gather's out-of-range offset)
TTDK_EXPORT long long ttdk_conv_wgrad4t8_ws(const TtdkConv* g, int splits) {
  using namespace ttdk;
  const int M = g->K, N = g->R * g->S * g->C;
  const long long K = static_cast<long long>(g->N) * g->P * g->Q;
  const long long xb = static_cast<long long>(g->N) * g->H * g->W * g->C, yb = K * g->K;
  if (!g4t_enabled() || g->C % 16 || g->K % 16 || M < 16 || N < 16 || K % 128 || K < 128 || g->dh != 1 ||
      g->dw != 1 || xb >= (1LL << 31) || yb >= (1LL << 31) || (!is_pointwise(g) && (g->P * g->Q < 2 || g->Q < 2)))
    return -1;
  const int ktiles = static_cast<int>(K / 128);
  splits = std::max(1, std::min(splits, ktiles / 2));
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  return static_cast<long long>(splits) * ceil_div(M, 256) * ceil_div(N, 256) * 256 * 256;
}

// fp8 convolution weight gradient dw[K][R][S][C] (+)= sa * sx * sum over pixels of dy8 (x) im2col(x8)
// on the 4-wave transposed-read kernel (g4t::gemm4t8_kernel): dy8 [pixels][K] OCP e5m2, x8 e4m3
// ([pixels][C] for unit-stride 1x1 convs, else gathered), sa / sx the inverse quantisation scales
// (device fp32); split-K summed inside the launch. ws: ttdk_conv_wgrad4t8_ws floats.
// hipErrorInvalidValue: the kernel does not take the conv (the caller keeps conv_wgrad_fp8).
TTDK_EXPORT int ttdk_conv_wgrad4t8(const uint8_t* x8, const uint8_t* dy8, const TtdkConv* g, float* dw, float* ws,
                                   int splits, int beta, const float* sa, const float* sx, hipStream_t st) {
  using namespace ttdk;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (ttdk_conv_wgrad4t8_ws(g, splits) < 0 || !sa || !sx || !al16(x8) || !al16(dy8) || !al16(dw))
    return hipErrorInvalidValue;
  const int M = g->K, N = g->R * g->S * g->C, K = g->N * g->P * g->Q;
  const int ktiles = K / 128;
  splits = std::max(1, std::min(splits, ktiles / 2));
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  const int tiles_m = ceil_div(M, 256), tiles_n = ceil_div(N, 256), tiles = tiles_m * tiles_n;
  int* ctr = nullptr;
  if (splits > 1) {
    ctr = big::tile_counters(st, tiles);
    if (!ctr || !ws) return hipErrorInvalidValue;
  }
  g4t::Gather G{};
  const dim3 grid(tiles * splits);
  if (is_pointwise(g)) {
    hipLaunchKernelGGL((g4t::gemm4t8_kernel<false>), grid, dim3(g4t::T), 0, st, dy8, static_cast<long long>(g->K), x8,
                       static_cast<long long>(g->C), M, N, K, tiles_m, tiles_n, splits, per, ws, dw, beta, sa, sx, ctr,
                       G, 0LL);
    return hipGetLastError();
  }
  G.H = g->H;
  G.W = g->W;
  G.C = g->C;
  G.Q = g->Q;
  G.PQ = g->P * g->Q;
  G.S = g->S;
  G.sh = g->sh;
  G.sw = g->sw;
  G.ph = g->ph;
  G.pw = g->pw;
  magic_div(static_cast<unsigned>(G.PQ), &G.pq_m, &G.pq_s);
  magic_div(static_cast<unsigned>(G.Q), &G.q_m, &G.q_s);
  const long long xb = static_cast<long long>(g->N) * g->H * g->W * g->C;
  hipLaunchKernelGGL((g4t::gemm4t8_kernel<true>), grid, dim3(g4t::T), 0, st, dy8, static_cast<long long>(g->K), x8, 0LL,
                     M, N, K, tiles_m, tiles_n, splits, per, ws, dw, beta, sa, sx, ctr, G, xb);
  return hipGetLastError();
}
