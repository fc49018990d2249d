// 4-wave 256 x 256 bf16 GEMM: one wave per SIMD, 128 x 128 outputs per wave, the 64 fp32
// accumulator tiles (256 registers) in the AGPR half of the register file.
//
// Why a second 256-row main loop (gemm_conv.h big::gemm256*_kernel is the 8-wave ping-pong
// form): at the BERT-Large FFN1 shape the 8-wave loop keeps the MFMA pipes 50 % busy and its
// waves wait 34 % of their cycles (two waves per SIMD taking turns at barriers; 24
// ds_read_b128 per 64 MFMAs), where a 4-wave tile of 128 x 128 per wave reads half the LDS
// bytes per MFMA (32 ds_read_b128 per 128 MFMAs) and needs no turn-taking
// (profiles/r3_gemm_pmc_ours_vs_hipblaslt.txt). Reference op: tf.layers.dense MatMul,
// /root/reference/distribute_training.py:54,61 and its gradients (:152).
//
// Structure (K-major A and B; C = A . B^T, A [M][K], B [N][K]):
//  * operand tiles reach LDS by buffer_load ... lds (LDS-DMA, 16 B per lane) from a buffer
//    resource per operand: one VGPR of per-lane offset per operand, the piece / K-tile offsets
//    are scalar (soffset), and rows past M / N read zeros (out-of-range buffer loads);
//  * LDS: two stages of one 64-deep K-tile each (A 256 x 128 B + B 256 x 128 B = 64 KB);
//    rows of 128 B with the 16-B chunk index XOR (row >> 1) & 7 (conflict-free b128 reads);
//  * per K-tile and wave: 32 ds_read_b128 (16 per 32-deep K-step, double-buffered fragment
//    registers) and 128 v_mfma_f32_16x16x32_bf16; the schedule is
//      phase 0: MFMAs of K-step 0 | fragment reads of K-step 1
//      lgkmcnt(0), barrier (the stage is free)
//      phase 1a: first 32 MFMAs of K-step 1 | LDS-DMA of K-tile kt + 2 into the freed stage
//      vmcnt(DMA of kt + 2 in flight), barrier (K-tile kt + 1 has landed for every wave)
//      phase 1b: last 32 MFMAs of K-step 1 | fragment reads of K-tile kt + 1, K-step 0
//    so every DMA has a whole K-tile of MFMA work (2048 MFMA cycles) to land;
//  * MFMA operands swapped (D = B . A^T) so a lane holds 4 consecutive output columns of one
//    row; the register epilogue pairs lanes (g, g ^ 1) for 16-B stores.
#include "gemm_conv.h"

#include <type_traits>

typedef __attribute__((ext_vector_type(4))) int ttd_i32x4_t;
extern "C" __device__ void ttd_raw_buffer_load_lds(ttd_i32x4_t rsrc, __attribute__((address_space(3))) void* lds,
                                                   int size, int voffset, int soffset, int offset,
                                                   int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

namespace ttdk {
namespace {
namespace g4 {

constexpr int BM = 256, BN = 256, T = 256;
constexpr int OPB = 256 * 128;  // bytes of one operand's K-tile image
constexpr int STAGE = 2 * OPB;  // A then B
constexpr int SMEM = 2 * STAGE; // 128 KB

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ ttd_i32x4_t make_srd(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  ttd_i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane(static_cast<int>((a >> 32) & 0xffffu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r[3] = 0x00020000;
  return r;
}

// K-major operand loader: 256 rows x 128 B per K-tile in 8 LDS-DMA pieces per thread. Piece i
// of thread tid: LDS bytes (i * 256 + tid) * 16 = image row i * 32 + tid / 8, slot tid % 8, which
// holds chunk slot ^ ((row >> 1) & 7) = (tid & 7) ^ ((tid >> 4) & 7) for every i (32-row steps
// leave the swizzle term unchanged). Rows past the operand's end are clamped to its last row
// (their outputs are never stored), so every access is in range whatever the buffer unit does
// with soffset in its range check; the K-tile offset is scalar (soffset).
struct LoadK {
  ttd_i32x4_t srd;
  uint32_t voff[8];
  __device__ __forceinline__ void init(const bf16_t* p, long long ld, int rows, int row0, int tid) {
    const uint32_t bytes = static_cast<uint32_t>(static_cast<long long>(rows) * ld * 2);
    srd = make_srd(p, bytes);
    const int chunk = (tid & 7) ^ ((tid >> 4) & 7);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = min(row0 + i * 32 + (tid >> 3), rows - 1);
      voff[i] = static_cast<uint32_t>((static_cast<long long>(r) * ld + chunk * 8) * 2);
    }
  }
  // pieces [I0, I1) of K-tile kt into the operand image at lds (wave-uniform)
  template <int I0, int I1>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = I0; i < I1; ++i)
      ttd_raw_buffer_load_lds(srd, (lds_void_t*)(lds + i * 4096 + wave * 1024), 16, static_cast<int>(voff[i]),
                              kt * 128, 0, 0);
  }
};

// Implicit-GEMM convolution A operand (AOP = 1): GEMM row = output pixel (n, p, q), K = (r, s, c)
// with one 64-channel K-tile inside one filter tap (C % 64 == 0). A row's K-tile address is the
// pixel's window-corner offset (per lane, per piece) plus the tap's offset (r W + s) C + c0
// (scalar, advanced by a cursor as the DMA walks the K-tiles); the buffer base sits SHIFT =
// (ph W + pw) C bytes before x so every in-image offset is >= 0. A tap outside the image (the
// padding) or a row past M gets an offset past the buffer's end: the buffer load returns zeros.
struct ConvA {
  int H, W, C, PQ, Q, sh, sw, ph, pw, R, S;
  int flip;  // data gradient: taps walked in the filter's reversed order (the [C][R][S][K] B operand)
  long long x_bytes;
};
constexpr uint32_t kOob = 0x80000000u;
struct LoadConv {
  ttd_i32x4_t srd;
  uint32_t voff[8];
  uint32_t vmask[8];  // bit t: tap t = r S + s lies inside the image for this piece's row
  __device__ __forceinline__ void init(const bf16_t* x, const ConvA& c, int M, int row0, int tid) {
    const long long shift = (static_cast<long long>(c.ph) * c.W + c.pw) * c.C * 2;
    srd = make_srd(reinterpret_cast<const char*>(x) - shift, static_cast<uint32_t>(c.x_bytes + shift));
    const int chunk = (tid & 7) ^ ((tid >> 4) & 7);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = row0 + i * 32 + (tid >> 3);
      const int mm = m < M ? m : 0;
      const int n = mm / c.PQ, rem = mm - n * c.PQ;
      const int p = rem / c.Q, q = rem - p * c.Q;
      const int h0 = p * c.sh - c.ph, w0 = q * c.sw - c.pw;
      voff[i] = static_cast<uint32_t>(((static_cast<long long>(n) * c.H + h0) * c.W + w0) * c.C * 2 + shift + chunk * 16);
      uint32_t mk = 0;
      for (int r = 0; r < c.R; ++r)
        for (int s2 = 0; s2 < c.S; ++s2)
          if (m < M && static_cast<unsigned>(h0 + r) < static_cast<unsigned>(c.H) &&
              static_cast<unsigned>(w0 + s2) < static_cast<unsigned>(c.W))
            mk |= 1u << (r * c.S + s2);
      vmask[i] = mk;
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int tap) const { return (vmask[i] >> tap) & 1u ? voff[i] : kOob; }
};
constexpr int kEkStat = 32;  // BN partial sums (sum, sum of squares) of the stored output per 128 rows
// feeding-BN epilogue of a data gradient (E.by, E.bmask, E.stat): stores g = dx * ReLU bits of the
// feeding conv+BN unit and its backward partial sums (sum g, sum g * y) per 128 rows
constexpr int kEkFeed = 64;

// sum over the 16 lanes of a DPP row (lane 15 of the row ends with the total)
__device__ __forceinline__ float row_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, false));
  return v;
}

__device__ __forceinline__ bf16x8_t rd(const char* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA piece with M0 already holding its LDS base; sets M0 for the NEXT piece right after
// issuing (the next piece is MFMAs away, so the SALU-write -> LDS-DMA-read hazard needs no
// s_nop): 2 issue slots per piece instead of a save / set / nop / restore sequence. Only valid
// where nothing else writes M0 (the compiler does not use it in these kernels: ds_* need no M0
// on gfx950 and every LDS-DMA here is this asm).
__device__ __forceinline__ void dma_chain(uint32_t voff, const ttd_i32x4_t& srd, int soff, uint32_t next_m0) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds\n\ts_mov_b32 m0, %3"
               :
               : "v"(voff), "s"(srd), "s"(soff), "s"(next_m0)
               : "memory");
}
__device__ __forceinline__ void m0_init(uint32_t v) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(v) : "memory");
}
using big::kEkBias;
using big::kEkDGelu;
using big::kEkBeta;
using big::kEkAux;
using big::kEkGelu;

// Register epilogue: acc[a][b] = C[m0 + wm*128 + a*16 + (lane & 15)][n0 + wn*128 + b*16 + 4*(lane >> 4) + v].
// Lanes g and g ^ 1 (g = lane >> 4) swap halves of the column-block pair (2p, 2p + 1) with ONE
// v_permlane16_swap per packed dword so each lane stores 8 consecutive columns (16 B): 16 rows
// x 64 B per store instruction. Measured with in-kernel stamps, the first form of this epilogue
// (a ds_bpermute round trip per exchange, one dependent bias / residual load per 4 columns) took
// 23k cycles per tile for bias + store alone, half the K = 1024 main loop: now the bias of the
// wave's 128 columns is loaded once (8 x 16 B) and residual / old-output loads run one row block
// ahead of the arithmetic.
template <int EK, bool CHECK>
__device__ __forceinline__ void epilogue(const f32x4_t (&acc)[8][8], const EpiParams& E, int m0, int n0, int M, int N,
                                         float alpha, int lane, int wm, int wn) {
  const int g = lane >> 4, i16 = lane & 15;
  const bool odd = g & 1;
  bf16_t* const out = static_cast<bf16_t*>(E.out);
  const int ncol = n0 + wn * 128 + 4 * g;  // column of block b = ncol + 16 b
  f32x4_t bias[8];
  if constexpr ((EK & kEkBias) != 0) {
#pragma unroll
    for (int b = 0; b < 8; ++b)
      bias[b] = (!CHECK || ncol + 16 * b < N) ? *reinterpret_cast<const f32x4_t*>(E.bias + ncol + 16 * b)
                                              : f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  constexpr bool FEED = (EK & kEkFeed) != 0;
  constexpr bool STATS = FEED || (EK & kEkStat) != 0;
  constexpr bool LD = (EK & (kEkDGelu | kEkBeta)) != 0;
  // STATS: per-lane column partials of the 4 columns of every block b (sum, sum of squares — FEED:
  // sum of g and of g * y); the 16 lanes of a group hold the same columns (rows i16 + 16 a)
  float ssum[8][4], ssq[8][4];
  if constexpr (STATS) {
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) ssum[b][j] = ssq[b][j] = 0.f;
  }
  uint2 ldv[2][8];  // [row-block parity][b]: residual (dGELU) or old output (beta), one row block ahead
  uint2 ldy[2][8];  // FEED: the feeding unit's conv output y, one row block ahead
  uint32_t ldk[2][2];  // FEED: its ReLU bits, block b's byte (8 channels holding the lane's 4) at bits 8 (b & 3) of word b >> 2
  auto load_rows = [&](int a, uint2 (&v)[8], uint2 (&yv)[8], uint32_t (&kv)[2]) {
    const int m = m0 + wm * 128 + a * 16 + i16;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int n = ncol + 16 * b;
      v[b] = make_uint2(0, 0);
      if constexpr (FEED) {
        yv[b] = make_uint2(0, 0);
        if ((b & 3) == 0) kv[b >> 2] = 0;
      }
      if (!CHECK || (m < M && n < N)) {
        if constexpr ((EK & kEkDGelu) != 0)
          v[b] = *reinterpret_cast<const uint2*>(E.residual + static_cast<long long>(m) * E.ldr + n);
        else if constexpr ((EK & kEkBeta) != 0)
          v[b] = *reinterpret_cast<const uint2*>(out + static_cast<long long>(m) * E.ldo + n);
        if constexpr (FEED) {
          const long long o = static_cast<long long>(m) * E.ldo + n;
          yv[b] = *reinterpret_cast<const uint2*>(E.by + o);
          kv[b >> 2] |= static_cast<uint32_t>(E.bmask ? E.bmask[o >> 3] : 0xffu) << (8 * (b & 3));
        }
      }
    }
  };
  if constexpr (LD || FEED) load_rows(0, ldv[0], ldy[0], ldk[0]);
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    if constexpr (LD || FEED)
      if (a + 1 < 8) load_rows(a + 1, ldv[(a + 1) & 1], ldy[(a + 1) & 1], ldk[(a + 1) & 1]);
    const int m = m0 + wm * 128 + a * 16 + i16;
    const bool mok = !CHECK || m < M;
    const long long row = static_cast<long long>(m) * E.ldo;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      uint32_t po[2][2], pa[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int b = 2 * p + j;
        f32x4_t v = acc[a][b] * alpha;
        if constexpr ((EK & kEkBias) != 0) v += bias[b];
        if constexpr (LD) {
          const uint2 w = ldv[a & 1][b];
          const float x0 = bf2f(static_cast<bf16_t>(w.x & 0xffff)), x1 = bf2f(static_cast<bf16_t>(w.x >> 16));
          const float x2 = bf2f(static_cast<bf16_t>(w.y & 0xffff)), x3 = bf2f(static_cast<bf16_t>(w.y >> 16));
          if constexpr ((EK & kEkDGelu) != 0) {
            v[0] *= gelu_tanh_grad(x0);
            v[1] *= gelu_tanh_grad(x1);
            v[2] *= gelu_tanh_grad(x2);
            v[3] *= gelu_tanh_grad(x3);
          } else {
            v[0] += x0;
            v[1] += x1;
            v[2] += x2;
            v[3] += x3;
          }
        }
        if constexpr ((EK & kEkAux) != 0) {
          pa[j][0] = pack_bf16x2(v[0], v[1]);
          pa[j][1] = pack_bf16x2(v[2], v[3]);
        }
        if constexpr ((EK & kEkGelu) != 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = gelu_tanh(v[q]);
        }
        if constexpr (FEED) {  // the masked gradient g = dx * relu'(the feeding unit's output)
          const uint32_t bits = (ldk[a & 1][b >> 2] >> (8 * (b & 3))) >> (ncol & 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = (bits >> q) & 1u ? v[q] : 0.f;
        }
        po[j][0] = pack_bf16x2(v[0], v[1]);
        po[j][1] = pack_bf16x2(v[2], v[3]);
        if constexpr (STATS) {  // statistics of the values actually stored
          if (mok) {
            float r[4];
            r[0] = bf2f(static_cast<bf16_t>(po[j][0] & 0xffff));
            r[1] = bf2f(static_cast<bf16_t>(po[j][0] >> 16));
            r[2] = bf2f(static_cast<bf16_t>(po[j][1] & 0xffff));
            r[3] = bf2f(static_cast<bf16_t>(po[j][1] >> 16));
            float yy[4] = {r[0], r[1], r[2], r[3]};
            if constexpr (FEED) {
              const uint2 w = ldy[a & 1][b];
              yy[0] = bf2f(static_cast<bf16_t>(w.x & 0xffff));
              yy[1] = bf2f(static_cast<bf16_t>(w.x >> 16));
              yy[2] = bf2f(static_cast<bf16_t>(w.y & 0xffff));
              yy[3] = bf2f(static_cast<bf16_t>(w.y >> 16));
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              ssum[b][q] += r[q];
              ssq[b][q] += r[q] * yy[q];
            }
          }
        }
      }
      // even rows (g even) keep block 2p's own columns and receive the odd neighbour's; odd
      // rows receive the even neighbour's block 2p + 1 columns: 8 consecutive columns per lane
      const int nst = odd ? ncol + 32 * p + 12 : ncol + 32 * p;
      auto swap_store = [&](uint32_t (&q)[2][2], bf16_t* base) {
        const auto s0 = __builtin_amdgcn_permlane16_swap(q[0][0], q[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(q[0][1], q[1][1], false, false);
        const uint4 w = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        if (mok && (!CHECK || nst < N)) *reinterpret_cast<uint4*>(base + row + nst) = w;
      };
      swap_store(po, out);
      if constexpr ((EK & kEkAux) != 0) swap_store(pa, E.aux);
    }
  }
  if constexpr (STATS) {
    // the 16 rows of a lane group hold the same columns: sum them across the DPP row; lane 15
    // writes this wave's 128-row partial row (m0 / 128 + wm) of E.stat [2 tiles_m][2][N]
    float* const st = E.stat + static_cast<long long>((m0 / 128) + wm) * 2 * N;
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float sa = row_sum16(ssum[b][j]), sb = row_sum16(ssq[b][j]);
        const int n = ncol + 16 * b + j;
        if (i16 == 15 && (!CHECK || n < N)) {
          st[n] = sa;
          st[N + n] = sb;
        }
      }
  }
}

template <int N, class F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

// read #r of a K-step's 16 fragments in first-use order of the a-major MFMA sweep:
// r = 0: A block 0; 1..8: B blocks 0..7; 9..15: A blocks 1..7
constexpr bool rd_is_a(int r) { return r == 0 || r >= 9; }
constexpr int rd_blk(int r) { return r == 0 ? 0 : (r <= 8 ? r - 1 : r - 8); }
constexpr int rd_of_a(int a) { return a == 0 ? 0 : 8 + a; }
constexpr int rd_of_b(int b) { return 1 + b; }
constexpr int cmax(int x, int y) { return x > y ? x : y; }
// phase-0 MFMA i = (a, b) = (i / 8, i % 8) needs K-step-0 reads up to need0(i); the K-step-1 reads
// issued before it (one before every 4th MFMA) are younger: lgkmcnt(15 - need + issued)
constexpr int need0(int i) { return cmax(rd_of_a(i / 8), rd_of_b(i % 8)); }
constexpr int lgk0(int i) { return 15 - need0(i) + (i / 4 + 1); }

// acc (+)= x . y^T as inline asm with the accumulator an AGPR operand (FIRST: C = 0)
template <bool FIRST>
__device__ __forceinline__ void mfma_acc(f32x4_t& c, const bf16x8_t& x, const bf16x8_t& y) {
  if constexpr (FIRST)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(y), "v"(x));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(y), "v"(x));
}

// Tile order: t (consecutive on one XCD after xcd_remap) walks column-major blocks of `group`
// tile rows, so the ~32 workgroups an XCD runs at once cover a group x (32 / group) block and
// share both operand panels in that XCD's L2 (row-major order: 1 A panel + 32 B panels per
// K-tile step, most of them from beyond the L2).
__device__ __forceinline__ void tile_of(int t, int tiles_m, int tiles_n, int group, int& tm, int& tn) {
  if (group <= 1) {
    tm = t / tiles_n;
    tn = t % tiles_n;
    return;
  }
  const int per = group * tiles_n;
  const int g0 = (t / per) * group;
  const int gm = min(tiles_m - g0, group);
  const int r = t - (t / per) * per;
  tm = g0 + r % gm;
  tn = r / gm;
}

// SCHED 3: the production one-tile-per-workgroup loop (hand-ordered inline asm); SCHED 0: a
// two-barrier schedule left to the compiler, kept as the A/B oracle of the hand ordering (and the
// form of K = 64, a single K-tile)
template <int EK, int SCHED, int AOP = 0>
__global__ __launch_bounds__(T, 1) void gemm4w_kernel(const bf16_t* __restrict__ A, long long lda,
                                                     const bf16_t* __restrict__ B, long long ldb, EpiParams E, int M,
                                                     int N, int K, int tiles_m, int tiles_n, int group, ConvA ca) {
  static_assert(AOP == 0 || SCHED == 3, "the convolution operand rides the hand-ordered loop");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int nblk = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nblk);
  int tm_, tn_;
  tile_of(t, tiles_m, tiles_n, group, tm_, tn_);
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ktiles = K / 64;

  LoadK la, lb;
  LoadConv lc;
  if constexpr (AOP == 1) lc.init(A, ca, M, m0, tid);
  else la.init(A, lda, M, m0, tid);
  lb.init(B, ldb, N, n0, tid);
  // AOP = 1: the A operand's DMA cursor (K-tile whose A pieces go out next): tap index, channel
  // offset, and the tap's scalar byte offset (r W + s) C + c0 (2 bytes per element)
  int c_c0 = 0, c_r = 0, c_s = 0;
  // (tap 0 in the operand's own order: the reversed walk starts at its last tap)
  int c_atap = ca.flip ? ca.R * ca.S - 1 : 0;
  int c_soff = ca.flip ? ((ca.R - 1) * ca.W + ca.S - 1) * ca.C * 2 : 0;
  auto c_advance = [&]() {
    c_c0 += 64;
    if (c_c0 == ca.C) {
      c_c0 = 0;
      if (++c_s == ca.S) {
        c_s = 0;
        ++c_r;
      }
    }
    const int ra = ca.flip ? ca.R - 1 - c_r : c_r, sa = ca.flip ? ca.S - 1 - c_s : c_s;
    c_atap = ra * ca.S + sa;
    c_soff = ((ra * ca.W + sa) * ca.C + c_c0) * 2;
  };

  // per-lane fragment offsets for K-step ks: row i16, chunk 4 ks + g, XOR (i16 >> 1) & 7
  const int i16 = lane & 15, g = lane >> 4;
  const int lk0 = i16 * 128 + (((g) ^ ((i16 >> 1) & 7)) << 4);
  const int lk1 = i16 * 128 + (((4 | g) ^ ((i16 >> 1) & 7)) << 4);
  const int aoff = wm * 16384, boff = OPB + wn * 16384;

  // accumulators zeroed in AGPRs up front: the empty "+a" statements pin them there before any
  // DMA or MFMA asm (all volatile, so the zero writes are far ahead of the first MFMA that reads
  // them as C); one loop body for every K-tile (a peeled first K-tile with C = 0 made hipcc
  // place the tiles differently in the two copies and shuffle them with v_accvgpr_mov between)
  f32x4_t acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+a"(acc[a][b]));
    }
  bf16x8_t fa[2][8], fb[2][8];

  auto stage = [&](int kt) { return smem + (kt & 1) * STAGE; };
  auto read = [&](const char* st, int lk, bf16x8_t (&xa)[8], bf16x8_t (&xb)[8]) {
    // order of first use in the a-major MFMA sweep: a0, b0..b7, a1..a7
    xa[0] = rd(st + aoff + lk);
#pragma unroll
    for (int b = 0; b < 8; ++b) xb[b] = rd(st + boff + b * 2048 + lk);
#pragma unroll
    for (int a = 1; a < 8; ++a) xa[a] = rd(st + aoff + a * 2048 + lk);
  };
  // MFMAs as inline asm with the accumulator an "a" operand: hipcc allocates the 64 tiles in
  // AGPRs and leaves them there (with the builtin it re-homed accumulators between the VGPR and
  // AGPR halves every K-tile: 368 v_accvgpr_* per 128 MFMAs). FIRST: C = 0 (no zero-fill writes
  // into AGPRs, whose VALU-write -> MFMA-read wait states hipcc would not pad inside asm).
  auto mma = [&](const bf16x8_t (&xa)[8], const bf16x8_t (&xb)[8], int a0, int a1, auto first) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = a0; a < a1; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if constexpr (decltype(first)::value)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[a][b]) : "v"(xb[b]), "v"(xa[a]));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[a][b]) : "v"(xb[b]), "v"(xa[a]));
      }
    __builtin_amdgcn_s_setprio(0);
  };
  using F = std::false_type;
  using Tr = std::true_type;

  if constexpr (SCHED == 0) {
  // prologue: K-tiles 0 and 1, wait for 0, read its K-step 0
  if (ktiles > 0) {
    la.issue<0, 8>(stage(0), 0, wave);
    lb.issue<0, 8>(stage(0) + OPB, 0, wave);
    if (ktiles > 1) {
      la.issue<0, 8>(stage(1), 1, wave);
      lb.issue<0, 8>(stage(1) + OPB, 1, wave);
      wait_vm<16>();
    } else {
      wait_vm<0>();
    }
    bar();
    read(stage(0), lk0, fa[0], fb[0]);
  }
  auto ktile = [&](int kt, auto first) {
    const bool has1 = kt + 1 < ktiles, has2 = kt + 2 < ktiles;
    char* cs = stage(kt);
    // phase 0: K-step 0 MFMAs, K-step 1 fragments
    read(cs, lk1, fa[1], fb[1]);
    mma(fa[0], fb[0], 0, 8, first);
    wait_lgkm0();
    bar();
    // phase 1a: DMA of K-tile kt + 2 into this stage
    if (has2) {
      la.issue<0, 8>(cs, kt + 2, wave);
      lb.issue<0, 8>(cs + OPB, kt + 2, wave);
    }
    mma(fa[1], fb[1], 0, 4, F{});
    if (has1) {
      if (has2) wait_vm<16>(); else wait_vm<0>();
    }
    bar();
    // phase 1b: K-tile kt + 1's K-step 0 fragments
    if (has1) read(stage(kt + 1), lk0, fa[0], fb[0]);
    mma(fa[1], fb[1], 4, 8, F{});
  };
  for (int kt = 0; kt < ktiles; ++kt) ktile(kt, F{});
  } else {
  // hand-ordered: the whole main loop as inline asm in a fixed issue order (hipcc grouped all 16
  // fragment reads and all 16 DMA pieces of a phase in front of its MFMAs; with one wave per
  // SIMD nothing else fills the MFMA pipe while they issue). LDS reads and DMA are counted by
  // hand (hipcc does not count asm); the phases are described at the SCHED 3 loop below.
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)smem));
  uint32_t va[2][2], vb[2][2];  // [stage][K-step] fragment base addresses (block offsets immediate)
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    va[st][0] = sb + st * STAGE + wm * 16384 + lk0;
    va[st][1] = sb + st * STAGE + wm * 16384 + lk1;
    vb[st][0] = sb + st * STAGE + OPB + wn * 16384 + lk0;
    vb[st][1] = sb + st * STAGE + OPB + wn * 16384 + lk1;
  }
  const uint32_t ldsw = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sb + wave * 1024)));
  auto rd1 = [&](auto R, uint32_t a_base, uint32_t b_base, bf16x8_t (&xa)[8], bf16x8_t (&xb)[8]) {
    constexpr int r = decltype(R)::value;
    if constexpr (rd_is_a(r))
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(xa[rd_blk(r)]) : "v"(a_base), "i"(rd_blk(r) * 2048));
    else
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(xb[rd_blk(r)]) : "v"(b_base), "i"(rd_blk(r) * 2048));
  };
  // DMA piece q (0..7 A, 8..15 B) of K-tile kt into stage st, M0 = its LDS base (chained: every
  // piece sets M0 for its successor; the issue order is stage st 0..15, stage st ^ 1 0..15, ...)
  auto m0_of = [&](int q, int st) {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<int>(ldsw + st * STAGE + (q < 8 ? 0 : OPB) + (q & 7) * 4096)));
  };
  auto dma1 = [&](auto Q, int st, int kt) {
    constexpr int q = decltype(Q)::value;
    if constexpr (AOP == 1 && q < 8) {
      dma_chain(lc.off(q, c_atap), lc.srd, c_soff, m0_of(q + 1, st));
      if constexpr (q == 7) c_advance();
    } else {
      const LoadK& L = q < 8 ? la : lb;
      dma_chain(L.voff[q & 7], L.srd, kt * 128, q < 15 ? m0_of(q + 1, st) : m0_of(0, st ^ 1));
    }
  };
  auto mfma1 = [&](int a, int b, const bf16x8_t& x, const bf16x8_t& y, auto first) {
    mfma_acc<decltype(first)::value>(acc[a][b], x, y);
  };
  // prologue: K-tiles 0 and 1, wait for 0, K-step-0 fragments of K-tile 0 (SCHED 3: K-tile kt
  // in stage (kt + ktiles) & 1, so that the last two K-tiles always sit in stages 0, 1)
  const int st0 = ktiles & 1;
  m0_init(m0_of(0, st0));
  static_for<16>([&](auto Q) { dma1(Q, st0, 0); });
  if (ktiles > 1) {
    static_for<16>([&](auto Q) { dma1(Q, st0 ^ 1, 1); });
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  {
  // SCHED 3: the stage of K-tile kt is released in two halves, so the DMA of K-tile kt + 2 starts
  // 32 MFMAs earlier than in the two-barrier loop (every piece gets >= 132 MFMAs, ~2100 cycles, to land
  // instead of >= 99) at the price of a third barrier; the stage index is compile-time (the
  // K-tiles go in pairs), so no per-K-tile selects of the fragment / DMA bases:
  //   A  (MFMAs  0-31, K-step 0): the 8 A fragments of K-step 1, one per 3 MFMAs;
  //      lgkmcnt(0), barrier: every wave is done with this stage's A half
  //   B  (MFMAs 32-63, K-step 0): the 8 B fragments of K-step 1 | DMA of K-tile kt + 2, A half;
  //      lgkmcnt(0), barrier: ... and with its B half
  //   C  (MFMAs 64-95, K-step 1): DMA of K-tile kt + 2, B half;
  //      vmcnt(16 pieces of kt + 2), barrier: K-tile kt + 1 has landed for every wave
  //   D  (MFMAs 96-127, K-step 1): the 16 K-step-0 fragments of K-tile kt + 1, one per 2 MFMAs.
  auto rda = [&](auto Bk, uint32_t base, bf16x8_t (&xa)[8]) {
    constexpr int b = decltype(Bk)::value;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(xa[b]) : "v"(base), "i"(b * 2048));
  };
  auto ktile3 = [&](int kt, auto stc, auto has2c) {
    constexpr int st = decltype(stc)::value;
    constexpr bool has2 = decltype(has2c)::value;
    static_for<32>([&](auto I) {  // A
      constexpr int i = decltype(I)::value, a = i / 8, b = i % 8;
      if constexpr (i % 3 == 0 && i / 3 < 8) rda(std::integral_constant<int, i / 3>{}, va[st][1], fa[1]);
      constexpr int issued = (i / 3 + 1) < 8 ? (i / 3 + 1) : 8;
      constexpr int pi = i == 0 ? 0 : i - 1;
      constexpr int issued_p = (pi / 3 + 1) < 8 ? (pi / 3 + 1) : 8;
      if constexpr (i == 0 || 15 - need0(i) + issued != 15 - need0(pi) + issued_p)
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(15 - need0(i) + issued) : "memory");
      mfma1(a, b, fa[0][a], fb[0][b], F{});
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    static_for<32>([&](auto I) {  // B
      constexpr int i = decltype(I)::value;
      if constexpr (i % 3 == 0 && i / 3 < 8) rda(std::integral_constant<int, i / 3>{}, vb[st][1], fb[1]);
      if constexpr (i % 4 == 2)
        if constexpr (has2) dma1(std::integral_constant<int, i / 4>{}, st, kt + 2);
      mfma1(4 + i / 8, i % 8, fa[0][4 + i / 8], fb[0][i % 8], F{});
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    static_for<32>([&](auto I) {  // C
      constexpr int i = decltype(I)::value;
      if constexpr (i % 4 == 0)
        if constexpr (has2) dma1(std::integral_constant<int, 8 + i / 4>{}, st, kt + 2);
      mfma1(i / 8, i % 8, fa[1][i / 8], fb[1][i % 8], F{});
    });
    if constexpr (has2) {
      asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    static_for<32>([&](auto I) {  // D
      constexpr int i = decltype(I)::value;
      if constexpr (i % 2 == 0) rd1(std::integral_constant<int, i / 2>{}, va[st ^ 1][0], vb[st ^ 1][0], fa[0], fb[0]);
      mfma1(4 + i / 8, i % 8, fa[1][4 + i / 8], fb[1][i % 8], F{});
    });
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // (ktiles >= 2, host-checked.) Straight-line code around the loops: MFMA sequences inside
  // if / else copies made hipcc allocate the accumulators per copy and spill (measured: 540
  // scratch accesses); an odd K-tile count starts in stage 1 instead
  if (st0) static_for<16>([&](auto R) { rd1(R, va[1][0], vb[1][0], fa[0], fb[0]); });
  else static_for<16>([&](auto R) { rd1(R, va[0][0], vb[0][0], fa[0], fb[0]); });
  int kt = 0;
  for (int i = 0; i < st0; ++i) {
    ktile3(0, S1{}, Tr{});
    kt = 1;
  }
  for (; kt < ktiles - 2; kt += 2) {
    ktile3(kt, S0{}, Tr{});
    ktile3(kt + 1, S1{}, Tr{});
  }
  ktile3(ktiles - 2, S0{}, F{});
  ktile3(ktiles - 1, S1{}, F{});
  }
  }
  // the last MFMAs' results -> the epilogue's v_accvgpr_read: XDL write -> read wait states
  // (hipcc pads nothing after asm); the empty "+a" statements order every read after the pad
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) asm volatile("" : "+a"(acc[a][b]));

  const float alpha = epi_alpha(E);
  if (m0 + BM <= M && n0 + BN <= N) epilogue<EK, false>(acc, E, m0, n0, M, N, alpha, lane, wm, wn);
  else epilogue<EK, true>(acc, E, m0, n0, M, N, alpha, lane, wm, wn);
}

// ============================================================================================
// gemm4p: the persistent 4-wave 256 x 256 kernel (TTD_G4_SCHED=30, opt-in) on the round-5
// two-barrier main loop (16x16x32 MFMAs, LDS-DMA staging; 61 % MFMA busy at 8192^3 with 13.8 %
// of wave cycles waiting, profiles/r5_gemm4_pmc_8192.txt). One workgroup per CU walks its
// XCD's tile range (xcd_remap order, column-major blocks of `group` tile rows): as soon as a
// tile's last K-tile is consumed, the next tile's first two K-tiles are DMA'd into the idle
// stages and only then does the register epilogue run, so the operand latency of tile i + 1
// hides under tile i's epilogue and its stores drain under tile i + 1's MFMAs. The first
// K-step of every tile runs its MFMAs with C = 0 (no accumulator zero-fill).
// Epilogues that load (dGELU residual, accumulate) issue the next tile's DMA after the
// epilogue instead: hipcc counts only its own loads, so an older DMA in the queue would make
// every epilogue load wait for it.

__device__ __forceinline__ void dma_piece(uint32_t m0v, uint32_t voff, const ttd_i32x4_t& srd, int soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(m0v), "v"(voff), "s"(srd), "s"(soff)
      : "memory");
}
template <int OFF>
__device__ __forceinline__ void ds_rd(bf16x8_t& d, uint32_t base) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"(OFF));
}

template <int EK>
__global__ __launch_bounds__(T, 1) void gemm4p_kernel(const bf16_t* __restrict__ A, long long lda,
                                                     const bf16_t* __restrict__ B, long long ldb, EpiParams E, int M,
                                                     int N, int K, int tiles_m, int tiles_n, int group,
                                                     int stagger, int* tq) {
  // (+16 B: the claimed next tile, broadcast to the workgroup; one __shared__ object)
  __shared__ __attribute__((aligned(16))) char smem[SMEM + 16];
  constexpr bool EPI_LOADS = (EK & (kEkDGelu | kEkBeta)) != 0;
  constexpr int EPI_ST = 32 * (((EK & kEkAux) != 0) ? 2 : 1);  // stores per lane, unchecked epilogue
  const int nblk = tiles_m * tiles_n;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ktiles = K / 64;
  // XCD x = blockIdx.x & 7 owns tiles [xbase, xbase + xcnt) of the order; its G8 workgroups
  // take idx = blockIdx.x >> 3, + G8, ... (the host launches a multiple of 8 workgroups)
  const int xcd = blockIdx.x & 7, G8 = gridDim.x >> 3;
  const int xq = nblk >> 3, xr = nblk & 7;
  const int xbase = xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq;
  const int xcnt = xq + (xcd < xr ? 1 : 0);
  int idx = blockIdx.x >> 3;
  if (idx >= xcnt) return;

  const int i16 = lane & 15, g = lane >> 4;
  const int lk0 = i16 * 128 + (((g) ^ ((i16 >> 1) & 7)) << 4);
  const int lk1 = i16 * 128 + (((4 | g) ^ ((i16 >> 1) & 7)) << 4);
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)smem));
  uint32_t va[2][2], vb[2][2];  // [stage][K-step] fragment bases (block offsets immediate)
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    va[st][0] = sb + st * STAGE + wm * 16384 + lk0;
    va[st][1] = sb + st * STAGE + wm * 16384 + lk1;
    vb[st][0] = sb + st * STAGE + OPB + wn * 16384 + lk0;
    vb[st][1] = sb + st * STAGE + OPB + wn * 16384 + lk1;
  }
  const uint32_t ldsw = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sb + wave * 1024)));
  LoadK la, lb;
  f32x4_t acc[8][8];
  bf16x8_t fa[2][8], fb[2][8];

  auto rd1 = [&](auto R, uint32_t a_base, uint32_t b_base, bf16x8_t (&xa)[8], bf16x8_t (&xb)[8]) {
    constexpr int r = decltype(R)::value;
    if constexpr (rd_is_a(r)) ds_rd<rd_blk(r) * 2048>(xa[rd_blk(r)], a_base);
    else ds_rd<rd_blk(r) * 2048>(xb[rd_blk(r)], b_base);
  };
  // LDS base of piece q (0..7 A, 8..15 B) in stage st; pieces are issued in the order
  // (stage st: 0..15), (stage st ^ 1: 0..15), ... so each sets M0 for its successor
  auto m0_of = [&](int q, int st) { return ldsw + st * STAGE + (q < 8 ? 0 : OPB) + (q & 7) * 4096; };
  auto dma1 = [&](auto Q, int st, int kt) {  // piece q of K-tile kt into stage st (M0 = its base)
    constexpr int q = decltype(Q)::value;
    const LoadK& L = q < 8 ? la : lb;
    const uint32_t nxt = q < 15 ? m0_of(q + 1, st) : m0_of(0, st ^ 1);
    dma_chain(L.voff[q & 7], L.srd, kt * 128, static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(nxt))));
  };
  auto mfma1 = [&](int a, int b, const bf16x8_t& x, const bf16x8_t& y, auto first) {
    mfma_acc<decltype(first)::value>(acc[a][b], x, y);
  };
  auto coords = [&](int i, int& m0, int& n0) {
    int tm, tn;
    tile_of(xbase + i, tiles_m, tiles_n, group, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  auto prologue = [&](int m0, int n0) {  // K-tiles 0 and 1 of tile (m0, n0) into stages 0 and 1
    la.init(A, lda, M, m0, tid);
    lb.init(B, ldb, N, n0, tid);
    m0_init(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(m0_of(0, 0)))));
    static_for<16>([&](auto Q) { dma1(Q, 0, 0); });
    if (ktiles > 1) static_for<16>([&](auto Q) { dma1(Q, 1, 1); });
  };
  // one K-tile of the two-barrier schedule (phase 0: K-step 0 | K-step-1 fragment reads; 1a: DMA
  // of K-tile kt + 2, A half; 1b: B half + K-step-0 reads of kt + 1); FIRST: phase 0 with C = 0; HAS2:
  // K-tile kt + 2 exists (compile-time: the steady-state loop body has no branch around its 16
  // DMA pieces — as run-time tests they were 16 scalar branches per K-tile)
  auto ktile = [&](int kt, auto first, auto has2c) {
    constexpr bool has2 = decltype(has2c)::value;
    const int st = kt & 1;
    static_for<64>([&](auto I) {
      constexpr int i = decltype(I)::value, a = i / 8, b = i % 8;
      if constexpr (i % 4 == 0) rd1(std::integral_constant<int, i / 4>{}, va[st][1], vb[st][1], fa[1], fb[1]);
      if constexpr (i == 0 || need0(i) > need0(i - 1 < 0 ? 0 : i - 1))
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(lgk0(i)) : "memory");
      mfma1(a, b, fa[0][a], fb[0][b], first);
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    static_for<32>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i % 4 == 0)
        if constexpr (has2) dma1(std::integral_constant<int, i / 4>{}, st, kt + 2);
      mfma1(i / 8, i % 8, fa[1][i / 8], fb[1][i % 8], std::false_type{});
    });
    if constexpr (has2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    static_for<32>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i % 4 == 1)
        if constexpr (has2) dma1(std::integral_constant<int, 8 + i / 4>{}, st, kt + 2);
      if constexpr (i % 2 == 0) rd1(std::integral_constant<int, i / 2>{}, va[st ^ 1][0], vb[st ^ 1][0], fa[0], fb[0]);
      mfma1(4 + i / 8, i % 8, fa[1][4 + i / 8], fb[1][i % 8], std::false_type{});
    });
  };

  int m0, n0;
  coords(idx, m0, n0);
  prologue(m0, n0);
  // Stagger: every workgroup walks identical tiles, so without it all 256 CUs reach their
  // epilogues together and the chip's HBM write bandwidth is shared by every CU's 128-256 KB of
  // stores at once (in-kernel stamps: a bias epilogue took 23k cycles per tile, half the main
  // loop, profiles/r5_gemm4p_stamps.txt). Workgroup i starts (i / 8) % 4 quarters of `stagger`
  // sleep units later (64 cycles each), so at any time about a quarter of the CUs store.
  if (stagger > 0) {
    const int q = (blockIdx.x >> 3) & 3;
    for (int k = 0; k < q * stagger; ++k) __builtin_amdgcn_s_sleep(127);
  }
  int prev = 0;  // what the previous tile left in the VMEM queue after this tile's DMA: 0 none,
                 // 1 an unchecked epilogue's EPI_ST stores, 2 a data-dependent count
  const float alpha = epi_alpha(E);
  for (;;) {
    // Tile queue (tq: 8 per-XCD counters + a finished-workgroup count): after its static first
    // tile a workgroup claims the next unclaimed tile of its XCD's range. In the two-stream
    // BERT step the side stream's weight gradients hold up to 192 CUs for hundreds of us, so
    // some workgroups of a persistent grid get a CU late; with a static share each would finish
    // its whole share late and hold the launch. The claim's round trip hides under the loop.
    int claim = 0;
    if (tq && tid == 0) claim = atomicAdd(tq + xcd, 1);
    // K-tile 0 has landed: the queue holds (K-tile 0, K-tile 1 [16 each], previous stores)
    if (prev == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (ktiles > 1) {
      if (prev == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 + EPI_ST > 63 ? 63 : 16 + EPI_ST) : "memory");
      else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      if (prev == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EPI_ST > 63 ? 63 : EPI_ST) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_barrier" ::: "memory");
    static_for<16>([&](auto R) { rd1(R, va[0][0], vb[0][0], fa[0], fb[0]); });
    if (ktiles >= 3) {
      ktile(0, std::true_type{}, std::true_type{});
      for (int kt = 1; kt < ktiles - 2; ++kt) ktile(kt, std::false_type{}, std::true_type{});
      ktile(ktiles - 2, std::false_type{}, std::false_type{});
      ktile(ktiles - 1, std::false_type{}, std::false_type{});
    } else {
      ktile(0, std::true_type{}, std::false_type{});
      if (ktiles == 2) ktile(1, std::false_type{}, std::false_type{});
    }
    if (tq && tid == 0) *reinterpret_cast<int*>(smem + SMEM) = claim;
    // every wave past its last LDS read before the stages are refilled
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int nidx = tq ? G8 + __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(smem + SMEM)) : idx + G8;
    const bool more = nidx < xcnt;
    int nm0 = 0, nn0 = 0;
    if (more) coords(nidx, nm0, nn0);
    if (!EPI_LOADS && more) prologue(nm0, nn0);
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) asm volatile("" : "+a"(acc[a][b]));
    const bool whole = m0 + BM <= M && n0 + BN <= N;
    if (whole) epilogue<EK, false>(acc, E, m0, n0, M, N, alpha, lane, wm, wn);
    else epilogue<EK, true>(acc, E, m0, n0, M, N, alpha, lane, wm, wn);
    if (!more) break;
    if (EPI_LOADS) {
      prologue(nm0, nn0);
      prev = 0;
    } else {
      prev = whole ? 1 : 2;
    }
    m0 = nm0;
    n0 = nn0;
    idx = nidx;
  }
  if (tq && tid == 0) {
    // every workgroup's last claim precedes its arrival here: the last to arrive resets the
    // queue for the next launch on this stream (graph replays included)
    if (atomicAdd(tq + 8, 1) == static_cast<int>(gridDim.x) - 1) {
#pragma unroll
      for (int i = 0; i < 9; ++i) tq[i] = 0;
    }
  }
}


// ------------------------------------------------------------------------------ fp8 forward
// fp8 convolution / GEMM on the block-scaled MFMA: C[M][N] (bf16) = sa * sb * A8 . B8^T with A8
// e4m3 K-major — the dense [M][K] rows of a unit-stride 1x1 conv input or the implicit-GEMM
// gather of x [N][H][W][C] (C % 128 == 0: a 128-channel K-tile inside one filter tap) — and B8 the
// [N][K] e4m3 filter (precision="fp8" forward convs; the 8-wave conv_fwd_fp8 kernel is the
// fallback). The 4-wave transposed-read kernel's fp8 form (gemm4t.hip gemm4t8_kernel) with
// K-major operands:
//  * the K-tile images are this file's [256 rows][128 B] (128 k per row), chunk c of row r at
//    c ^ ((r >> 1) & 7): the loaders are the bf16 ones with byte offsets;
//  * a lane's 32 x 32 x 64 fragment (row l & 31, k 32 (l >> 5) .. +31 of the K-step) is two
//    ds_read_b128 of consecutive chunks (16 consecutive rows per 16-lane group: all 64 banks);
//  * two K-steps of 64 k per K-tile, 4 A + 4 B fragments per K-step (64 VGPRs, two sets), 16
//    MFMAs of 32 passes into 4 x 4 accumulators of 16 AGPRs; the phase schedule and DMA order of
//    gemm4t8_kernel (one DMA piece per MFMA in the second K-step, one barrier after each K-step);
//  * epilogue: bf16 store (4 columns per lane and accumulator quarter) and, with `stat`, the BN
//    partial sums (sum, sum of squares of the stored values) per 128 rows: [2 ceil(M/256)][2][N].
// AOP: 0 dense A, 1 conv gather. B_E5M2: the A operand in OCP e5m2 (data gradients).
typedef __attribute__((ext_vector_type(8))) int ttd_i32x8_t;
typedef __attribute__((ext_vector_type(16))) float ttd_f32x16_t;
typedef __attribute__((address_space(3))) bf16x8_t lds_b8x8_t;  // a 16-B LDS read (32-bit LDS address)

template <bool FIRST, bool E5M2>
__device__ __forceinline__ void mfma8k(ttd_f32x16_t& c, const ttd_i32x8_t& a, const ttd_i32x8_t& b, int one) {
  // src0 = the B fragment (filter, e4m3), src1 = the A fragment (blgp 1 when e5m2); the leading
  // s_nop 1: `one` may be a VALU write right before the asm
  if constexpr (FIRST && E5M2)
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] blgp:1"
                 : "=a"(c) : "v"(b), "v"(a), "v"(one) : "memory");
  else if constexpr (FIRST)
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0]"
                 : "=a"(c) : "v"(b), "v"(a), "v"(one) : "memory");
  else if constexpr (E5M2)
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] blgp:1"
                 : "+a"(c) : "v"(b), "v"(a), "v"(one) : "memory");
  else
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
                 : "+a"(c) : "v"(b), "v"(a), "v"(one) : "memory");
}

struct K8Args {
  const uint8_t* A;
  long long lda;  // AOP 0
  const uint8_t* B;
  long long ldb;
  bf16_t* out;
  long long ldo;
  float* stat;  // nullptr: no statistics
  const bf16_t* by;       // FEED: the feeding unit's conv output y [M][ldo]
  const uint8_t* bmask;   // FEED: its ReLU bits (bit n of byte (m ldo + n) / 8)
  int beta;               // FEED: g = (dx + the stored gradient) * bits (a shortcut-gradient accumulate)
  const float* sa;
  const float* sb;
  int M, N, K, tiles_m, tiles_n, group;
};

// FEED (data gradients): g = dx * ReLU bits of the feeding conv+BN unit is stored, the statistics
// are (sum g, sum g y) — the bf16 feeding-BN epilogue of this file
template <int AOP, bool E5M2, bool FEED = false>
__global__ __launch_bounds__(T, 1) void gemm4k8_kernel(K8Args P, ConvA ca) {
  constexpr int NA = 4, NB = 4, NF = 8, NMF = 16, PA = 8, NQ = 16, NR = 2 * NF, H0 = NMF, H1 = NMF / 2;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  const int M = P.M, N = P.N;
  const int nblk = P.tiles_m * P.tiles_n;
  const int t = xcd_remap(blockIdx.x, nblk);
  int tm_, tn_;
  tile_of(t, P.tiles_m, P.tiles_n, P.group, tm_, tn_);
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = P.K / 128;

  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)smem));
  // fragment read base: row (l & 31) of the wave's block 0, chunk ((l >> 5) << 1) ^ ((l >> 1) & 7);
  // K-step s, read q: chunk ^ (4 s | q) (immediate XOR), block j: + 32 j rows
  const uint32_t L = static_cast<uint32_t>(((lane >> 5) << 1) ^ ((lane >> 1) & 7));
  const uint32_t rA = sb + static_cast<uint32_t>((wm * 128 + (lane & 31)) * 128) + (L << 4);
  const uint32_t rB = sb + OPB + static_cast<uint32_t>((wn * 128 + (lane & 31)) * 128) + (L << 4);
  const uint32_t ldsw = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sb + wave * 1024)));

  // loaders: piece i of thread tid = image row 32 i + tid / 8, physical chunk tid % 8 = logical
  // chunk (tid & 7) ^ ((tid >> 4) & 7); rows past the end clamped (A dense, B) or zero (A conv)
  const int chunk = (tid & 7) ^ ((tid >> 4) & 7);
  ttd_i32x4_t srd_a, srd_b;
  uint32_t voa[8], vob[8], vmask[8];
  srd_b = make_srd(P.B, static_cast<uint32_t>(static_cast<long long>(N) * P.ldb));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = min(n0 + i * 32 + (tid >> 3), N - 1);
    vob[i] = static_cast<uint32_t>(static_cast<long long>(r) * P.ldb + chunk * 16);
  }
  long long shift = 0;
  if constexpr (AOP == 0) {
    srd_a = make_srd(P.A, static_cast<uint32_t>(static_cast<long long>(M) * P.lda));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = min(m0 + i * 32 + (tid >> 3), M - 1);
      voa[i] = static_cast<uint32_t>(static_cast<long long>(r) * P.lda + chunk * 16);
      vmask[i] = 0;
    }
  } else {
    shift = (static_cast<long long>(ca.ph) * ca.W + ca.pw) * ca.C;
    srd_a = make_srd(P.A - shift, static_cast<uint32_t>(ca.x_bytes + shift));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + i * 32 + (tid >> 3);
      const int mm = m < M ? m : 0;
      const int n = mm / ca.PQ, rem = mm - n * ca.PQ;
      const int p = rem / ca.Q, q = rem - p * ca.Q;
      const int h0 = p * ca.sh - ca.ph, w0 = q * ca.sw - ca.pw;
      voa[i] = static_cast<uint32_t>(((static_cast<long long>(n) * ca.H + h0) * ca.W + w0) * ca.C + shift + chunk * 16);
      uint32_t mk = 0;
      for (int r = 0; r < ca.R; ++r)
        for (int s2 = 0; s2 < ca.S; ++s2)
          if (m < M && static_cast<unsigned>(h0 + r) < static_cast<unsigned>(ca.H) &&
              static_cast<unsigned>(w0 + s2) < static_cast<unsigned>(ca.W))
            mk |= 1u << (r * ca.S + s2);
      vmask[i] = mk;
    }
  }
  // conv A cursor (the K-tile whose A pieces go out next): tap, channel offset, scalar bytes
  // (flip, data gradients: the taps in the filter's reversed order, starting at the last)
  int c_c0 = 0, c_r = 0, c_s = 0;
  int c_tap = ca.flip ? ca.R * ca.S - 1 : 0;
  int c_soff = ca.flip ? ((ca.R - 1) * ca.W + ca.S - 1) * ca.C : 0;
  auto c_advance = [&]() {
    c_c0 += 128;
    if (c_c0 == ca.C) {
      c_c0 = 0;
      if (++c_s == ca.S) {
        c_s = 0;
        ++c_r;
      }
    }
    const int ra = ca.flip ? ca.R - 1 - c_r : c_r, sa2 = ca.flip ? ca.S - 1 - c_s : c_s;
    c_tap = ra * ca.S + sa2;
    c_soff = (ra * ca.W + sa2) * ca.C + c_c0;
  };
  int one = 127;
  asm volatile("" : "+v"(one));

  ttd_f32x16_t acc[NA][NB];
  bf16x8_t fr[2][NF][2];  // [set][fragment: 0..NA-1 A, NA.. B][read q]

  auto rd1 = [&](auto R, auto S, int st, auto SET) {
    constexpr int r = decltype(R)::value, s = decltype(S)::value, set = decltype(SET)::value;
    constexpr int fi = r / 2, q = r % 2;
    constexpr bool isa = fi == 0 || fi > NB;
    constexpr int blk = fi == 0 ? 0 : (fi <= NB ? fi - 1 : fi - NB);
    const uint32_t base = (isa ? rA : rB) + st * STAGE;
    const uint32_t addr = (base ^ static_cast<uint32_t>((4 * s | q) << 4)) + blk * 4096;
    fr[set][isa ? blk : NA + blk][q] = *reinterpret_cast<const lds_b8x8_t*>(static_cast<uintptr_t>(addr));
  };
  auto frag = [&](int set, int slot) {
    return __builtin_bit_cast(ttd_i32x8_t, __builtin_shufflevector(fr[set][slot][0], fr[set][slot][1], 0, 1, 2, 3, 4,
                                                                     5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
  };
  auto m0_of = [&](int qq, int st) {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
        static_cast<int>(ldsw + st * STAGE + (qq < PA ? qq * 4096 : OPB + (qq - PA) * 4096))));
  };
  auto dma1 = [&](auto Q, int st, int kt) {
    constexpr int qq = decltype(Q)::value;
    const uint32_t next = qq < NQ - 1 ? m0_of(qq + 1, st) : m0_of(0, st ^ 1);
    if constexpr (qq < PA) {
      if constexpr (AOP == 0) dma_chain(voa[qq], srd_a, kt * 128, next);
      else dma_chain((vmask[qq] >> c_tap) & 1u ? voa[qq] : kOob, srd_a, c_soff, next);
      if constexpr (AOP == 1 && qq == PA - 1) c_advance();
    } else {
      dma_chain(vob[qq - PA], srd_b, kt * 128, next);
    }
  };

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
      mfma8k<FIRST, E5M2>(acc[i / NB][i % NB], frag(0, i / NB), frag(0, NA + i % NB), one);
    });
    wait_lgkm0();
    asm volatile("s_barrier" ::: "memory");
    static_for<H1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (has2) dma1(std::integral_constant<int, i>{}, st, kt + 2);
      mfma8k<false, E5M2>(acc[i / NB][i % NB], frag(1, i / NB), frag(1, NA + i % NB), one);
    });
    if constexpr (has2) wait_vm<PA>();
    else wait_vm<0>();
    asm volatile("s_barrier" ::: "memory");
    static_for<H1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (has2) dma1(std::integral_constant<int, PA + i>{}, st, kt + 2);
      static_for<NR>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if constexpr (j * H1 / NR == i) rd1(J, std::integral_constant<int, 0>{}, st ^ 1, std::integral_constant<int, 0>{});
      });
      mfma8k<false, E5M2>(acc[NA / 2 + i / NB][i % NB], frag(1, NA / 2 + i / NB), frag(1, NA + i % NB), one);
    });
  };

  m0_init(m0_of(0, 0));
  static_for<NQ>([&](auto Q) { dma1(Q, 0, 0); });
  static_for<NQ>([&](auto Q) { dma1(Q, 1, 1); });
  wait_lgkm0();
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
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) asm volatile("" : "+a"(acc[a][b]));

  // epilogue: lane l, accumulator (a, b), quarter v4: row m0 + 128 wm + 32 a + (l & 31), columns
  // n0 + 128 wn + 32 b + 8 v4 + 4 (l >> 5) .. +3
  const float scale = P.sa[0] * P.sb[0];
  const bool stats = P.stat != nullptr;
  const int hi = lane >> 5;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float ssum[4][4], ssq[4][4];
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4)
#pragma unroll
      for (int j = 0; j < 4; ++j) ssum[v4][j] = ssq[v4][j] = 0.f;
    // FEED: this column block's y values and ReLU bytes for all 16 (a, v4) issued up front (16
    // loads in flight per lane instead of one exposed latency per store)
    uint2 fy[NA][4], fo[NA][4];
    uint32_t fb[NA][4];
    if constexpr (FEED) {
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const int m = m0 + wm * 128 + a * 32 + (lane & 31);
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4) {
          const int n = n0 + wn * 128 + b * 32 + 8 * v4 + 4 * hi;
          const long long o = static_cast<long long>(m) * P.ldo + n;
          const bool ok = m < M && n < N;
          fy[a][v4] = ok ? *reinterpret_cast<const uint2*>(P.by + o) : make_uint2(0, 0);
          fb[a][v4] = ok ? static_cast<uint32_t>(P.bmask[o >> 3]) : 0u;
          fo[a][v4] = ok && P.beta ? *reinterpret_cast<const uint2*>(P.out + o) : make_uint2(0, 0);
        }
      }
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      asm volatile("" : "+a"(acc[a][b]));
      const int m = m0 + wm * 128 + a * 32 + (lane & 31);
      const bool mok = m < M;
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4) {
        const int n = n0 + wn * 128 + b * 32 + 8 * v4 + 4 * hi;
        float x[4] = {acc[a][b][4 * v4] * scale, acc[a][b][4 * v4 + 1] * scale, acc[a][b][4 * v4 + 2] * scale,
                      acc[a][b][4 * v4 + 3] * scale};
        const bool ok = mok && n < N;
        const long long o = static_cast<long long>(m) * P.ldo + n;
        float yv[4];
        if constexpr (FEED) {
          const uint32_t bits = fb[a][v4] >> (n & 7);
          const uint2 yw = fy[a][v4];
          yv[0] = bf2f(static_cast<bf16_t>(yw.x & 0xffff));
          yv[1] = bf2f(static_cast<bf16_t>(yw.x >> 16));
          yv[2] = bf2f(static_cast<bf16_t>(yw.y & 0xffff));
          yv[3] = bf2f(static_cast<bf16_t>(yw.y >> 16));
          const uint2 ow = fo[a][v4];  // (the bf16 path's rounding: bf16(dx) + old, then the mask)
          const float od[4] = {bf2f(static_cast<bf16_t>(ow.x & 0xffff)), bf2f(static_cast<bf16_t>(ow.x >> 16)),
                               bf2f(static_cast<bf16_t>(ow.y & 0xffff)), bf2f(static_cast<bf16_t>(ow.y >> 16))};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (P.beta) x[j] = bf2f(f2bf(x[j])) + od[j];
            x[j] = (bits >> j) & 1u ? x[j] : 0.f;
          }
        }
        const uint2 w = make_uint2(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]));
        if (ok) *reinterpret_cast<uint2*>(P.out + o) = w;
        if (stats && ok) {
          const float r[4] = {bf2f(static_cast<bf16_t>(w.x & 0xffff)), bf2f(static_cast<bf16_t>(w.x >> 16)),
                              bf2f(static_cast<bf16_t>(w.y & 0xffff)), bf2f(static_cast<bf16_t>(w.y >> 16))};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ssum[v4][j] += r[j];
            ssq[v4][j] += r[j] * (FEED ? yv[j] : r[j]);
          }
        }
      }
    }
    if (stats) {
      // the 32 lanes of a half-wave hold the same columns (rows l & 31): sum them; lane 31 / 63
      // writes this wave's 128-row partial row (m0 / 128 + wm)
      float* const st = P.stat + static_cast<long long>((m0 / 128) + wm) * 2 * N;
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // DPP row sums (lane 15 of each 16-lane row), then row_bcast:15 adds row 0's total into
          // row 1 (and row 2's into row 3): lanes 31 / 63 hold the half-wave totals
          float s = row_sum16(ssum[v4][j]), q2 = row_sum16(ssq[v4][j]);
          s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0x142, 0xa, 0xf, false));
          q2 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, q2), 0x142, 0xa, 0xf, false));
          const int n = n0 + wn * 128 + b * 32 + 8 * v4 + 4 * hi + j;
          if ((lane & 31) == 31 && n < N) {
            st[n] = s;
            st[N + n] = q2;
          }
        }
    }
  }
}

}  // namespace g4
}  // namespace
}  // namespace ttdk

// TTD_G4_SCHED: main-loop form. 3 (default) = one tile per workgroup, hand-ordered, the stage
// released in two halves (3 barriers per K-tile, every DMA piece >= 132 MFMAs to land): same box,
// interleaved, tools/g4_bench.py: 8192^3 1516 vs 1435 TF/s for the two-barrier round-5 loop
// (SCHED 2, removed: git history), hipBLASLt 1578; BERT qkv 1129 vs 1086, ffn2 1330 vs 1283,
// ffn1 dgrad 1322 vs 1297 TF/s;
// 30 = the persistent SCHED-2 kernel (gemm4p, next tile's DMA under this tile's epilogue);
// 0 = the compiler-scheduled one-tile loop (oracle). With the branch-free steady loop (same box,
// tools/g4_bench.py): 8192^3 1515 (2) vs 1301 (30) TF/s, hipBLASLt 1650; BERT-Large step
// 154.8 / 156.2 vs 158.7 ms. (Measured and removed, round 5: all 16 DMA pieces in phase 1a,
// one barrier per K-tile, a VGPR-staged 32x32x16 form, in-kernel phase stamps — git history.)
static int& g4_sched() {
  static int v = ttdk::getenv_int("TTD_G4_SCHED", 3);
  return v;
}
static int g4_cus() { return ttdk::big::device_cus(); }
// TTD_G4_STAGGER: stagger the persistent workgroups' tile phases (default off: +8 % on the
// GELU + aux epilogue, -10 % on the bias-only shapes, tools/g4_bench.py)
static int& g4_stagger() {
  static int v = ttdk::getenv_int("TTD_G4_STAGGER", 0);
  return v;
}
TTDK_EXPORT int ttdk_set_g4_stagger(int v) {
  const int old = g4_stagger();
  g4_stagger() = v;
  return old;
}

// TTD_G4_GROUP: tile rows per column-major tile block (1 = row-major order)
static int& g4_group() {
  static int v = ttdk::getenv_int("TTD_G4_GROUP", 8);
  return v;
}
TTDK_EXPORT int ttdk_set_g4_group(int v) {
  const int old = g4_group();
  g4_group() = v;
  return old;
}
TTDK_EXPORT int ttdk_set_g4_sched(int v) {
  const int old = g4_sched();
  g4_sched() = v;
  return old;
}

// Forward convolution y[M = N P Q][K] = conv(x[N][H][W][C], w[K][R][S][C]) on the 4-wave kernel
// (hand-ordered SCHED 3 loop), plain bf16 store (epi: out with ldo = K, optionally stat — nothing
// else). stat receives the BN partial sums (sum, sum of squares) of the stored output per 128
// rows: [2 ceil(M / 256)][2][K]. Unit-stride 1x1 convs read x as a dense [M][C] operand, the
// others through the implicit-GEMM gather (g4::LoadConv). Needs C % 64 == 0 (a K-tile inside one
// tap), R S C >= 128, no dilation. hipErrorInvalidValue: not taken (the caller keeps conv_fwd).
TTDK_EXPORT int ttdk_conv_fwd4w(const bf16_t* x, const bf16_t* w, const TtdkConv* g, const TtdkEpilogue* epi,
                                hipStream_t st) {
  using namespace ttdk;
  EpiParams pe = to_epi(epi);
  const int M = g->N * g->P * g->Q, N = g->K, K = g->R * g->S * g->C;
  const long long xb = static_cast<long long>(g->N) * g->H * g->W * g->C * 2;
  const long long shift = (static_cast<long long>(g->ph) * g->W + g->pw) * g->C * 2;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g->C % 64 || K < 128 || N % 8 || g->dh != 1 || g->dw != 1 || g->R * g->S > 32 || M < 1 || !al16(x) ||
      !al16(w) || !al16(pe.out) || xb + shift >= (1LL << 31) || (static_cast<long long>(N) + 256) * K * 2 >= (1LL << 32) ||
      static_cast<long long>(M) * N * 2 >= (1LL << 40) || pe.ldo != N || pe.bias || pe.residual ||
      pe.act != kActNone || pe.aux || pe.beta || pe.remap || pe.mode != 0 || pe.by || pe.bH || pe.alpha != 1.f ||
      pe.ascale0 || pe.ascale1)
    return hipErrorInvalidValue;
  const int tm = ceil_div(M, g4::BM), tn = ceil_div(N, g4::BN);
  const int group = g4_group();
  const dim3 grid(tm * tn);
  if (is_pointwise(g)) {
    if (pe.stat)
      hipLaunchKernelGGL((g4::gemm4w_kernel<g4::kEkStat, 3, 0>), grid, dim3(g4::T), 0, st, x,
                         static_cast<long long>(g->C), w, static_cast<long long>(K), pe, M, N, K, tm, tn, group,
                         g4::ConvA{});
    else
      hipLaunchKernelGGL((g4::gemm4w_kernel<0, 3, 0>), grid, dim3(g4::T), 0, st, x, static_cast<long long>(g->C), w,
                         static_cast<long long>(K), pe, M, N, K, tm, tn, group, g4::ConvA{});
    return hipGetLastError();
  }
  const g4::ConvA ca{g->H, g->W, g->C, g->P * g->Q, g->Q, g->sh, g->sw, g->ph, g->pw, g->R, g->S, 0, xb};
  if (pe.stat)
    hipLaunchKernelGGL((g4::gemm4w_kernel<g4::kEkStat, 3, 1>), grid, dim3(g4::T), 0, st, x, 0LL, w,
                       static_cast<long long>(K), pe, M, N, K, tm, tn, group, ca);
  else
    hipLaunchKernelGGL((g4::gemm4w_kernel<0, 3, 1>), grid, dim3(g4::T), 0, st, x, 0LL, w, static_cast<long long>(K),
                       pe, M, N, K, tm, tn, group, ca);
  return hipGetLastError();
}

// Unit-stride data gradient dx[N H W][C] = conv_transpose(dy[N][P][Q][K], w) on the 4-wave kernel:
// wt = w transposed to [C][R][S][K] (the B operand, K-major), dy gathered as a forward conv with
// padding (R - 1 - ph, S - 1 - pw) whose taps are walked in reverse (ConvA::flip). epi: out with
// ldo = C, and either nothing else (plain store) or the feeding-BN epilogue (by, bmask, stat:
// g = dx * ReLU bits stored, partial sums (sum g, sum g * y) per 128 rows, [2 ceil(M / 256)][2][C]).
// Needs K % 64 == 0 (dy channels), R S K >= 128. hipErrorInvalidValue: not taken.
TTDK_EXPORT int ttdk_conv_dgrad4w(const bf16_t* dy, const bf16_t* wt, const TtdkConv* g, const TtdkEpilogue* epi,
                                  hipStream_t st) {
  using namespace ttdk;
  EpiParams pe = to_epi(epi);
  const int M = g->N * g->H * g->W, N = g->C, K = g->R * g->S * g->K;
  const long long yb = static_cast<long long>(g->N) * g->P * g->Q * g->K * 2;
  const int pho = g->R - 1 - g->ph, pwo = g->S - 1 - g->pw;
  const long long shift = (static_cast<long long>(pho) * g->Q + pwo) * g->K * 2;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g->sh != 1 || g->sw != 1 || g->dh != 1 || g->dw != 1 || g->K % 64 || K < 128 || N % 8 || g->R * g->S > 32 ||
      pho < 0 || pwo < 0 || M < 1 || !al16(dy) || !al16(wt) || !al16(pe.out) || yb + shift >= (1LL << 31) ||
      (static_cast<long long>(N) + 256) * K * 2 >= (1LL << 32) || pe.ldo != N || pe.bias || pe.residual ||
      pe.act != kActNone || pe.aux || pe.beta || pe.remap || pe.mode != 0 || pe.bH || pe.by2 || pe.stat2 ||
      pe.alpha != 1.f || pe.ascale0 || pe.ascale1 || (pe.by != nullptr) != (pe.stat != nullptr) ||
      (pe.by && !al16(pe.by)))
    return hipErrorInvalidValue;
  const int tm = ceil_div(M, g4::BM), tn = ceil_div(N, g4::BN);
  const g4::ConvA ca{g->P, g->Q, g->K, g->H * g->W, g->W, 1, 1, pho, pwo, g->R, g->S, 1, yb};
  if (pe.by)
    hipLaunchKernelGGL((g4::gemm4w_kernel<g4::kEkFeed, 3, 1>), dim3(tm * tn), dim3(g4::T), 0, st, dy, 0LL, wt,
                       static_cast<long long>(K), pe, M, N, K, tm, tn, g4_group(), ca);
  else
    hipLaunchKernelGGL((g4::gemm4w_kernel<0, 3, 1>), dim3(tm * tn), dim3(g4::T), 0, st, dy, 0LL, wt,
                       static_cast<long long>(K), pe, M, N, K, tm, tn, g4_group(), ca);
  return hipGetLastError();
}

// C[M,N] = epilogue(alpha * A . B^T), A [M][K] (lda), B [N][K] (ldb) bf16 K-major; K % 64 == 0,
// N % 8 == 0, ldo % 8 == 0, 16-B aligned operands and outputs. Returns hipErrorInvalidValue for
// shapes this kernel does not take (the caller keeps another path).
TTDK_EXPORT int ttdk_gemm4w_bf16(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                 const TtdkEpilogue* epi, hipStream_t st) {
  using namespace ttdk;
  EpiParams pe = to_epi(epi);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const long long lim = 1LL << 32;
  if (K < 64 || K % 64 || N % 8 || lda % 8 || ldb % 8 || pe.ldo % 8 || !al16(A) || !al16(B) || !al16(pe.out) ||
      (static_cast<long long>(M) + 256) * lda * 2 >= lim || (static_cast<long long>(N) + 256) * ldb * 2 >= lim ||
      pe.mode != 0 || pe.remap || pe.stat || pe.by || pe.bH || (pe.bias && !al16(pe.bias)) ||
      (pe.aux && !al16(pe.aux)) || (pe.residual && ((reinterpret_cast<uintptr_t>(pe.residual) & 7) || pe.ldr % 4)))
    return hipErrorInvalidValue;
  int ek = -1;
  if (pe.act == kActNone && !pe.residual) ek = 0;
  else if (pe.act == kActGelu && !pe.residual) ek = g4::kEkGelu;
  else if (pe.act == kActDGelu && pe.residual) ek = g4::kEkDGelu;
  if (ek < 0) return hipErrorInvalidValue;
  if (pe.bias) ek |= g4::kEkBias;
  if (pe.beta) ek |= g4::kEkBeta;
  if (pe.aux) ek |= g4::kEkAux;
  const int tm = ceil_div(M, g4::BM), tn = ceil_div(N, g4::BN);
  const int sched = g4_sched();
  const int group = g4_group();
  // stagger of the persistent kernel's workgroups: a quarter tile in s_sleep 127 units (~8k
  // cycles each), from the K-tile count (~3k cycles per K-tile + the epilogue)
  const int stag = g4_stagger() ? std::max(1, ((K / 64) * 3000 + 20000) / 4 / 8128) : 0;
  // the persistent kernel's tile queue: the stream's counter buffer (gemm_conv.h tile_counters),
  // last 16 ints, shared with gemm256p_kernel (same-stream launches never overlap; each launch
  // leaves it zeroed). TTD_G4_QUEUE=0: static tile shares.
  static const int queue = getenv_int("TTD_G4_QUEUE", 1);
  int* tq = nullptr;
  if (queue && g4_cus() % 8 == 0) {
    int* c = big::tile_counters(st, 0);
    if (c) tq = c + big::kMaxCtr - 16;
  }
#define TTDK_G4_ONE(EKV) /* one tile per workgroup: SCHED 3 (>= 2 K-tiles), else the compiler's loop */  \
  if (K >= 128)                                                                                             \
    hipLaunchKernelGGL((g4::gemm4w_kernel<EKV, 3>), dim3(tm * tn), dim3(g4::T), 0, st, A, lda, B, ldb, pe, M,  \
                       N, K, tm, tn, group, g4::ConvA{});                                                   \
  else                                                                                                      \
    hipLaunchKernelGGL((g4::gemm4w_kernel<EKV, 0>), dim3(tm * tn), dim3(g4::T), 0, st, A, lda, B, ldb, pe, M,  \
                       N, K, tm, tn, group, g4::ConvA{});
#define TTDK_G4(EKV)                                                                                        \
  case EKV:                                                                                                 \
    switch (sched) {                                                                                        \
      case 0: hipLaunchKernelGGL((g4::gemm4w_kernel<EKV, 0>), dim3(tm * tn), dim3(g4::T), 0, st, A, lda, B, \
                                 ldb, pe, M, N, K, tm, tn, group, g4::ConvA{}); break;                             \
      case 30: {                                                                                          \
        const int grid = std::min(tm * tn, g4_cus()) & ~7;                                                  \
        if (grid < 8 || tm * tn <= g4_cus()) { /* one tile per workgroup: nothing to overlap */           \
          TTDK_G4_ONE(EKV)                                                                                  \
          break;                                                                                            \
        }                                                                                                   \
        hipLaunchKernelGGL((g4::gemm4p_kernel<EKV>), dim3(grid), dim3(g4::T), 0, st, A, lda, B, ldb, pe, M, N,  \
                           K, tm, tn, group, stag, tq);                                                     \
        break;                                                                                              \
      }                                                                                                     \
      default: TTDK_G4_ONE(EKV) break;                                                                      \
    }                                                                                                       \
    return hipGetLastError();
  switch (ek) {
    TTDK_G4(0)
    TTDK_G4(g4::kEkBias)
    TTDK_G4(g4::kEkBias | g4::kEkAux | g4::kEkGelu)
    TTDK_G4(g4::kEkDGelu)
    TTDK_G4(g4::kEkBeta)
    default: break;
  }
#undef TTDK_G4
#undef TTDK_G4_ONE
  return hipErrorInvalidValue;
}

// fp8 forward convolution on the 4-wave kernel (g4::gemm4k8_kernel): y[M = N P Q][K] (bf16) =
// sa * sw * conv(x8 [N][H][W][C] e4m3, w8 [K][R][S][C] e4m3), unit-stride 1x1 convs reading x8 as
// dense [M][C] rows, the others through the implicit-GEMM gather; stat (optional): BN partial sums
// of the stored output per 128 rows, [2 ceil(M / 256)][2][K]. Needs C % 128 == 0, K % 8 == 0,
// no dilation, operands under 2 GiB. hipErrorInvalidValue: not taken (the caller keeps the 8-wave
// conv_fwd_fp8).
TTDK_EXPORT int ttdk_conv_fwd4k8(const uint8_t* x8, const uint8_t* w8, const TtdkConv* g, bf16_t* out, float* stat,
                                 const float* sa, const float* sw, hipStream_t st) {
  using namespace ttdk;
  const int M = g->N * g->P * g->Q, N = g->K, K = g->R * g->S * g->C;
  const long long xb = static_cast<long long>(g->N) * g->H * g->W * g->C;
  const long long shift = (static_cast<long long>(g->ph) * g->W + g->pw) * g->C;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g->C % 128 || N % 8 || N < 8 || M < 1 || g->dh != 1 || g->dw != 1 || g->R * g->S > 32 || !sa || !sw ||
      !al16(x8) || !al16(w8) || !al16(out) || xb + shift >= (1LL << 31) ||
      (static_cast<long long>(N) + 256) * K >= (1LL << 32))
    return hipErrorInvalidValue;
  g4::K8Args P{};
  P.A = x8;
  P.lda = g->C;
  P.B = w8;
  P.ldb = K;
  P.out = out;
  P.ldo = N;
  P.stat = stat;
  P.sa = sa;
  P.sb = sw;
  P.M = M;
  P.N = N;
  P.K = K;
  P.tiles_m = ceil_div(M, g4::BM);
  P.tiles_n = ceil_div(N, g4::BN);
  P.group = g4_group();
  const dim3 grid(P.tiles_m * P.tiles_n);
  if (is_pointwise(g)) {
    if (static_cast<long long>(M) * g->C >= (1LL << 32)) return hipErrorInvalidValue;
    hipLaunchKernelGGL((g4::gemm4k8_kernel<0, false>), grid, dim3(g4::T), 0, st, P, g4::ConvA{});
    return hipGetLastError();
  }
  g4::ConvA ca{g->H, g->W, g->C, g->P * g->Q, g->Q, g->sh, g->sw, g->ph, g->pw, g->R, g->S, 0, xb};
  hipLaunchKernelGGL((g4::gemm4k8_kernel<1, false>), grid, dim3(g4::T), 0, st, P, ca);
  return hipGetLastError();
}

// fp8 data gradient of a unit-stride conv on the 4-wave kernel (g4::gemm4k8_kernel, A = dy8 in OCP
// e5m2 gathered as a forward conv with padding R - 1 - ph and the taps reversed, B = the [C][R][S][K]
// e4m3 filter; dense dy8 rows for 1x1 convs): dx (bf16) = sa * sw * ..., with by / bmask / stat the
// feeding-BN epilogue (g = dx * ReLU bits stored, (sum g, sum g y) per 128 rows: [2 ceil(M/256)][2][C]),
// else a plain store; beta (with the feeding epilogue only): g = (dx + out) * bits. Needs K % 128 == 0
// (the gradient's channels), C % 8 == 0.
// hipErrorInvalidValue: not taken (the caller keeps conv_dgrad_fp8's 8-wave kernel).
TTDK_EXPORT int ttdk_conv_dgrad4k8(const uint8_t* dy8, const uint8_t* wt8, const TtdkConv* g, bf16_t* out,
                                   const bf16_t* by, const uint8_t* bmask, float* stat, int beta, const float* sa,
                                   const float* sw, hipStream_t st) {
  using namespace ttdk;
  const int M = g->N * g->H * g->W, N = g->C, K = g->R * g->S * g->K;
  const long long yb = static_cast<long long>(g->N) * g->P * g->Q * g->K;
  const int pho = g->R - 1 - g->ph, pwo = g->S - 1 - g->pw;
  const long long shift = (static_cast<long long>(pho) * g->Q + pwo) * g->K;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g->sh != 1 || g->sw != 1 || g->dh != 1 || g->dw != 1 || g->K % 128 || N % 8 || N < 8 || g->R * g->S > 32 ||
      pho < 0 || pwo < 0 || M < 1 || !sa || !sw || !al16(dy8) || !al16(wt8) || !al16(out) ||
      yb + shift >= (1LL << 31) || (static_cast<long long>(N) + 256) * K >= (1LL << 32) ||
      (by != nullptr) != (stat != nullptr) || (by != nullptr) != (bmask != nullptr) || (by && (reinterpret_cast<uintptr_t>(by) & 7)) ||
      (beta && !by))
    return hipErrorInvalidValue;
  g4::K8Args P{};
  P.B = wt8;
  P.ldb = K;
  P.out = out;
  P.ldo = N;
  P.stat = stat;
  P.by = by;
  P.bmask = bmask;
  P.beta = beta;
  P.sa = sa;
  P.sb = sw;
  P.M = M;
  P.N = N;
  P.K = K;
  P.tiles_m = ceil_div(M, g4::BM);
  P.tiles_n = ceil_div(N, g4::BN);
  P.group = g4_group();
  const dim3 grid(P.tiles_m * P.tiles_n);
  const bool feed = by != nullptr;
  if (g->R == 1 && g->S == 1 && g->ph == 0 && g->pw == 0) {
    P.A = dy8;
    P.lda = g->K;
    if (feed) hipLaunchKernelGGL((g4::gemm4k8_kernel<0, true, true>), grid, dim3(g4::T), 0, st, P, g4::ConvA{});
    else hipLaunchKernelGGL((g4::gemm4k8_kernel<0, true, false>), grid, dim3(g4::T), 0, st, P, g4::ConvA{});
    return hipGetLastError();
  }
  P.A = dy8;
  const g4::ConvA ca{g->P, g->Q, g->K, g->H * g->W, g->W, 1, 1, pho, pwo, g->R, g->S, 1, yb};
  if (feed) hipLaunchKernelGGL((g4::gemm4k8_kernel<1, true, true>), grid, dim3(g4::T), 0, st, P, ca);
  else hipLaunchKernelGGL((g4::gemm4k8_kernel<1, true, false>), grid, dim3(g4::T), 0, st, P, ca);
  return hipGetLastError();
}
