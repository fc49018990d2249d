// Persistent streaming GEMM for the memory-bound pointwise (1x1, unit-stride) convolutions of
// ResNet's wide stages, with the neighbouring BatchNorm pass fused in as an operand PROLOGUE.
//
// Why (rocprofv3 + per-launch event timing, profiles/r2_*): at batch 1024 the 56x56 and 28x28
// 1x1 convs move 0.4-1.6 GB per launch with K = 64..512, i.e. they are HBM streams with a
// little MFMA work. The tiled engines (gemm_conv.h) run them one output tile per workgroup
// with one workgroup per CU, so every tile pays its own start-up, operand fetch and epilogue
// latency in sequence (the c1 data gradients with the BN-statistics epilogue ran at 3.0-3.4
// TB/s), and the BN apply / backward-apply passes around them each cost a full extra HBM pass.
//
// Design (MI355X-first):
//  * one persistent 512-thread workgroup per CU; each owns one BN-wide slice of the output
//    columns and keeps that slice of the weights resident in LDS for the whole launch (loaded
//    once), then walks M tiles (BM rows) with a stride of the grid;
//  * the A tile is register-staged, so a prologue can transform it on its way to LDS:
//      PRO 0  A' = x
//      PRO 1  A' = relu(x*scale + shift [+ r | + r*rscale + rshift])   (BN forward apply of the
//             producing unit, + residual / projection-shortcut BN) — A' (the unit's output) and
//             its ReLU bit mask are also stored once (slice 0), as the apply pass would have;
//      PRO 2  A' = a*(x . mask) + b*y + c   (BN backward apply: the unit's dz) — dz is stored
//             once for the weight gradient;
//    so the standalone apply pass and this GEMM's re-read of its output disappear;
//  * the next tile's global loads are issued right after the current tile is in LDS, so they
//    fly under the MFMAs and the epilogue of the current tile;
//  * each thread owns one fixed 8-channel group of A (K/8 divides 512), so the per-channel BN
//    coefficients live in registers;
//  * MFMA v_mfma_f32_16x16x32_bf16 with swapped operands (D = B.A^T): every lane ends up with 4
//    consecutive columns of one row; the tile is staged through LDS (aliasing the A buffer) and
//    written by whole 16-B row chunks through the shared epilogue (gemm_conv.h epi_rows: bias,
//    residual, accumulate, BN partial statistics, ReLU-masked BN-backward statistics);
//  * workgroups that work on the same M tile (the column slices) sit on one XCD (b % 8 equal),
//    so their shared A reads hit one L2 (speed only, never correctness).
#include "gemm_conv.h"

namespace ttdk {
namespace {
namespace pw {

constexpr int THR = 512;
constexpr int NW = THR / 64;

struct Pro {
  const bf16_t* x;       // A source [M][K], row stride K
  const bf16_t* x2;      // PRO 1: residual (or null); PRO 2: y (BN input)
  const uint8_t* mask;   // PRO 2: ReLU bits of x's unit (1 bit per element) or null
  const float* s;        // PRO 1: scale[K]; PRO 2: coef[3][K] (a, b, c)
  const float* b;        // PRO 1: shift[K]
  const float* rs;       // PRO 1: residual BN scale/shift (projection shortcut) or null
  const float* rb;
  bf16_t* side;          // transformed operand written back (slice 0), or null
  uint8_t* side_mask;    // PRO 1: ReLU bit mask of `side`, or null
  int relu;
  const bf16_t* xw;      // WG: the conv input X [M][N] (row stride N)
  float* wslab;          // WG: per-workgroup weight-gradient partials [gridDim.x][K][N]
};

// Transposed MFMA operand from a K-major [rows][64] tile image (kmaj_off layout): operand row =
// image column colbase + (lane & 15), its 8 K-values = image rows ms*32 + 8*(lane >> 4) + 0..7
// (the mn_frag pattern of gemm_conv.h on this image's swizzle; ds_read_b64_tr_b16).
__device__ __forceinline__ bf16x8_t kmaj_tr_frag(const char* lds, int colbase, int ms, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int r = ms * 32 + 8 * g + q;
  const int col = colbase + 4 * p;
  const s16x4_t lo = lds_read_tr(lds + kmaj_off(r, col >> 3) + (col & 7) * 2);
  const s16x4_t hi = lds_read_tr(lds + kmaj_off(r + 4, col >> 3) + (col & 7) * 2);
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ void load8f(const float* p, float (&d)[8]) {
  const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p), c = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    d[j] = a[j];
    d[4 + j] = c[j];
  }
}

// LDS-DMA of one 16-B (or 4-B) piece per lane into a wave-uniform LDS base (lane l lands at
// base + l*size). Inline asm on purpose: hipcc does not count it, so it never turns the waits
// for the register-staged A loads into vmcnt(0) drains (cdna_hip_programming.md §5, "Pipelining
// across barriers"); the kernel retires these pieces itself (s_waitcnt vmcnt(0) before the
// epilogue reads them). M0 is saved and restored inside the statement.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_);  // wave-uniform by construction
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(const void* src, uint32_t lds_) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  typedef __attribute__((address_space(3))) const char lds_char_t;
  return (uint32_t)(size_t)(lds_char_t*)(p);  // generic -> LDS address-space cast, then the 32-bit offset
}

// DMA = true: the epilogue's own inputs (the accumulate target `out` when beta, the BN-statistics
// source `by`, its ReLU bits `bmask`) are fetched by LDS-DMA at the start of the tile, so they
// fly under the prologue / MFMA / staging instead of being loaded row batch by row batch in
// registers (the register epilogue ran the short-K dgrads at ~3.5 TB/s). by2 / residual are not
// supported there (the host picks DMA only without them).
// WG = true (PRO 2, one column slice: BN == N): the same conv's WEIGHT gradient is fused in.
// dW[K][N] = A'^T . X with A' = the dz tile already in LDS (never stored to HBM) and X the conv
// input tile (register-staged beside A, K-major image in LDS); each workgroup keeps its dW
// partial (waves in a (K/32) x (N/(16*WNB)) grid, 32 x 16*WNB each; 32 fp32 per lane at
// K * N = 16384) over all its tiles
// and stores it once as slab blockIdx.x of pa.wslab; the host folds the slabs. This removes the
// dz store and the separate weight-gradient pass's re-read of dz and X.
template <int K, int BN, int BM, int PRO, int WM, bool DMA, bool WG = false>
__global__ __launch_bounds__(THR, 1) void pw_kernel(Pro pa, const bf16_t* __restrict__ w, long long ldw, EpiParams E,
                                                   int M, int N, int tiles_m, int nslices) {
  // weight-gradient wave tiles: 32 k x (16 * WNB) n, 8 of them covering K x BN
  constexpr int WNB = WG ? (K * BN) / (NW * 32 * 16) : 1;
  constexpr int WGN = BN / (16 * WNB);
  static_assert(!WG || (PRO == 2 && K % 32 == 0 && WNB >= 1 && BN % (16 * WNB) == 0 && (K / 32) * WGN == NW),
                "fused weight gradient: BN-bwd prologue, (K/32) x (BN/(16*WNB)) = 8 wave tiles");
  constexpr int WN = NW / WM;
  constexpr int WR = BM / WM, WC = BN / WN;  // rows / cols per wave
  constexpr int TM = WR / 16, TN = WC / 16;
  constexpr int KS = K / 64;                 // 64-wide k sub-tiles (128-B LDS rows)
  constexpr int CPR = K / 8;                 // 16-B chunks per A row
  constexpr int APASS = THR / CPR;           // A rows per pass
  constexpr int NA = BM / APASS;             // A chunks per thread per tile
  static_assert(THR % CPR == 0 && BM % APASS == 0 && NA >= 1, "A tile mapping");
  static_assert(WR % 16 == 0 && WC % 16 == 0, "wave tile");
  constexpr int SB = BN * K * 2;
  constexpr int SA = BM * K * 2;
  constexpr int PITCH = BN * 2 + 16;
  constexpr int SE = BM * PITCH + NW * 3 * BN * 4;
  constexpr int SAE = SA > SE ? SA : SE;
  constexpr int SDT = DMA ? BM * BN * 2 : 0;  // one bf16 epilogue-input tile
  constexpr int SD = DMA ? 2 * SDT + BM * BN / 8 : 0;
  // WG: X tile image (BM x BN, BN/64 sub-tiles of BM x 128 B); it lives in the epilogue-staging
  // tail of the A region when that is large enough (the staging is written only after the
  // weight-gradient MFMAs), else after the DMA region
  constexpr int SX = WG ? BM * BN * 2 : 0;
  constexpr bool XALIAS = WG && SE - SA >= SX;
  constexpr int SXE = WG && !XALIAS ? SX : 0;
  static_assert(SB + SAE + SD + SXE <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[SB + SAE + SD + SXE];
  char* const sB = smem;
  char* const sA = smem + SB;  // A tile; the epilogue staging aliases it
  char* const sDo = smem + SB + SAE;  // DMA: old `out` (beta), `by`, ReLU bits
  char* const sDy = sDo + SDT;
  char* const sDm = sDo + 2 * SDT;
  char* const sX = XALIAS ? sA + SA : smem + SB + SAE + SD;

  const int b = blockIdx.x;
  const int xcd = b & 7, rq = b >> 3;
  const int slice = rq % nslices;
  const int g = xcd + 8 * (rq / nslices);
  const int G = gridDim.x / nslices;
  const int n0 = slice * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // resident weight slice: rows n0 .. n0+BN of w[N][K]
  for (int q = tid; q < BN * CPR; q += THR) {
    const int row = q / CPR, c = q % CPR;
    const int n = n0 + row;
    const uint4 v = n < N ? ldg16(w + static_cast<long long>(n) * ldw + c * 8) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(sB + (c >> 3) * (BN * 128) + kmaj_off(row, c & 7)) = v;
  }

  // this thread's fixed A channel group and its BN coefficients
  const int ac = tid % CPR, ar = tid / CPR;
  float k0[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k0[j] = k1[j] = k2[j] = k3[j] = 0.f;
  if constexpr (PRO == 1) {
    load8f(pa.s + ac * 8, k0);
    load8f(pa.b + ac * 8, k1);
    if (pa.rs) {
      load8f(pa.rs + ac * 8, k2);
      load8f(pa.rb + ac * 8, k3);
    }
  } else if constexpr (PRO == 2) {
    load8f(pa.s + ac * 8, k0);
    load8f(pa.s + K + ac * 8, k1);
    load8f(pa.s + 2 * K + ac * 8, k2);
  }
  const bool write_side = slice == 0 && pa.side != nullptr;

  uint4 ra[NA], rx[NA];
  uint32_t rm[NA];
  constexpr int XCPR = BN / 8;                          // 16-B chunks per X row
  constexpr int NXL = WG ? (BM * XCPR) / THR : 1;       // X chunks per thread per tile
  static_assert(!WG || (BM * XCPR) % THR == 0, "X tile mapping");
  uint4 rw[NXL];
  f32x4_t wacc[WG ? 2 : 1][WNB];
  if constexpr (WG) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < WNB; ++c) wacc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  auto load_tile = [&](int t) {
    const long long m0 = static_cast<long long>(t) * BM;
    if constexpr (WG) {
#pragma unroll
      for (int i = 0; i < NXL; ++i) {
        const int q = tid + THR * i;
        const long long row = m0 + q / XCPR;
        rw[i] = row < M ? ldg16(pa.xw + row * BN + (q % XCPR) * 8) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const long long row = m0 + ar + APASS * i;
      const bool ok = row < M;
      const long long off = row * K + ac * 8;
      ra[i] = ok ? ldg16(pa.x + off) : make_uint4(0, 0, 0, 0);
      if constexpr (PRO == 1) {
        if (pa.x2) rx[i] = ok ? ldg16(pa.x2 + off) : make_uint4(0, 0, 0, 0);
      } else if constexpr (PRO == 2) {
        rx[i] = ok ? ldg16(pa.x2 + off) : make_uint4(0, 0, 0, 0);
        rm[i] = (ok && pa.mask) ? pa.mask[off >> 3] : 0xffu;
      }
    }
  };
  auto stage_tile = [&](int t) {
    const long long m0 = static_cast<long long>(t) * BM;
    if constexpr (WG) {
#pragma unroll
      for (int i = 0; i < NXL; ++i) {
        const int q = tid + THR * i;
        const int row = q / XCPR, cc = q % XCPR;
        *reinterpret_cast<uint4*>(sX + (cc >> 3) * (BM * 128) + kmaj_off(row, cc & 7)) = rw[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int lrow = ar + APASS * i;
      const long long row = m0 + lrow;
      const bool ok = row < M;
      const long long off = row * K + ac * 8;
      uint4 v = ra[i];
      if constexpr (PRO == 1) {  // = apply_kernel (batchnorm.hip), element for element
        float f[8];
        unpack8(ra[i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = f[j] * k0[j] + k1[j];
        if (pa.x2) {
          float r[8];
          unpack8(rx[i], r);
          if (pa.rs) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += r[j] * k2[j] + k3[j];
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += r[j];
          }
        }
        if (pa.relu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = relu(f[j]);
        }
        v = ok ? pack8(f) : make_uint4(0, 0, 0, 0);
        if (write_side && ok) {
          *reinterpret_cast<uint4*>(pa.side + off) = v;
          if (pa.side_mask) {
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            uint32_t mb = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t h = (wv[j >> 1] >> (16 * (j & 1))) & 0xffffu;
              mb |= ((h & 0x7fffu) != 0 && !(h & 0x8000u) ? 1u : 0u) << j;
            }
            pa.side_mask[off >> 3] = static_cast<uint8_t>(mb);
          }
        }
      } else if constexpr (PRO == 2) {  // = bwd_apply_kernel
        float gq[8], yf[8];
        unpack8(ra[i], gq);
#pragma unroll
        for (int j = 0; j < 8; ++j) gq[j] = (rm[i] >> j) & 1u ? gq[j] : 0.f;
        unpack8(rx[i], yf);
#pragma unroll
        for (int j = 0; j < 8; ++j) gq[j] = k0[j] * gq[j] + k1[j] * yf[j] + k2[j];
        v = ok ? pack8(gq) : make_uint4(0, 0, 0, 0);
        if (write_side && ok) *reinterpret_cast<uint4*>(pa.side + off) = v;
      }
      *reinterpret_cast<uint4*>(sA + (ac >> 3) * (BM * 128) + kmaj_off(lrow, ac & 7)) = v;
    }
  };

  auto issue_epi_dma = [&](int t) {
    const long long m0 = static_cast<long long>(t) * BM;
    constexpr int CPRE = BN / 8;          // 16-B chunks per tile row
    constexpr int NI = BM * BN / 8 / 64;  // wave instructions per tile
#pragma unroll
    for (int i = wave; i < NI; i += NW) {
      const int q = i * 64 + lane;
      const int row = q / CPRE, cc = q % CPRE;
      const long long m = m0 + row;
      const bool ok = m < M;
      const long long o = (m * E.ldo + n0 + cc * 8) * 2;
      if (E.beta)
        dma16(ok && beta_row(E, static_cast<int>(m)) ? static_cast<const char*>(E.out) + o
                                                     : reinterpret_cast<const char*>(big::g_zero),
              lds_addr(sDo) + i * 1024);
      if (E.by)
        dma16(ok ? reinterpret_cast<const char*>(E.by) + o : reinterpret_cast<const char*>(big::g_zero),
              lds_addr(sDy) + i * 1024);
    }
    if (E.bmask) {
      constexpr int WPR = BN / 32;           // 4-B mask words per tile row
      constexpr int NI4 = BM * BN / 32 / 64;
#pragma unroll
      for (int i = wave; i < NI4; i += NW) {
        const int wd = i * 64 + lane;
        const int row = wd / WPR, wi = wd % WPR;
        const long long m = m0 + row;
        dma4(m < M ? reinterpret_cast<const char*>(E.bmask) + (m * E.ldo + n0) / 8 + wi * 4
                   : reinterpret_cast<const char*>(big::g_zero),
             lds_addr(sDm) + i * 256);
      }
    }
  };

  int t = g;
  if (t < tiles_m) load_tile(t);
  for (; t < tiles_m; t += G) {
    stage_tile(t);
    __syncthreads();
    if constexpr (DMA) issue_epi_dma(t);     // lands under the MFMAs and the staging below
    if (t + G < tiles_m) load_tile(t + G);  // in flight under this tile's MFMAs and epilogue
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int c = 0; c < TN; ++c) acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sub = 0; sub < KS; ++sub) {
      const char* pA = sA + sub * (BM * 128);
      const char* pB = sB + sub * (BN * 128);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t af[TM], bfr[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
          af[a] = lds_read_b128(pA + kmaj_off(wm * WR + a * 16 + (lane & 15), ks * 4 + (lane >> 4)));
#pragma unroll
        for (int c = 0; c < TN; ++c)
          bfr[c] = lds_read_b128(pB + kmaj_off(wn * WC + c * 16 + (lane & 15), ks * 4 + (lane >> 4)));
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int c = 0; c < TN; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[c], af[a], acc[a][c], 0, 0, 0);
      }
    }
    if constexpr (WG) {
      // dW[k][n] += sum over this tile's rows of dz[m][k] * X[m][n]: lane holds n = 4g + i of
      // each 16-block, k = lane & 15 (rows past M are zero in both images)
      const int wk = wave / WGN, wx = wave % WGN;
#pragma unroll
      for (int ms = 0; ms < BM / 32; ++ms) {
        bf16x8_t kf[2], nf[WNB];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int kc = wk * 32 + a * 16;
          kf[a] = kmaj_tr_frag(sA + (kc >> 6) * (BM * 128), kc & 63, ms, lane);
        }
#pragma unroll
        for (int c = 0; c < WNB; ++c) {
          const int nc = wx * (16 * WNB) + c * 16;
          nf[c] = kmaj_tr_frag(sX + (nc >> 6) * (BM * 128), nc & 63, ms, lane);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < WNB; ++c) wacc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nf[c], kf[a], wacc[a][c], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done reading sA: stage the tile over it
    const int m0 = t * BM;
    const int gq4 = lane >> 4, i16 = lane & 15;
    const float alpha_e = epi_alpha(E);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int c = 0; c < TN; ++c) {
        const int r = wm * WR + a * 16 + i16, cc = wn * WC + c * 16 + 4 * gq4;
        const f32x4_t v = acc[a][c] * alpha_e;
        *reinterpret_cast<uint2*>(sA + r * PITCH + cc * 2) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    __syncthreads();
    constexpr int ECPR = BN / 8;
    constexpr int RPP = THR / ECPR;
    const int c = tid % ECPR, r0 = tid / ECPR;
    const int n = n0 + c * 8;
    const bool nfull = n + 8 <= N;
    const bool vst = nfull && (E.ldo & 7) == 0;
    const bool vres = nfull && (E.ldr & 7) == 0;
    float bias8[8], s8[8], q8[8], r8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bias8[j] = (E.bias && n + j < N) ? E.bias[n + j] : 0.f;
      s8[j] = q8[j] = r8[j] = 0.f;
    }
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces landed
      __syncthreads();                                    // ... and every other wave's
      bf16_t* outp = static_cast<bf16_t*>(E.out);
#pragma unroll 2
      for (int r = r0; r < BM; r += RPP) {
        const int m = m0 + r;
        if (m >= M) break;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(sA + r * PITCH + c * 16), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += bias8[j];
        if (E.beta) {
          float ov[8];
          unpack8(*reinterpret_cast<const uint4*>(sDo + r * (BN * 2) + c * 16), ov);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] += ov[j];
        }
        if (E.act == kActRelu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = relu(f[j]);
        }
        if (E.by) {
          const uint32_t mb = E.bmask ? static_cast<uint32_t>(*reinterpret_cast<const uint8_t*>(sDm + r * (BN / 8) + c))
                                      : 0xffu;
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = (mb >> j) & 1u ? f[j] : 0.f;
        }
        const uint4 packed = pack8(f);
        *reinterpret_cast<uint4*>(outp + static_cast<long long>(m) * E.ldo + n) = packed;
        if (E.stat) {
          float sv[8], yv[8];
          unpack8(packed, sv);
          if (E.by) unpack8(*reinterpret_cast<const uint4*>(sDy + r * (BN * 2) + c * 16), yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            s8[j] += sv[j];
            q8[j] += sv[j] * (E.by ? yv[j] : sv[j]);
          }
        }
      }
    } else if (E.beta || E.residual || E.by) {
      epi_rows<BM, RPP, PITCH, true, PRO == 0 ? 4 : 2>(E, sA, c, r0, n, m0, M, N, vst, vres, bias8, s8, q8, r8);
    } else {
      epi_rows<BM, RPP, PITCH, false>(E, sA, c, r0, n, m0, M, N, vst, vres, bias8, s8, q8, r8);
    }
    if (E.stat) {
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
      float* red = reinterpret_cast<float*>(sA + BM * PITCH);  // [NW][3][BN]
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
          E.stat[(static_cast<long long>(t) * 2 + 0) * N + n0 + t2] = ss;
          E.stat[(static_cast<long long>(t) * 2 + 1) * N + n0 + t2] = qq;
          if (E.stat2) {
            E.stat2[(static_cast<long long>(t) * 2 + 0) * N + n0 + t2] = ss;
            E.stat2[(static_cast<long long>(t) * 2 + 1) * N + n0 + t2] = rr;
          }
        }
      }
    }
    __syncthreads();  // staging / statistics reads done before the next tile overwrites sA
  }
  if constexpr (WG) {
    const int wk = wave / WGN, wx = wave % WGN;
    float* slab = pa.wslab + static_cast<long long>(blockIdx.x) * K * BN;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < WNB; ++c) {
        const int k = wk * 32 + a * 16 + (lane & 15), n = wx * (16 * WNB) + c * 16 + 4 * (lane >> 4);
        *reinterpret_cast<f32x4_t*>(slab + k * BN + n) = wacc[a][c];
      }
  }
}

// (K, N) -> tile: BN (column slice kept in LDS), BM (rows per tile), DMA epilogue; 0 = not
// handled here. `dma` asks for the LDS-DMA epilogue (accumulate / BN-statistics inputs).
struct Cfg {
  int bn, bm, dma;
};
inline Cfg pick(int N, int K, bool dma) {
  if (N % 64 || N < 64) return {0, 0, 0};
  if (dma) {
    switch (K) {
      case 64:
        return {N >= 256 ? 256 : N, 64, 1};
      case 128:
        return {N >= 128 ? 128 : 64, 64, 1};
      case 256:
        return {64, 128, 1};
      default:
        return {0, 0, 0};
    }
  }
  switch (K) {
    case 64:
    case 128:
      return {N >= 256 ? 256 : N, 128, 0};
    case 256:
      return {N >= 128 ? 128 : 64, N >= 128 ? 64 : 128, 0};
    case 512:
      return {64, 64, 0};
    default:
      return {0, 0, 0};
  }
}

inline int grid_for(int M, int N, int BN, int BM, int max_wgs = 0) {
  const int nsl = ceil_div(N, BN), tiles = ceil_div(M, BM);
  int cus = big::device_cus();
  if (max_wgs > 0 && max_wgs < cus) cus = max_wgs;  // a side-stream launch leaves CUs to the main chain
  int gq = cus / (8 * nsl);  // one persistent workgroup per (free) CU in all
  if (gq < 1) gq = 1;
  const int need = ceil_div(tiles, 8);
  if (gq > need) gq = need;
  return 8 * nsl * gq;
}

template <int K, int BN, int BM, int PRO, int WM, bool DMA, bool WG = false>
hipError_t launch(const Pro& pa, const bf16_t* w, long long ldw, const EpiParams& E, int M, int N, hipStream_t st,
                  int grid = 0) {
  const int nsl = ceil_div(N, BN), tiles = ceil_div(M, BM);
  if (grid <= 0) grid = grid_for(M, N, BN, BM);
  hipLaunchKernelGGL((pw_kernel<K, BN, BM, PRO, WM, DMA, WG>), dim3(grid), dim3(THR), 0, st, pa, w, ldw, E, M, N,
                     tiles, nsl);
  return hipGetLastError();
}

// The fused data + weight gradient (WG) instantiations: the (K, N) = (256, 64) and (64, 256)
// stage-2 shapes (one column slice, K * N = 16384) and the first block's (64, 64) c1.
inline hipError_t dispatch_wg(const Pro& pa, const bf16_t* w, long long ldw, const EpiParams& E, int M, int N, int K,
                              bool dma, int grid, hipStream_t st) {
  const Cfg c = pick(N, K, dma);
  if (c.bn != N) return hipErrorInvalidValue;
#define PW_WG_CASE(K_, BN_, BM_, WM_, D_)                     \
  if (K == K_ && c.bn == BN_ && c.bm == BM_ && c.dma == D_) \
    return launch<K_, BN_, BM_, 2, WM_, D_, true>(pa, w, ldw, E, M, N, st, grid);
  PW_WG_CASE(64, 256, 128, 2, false)
  PW_WG_CASE(256, 64, 128, 4, false)
  PW_WG_CASE(64, 256, 64, 2, true)
  PW_WG_CASE(256, 64, 128, 4, true)
  PW_WG_CASE(64, 64, 128, 4, false)
  PW_WG_CASE(64, 64, 64, 4, true)
#undef PW_WG_CASE
  return hipErrorInvalidValue;
}

template <int PRO>
hipError_t dispatch(const Pro& pa, const bf16_t* w, long long ldw, const EpiParams& E, int M, int N, int K, bool dma,
                    hipStream_t st) {
  const Cfg c = pick(N, K, dma);
#define PW_CASE(K_, BN_, BM_, WM_, D_)                                 \
  if (K == K_ && c.bn == BN_ && c.bm == BM_ && c.dma == D_) \
    return launch<K_, BN_, BM_, PRO, WM_, D_>(pa, w, ldw, E, M, N, st);
  PW_CASE(64, 256, 128, 2, false)
  PW_CASE(64, 128, 128, 2, false)
  PW_CASE(64, 64, 128, 4, false)
  PW_CASE(128, 256, 128, 2, false)
  PW_CASE(128, 128, 128, 2, false)
  PW_CASE(128, 64, 128, 4, false)
  PW_CASE(256, 128, 64, 2, false)
  PW_CASE(256, 64, 128, 4, false)
  PW_CASE(512, 64, 64, 4, false)
  PW_CASE(64, 256, 64, 2, true)
  PW_CASE(64, 128, 64, 2, true)
  PW_CASE(64, 64, 64, 4, true)
  PW_CASE(128, 128, 64, 2, true)
  PW_CASE(128, 64, 64, 4, true)
  PW_CASE(256, 64, 128, 4, true)
#undef PW_CASE
  return hipErrorInvalidValue;
}

}  // namespace pw
}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Rows per output tile (the BN partial-statistics row count is ceil(M / rows)) of ttdk_pw_conv
// for an N x K pointwise conv, or 0 when the shape is not handled by the streaming kernel.
TTDK_EXPORT int ttdk_pw_rows(int N, int K, int dma) { return pw::pick(N, K, dma != 0).bm; }

// Workgroups (= weight-gradient slabs) of ttdk_pw_conv_wgrad for this shape; 0 = not fusable.
// max_wgs > 0 caps the persistent grid (a launch on the side stream must not hold every CU).
TTDK_EXPORT int ttdk_pw_wgrad_slabs(int M, int N, int K, int dma, int max_wgs) {
  const pw::Cfg c = pw::pick(N, K, dma != 0);
  const bool shape = (K * N == 16384 && N % 64 == 0) || (K == 64 && N == 64);
  if (c.bm == 0 || c.bn != N || K % 32 || !shape) return 0;
  return pw::grid_for(M, N, c.bn, c.bm, max_wgs);
}

// out[M, N] = epilogue( A'[M, K] . w[N, K]^T ) with A' from the prologue `pro` (see above).
// x, x2: [M][K] bf16 (row stride K); mask_in: bits of x (pro 2); s/b/rs/rb: BN coefficients
// (pro 1: scale, shift, residual scale/shift; pro 2: s = coef[3][K]); side/side_mask: where the
// prologue stores A' (and its ReLU bits). The epilogue descriptor is the GEMM engine's.
TTDK_EXPORT int ttdk_pw_conv(const bf16_t* x, const bf16_t* x2, const uint8_t* mask_in, const float* s, const float* b,
                             const float* rs, const float* rb, bf16_t* side, uint8_t* side_mask, int relu, int pro,
                             const bf16_t* w, long long ldw, int M, int N, int K, const TtdkEpilogue* epi,
                             hipStream_t st) {
  const EpiParams e0 = to_epi(epi);
  // the LDS-DMA epilogue serves the accumulate / BN-statistics inputs (no residual, no second source)
  const bool dma = (e0.beta || e0.by) && !e0.residual && !e0.by2 && e0.act == 0 && !e0.bias;
  if (pw::pick(N, K, dma).bm == 0 || ldw % 8 || (reinterpret_cast<uintptr_t>(x) & 15) || pro < 0 || pro > 2) return hipErrorInvalidValue;
  const EpiParams e = to_epi(epi);
  if (e.mode != 0 || e.remap || e.ldo % 8 || (e.residual && e.ldr % 8)) return hipErrorInvalidValue;
  if (pro == 1 && (!s || !b || (rs && (!rb || !x2)))) return hipErrorInvalidValue;
  if (pro == 2 && (!s || !x2)) return hipErrorInvalidValue;
  if (side_mask && pro != 1) return hipErrorInvalidValue;
  const pw::Pro pa{x, x2, mask_in, s, b, rs, rb, side, side_mask, relu, nullptr, nullptr};
  switch (pro) {
    case 0:
      return pw::dispatch<0>(pa, w, ldw, e, M, N, K, dma, st);
    case 1:
      return pw::dispatch<1>(pa, w, ldw, e, M, N, K, dma, st);
    default:
      return pw::dispatch<2>(pa, w, ldw, e, M, N, K, dma, st);
  }
}

// ttdk_pw_conv with pro = 2 (BN backward as the operand prologue) and the conv's weight gradient
// fused in (see pw_kernel WG): dx = epilogue(dz . w^T) as ttdk_pw_conv, dw[K][N] (fp32, += when
// beta_w) = dz^T . xw with dz never stored; ws: ttdk_pw_wgrad_slabs(M, N, K, dma, max_wgs) * K * N
// floats. dw == null: the slabs are left in ws for the caller to fold (ttdk_splitk_reduce), e.g. on
// the weight-gradient side stream so the data-gradient chain does not wait for the fold.
TTDK_EXPORT int ttdk_pw_conv_wgrad(const bf16_t* g, const bf16_t* y, const uint8_t* mask_in, const float* coef,
                                   const bf16_t* xw, const bf16_t* w, long long ldw, int M, int N, int K,
                                   const TtdkEpilogue* epi, float* dw, float* ws, int beta_w, int max_wgs,
                                   hipStream_t st) {
  const EpiParams e = to_epi(epi);
  const bool dma = (e.beta || e.by) && !e.residual && !e.by2 && e.act == 0 && !e.bias;
  const int slabs = ttdk_pw_wgrad_slabs(M, N, K, dma, max_wgs);
  if (!slabs || !g || !y || !coef || !xw || !ws || ldw % 8 || (reinterpret_cast<uintptr_t>(g) & 15) ||
      (reinterpret_cast<uintptr_t>(xw) & 15) || e.mode != 0 || e.remap || e.ldo % 8 || (e.residual && e.ldr % 8))
    return hipErrorInvalidValue;
  const pw::Pro pa{g, y, mask_in, coef, nullptr, nullptr, nullptr, nullptr, nullptr, 1, xw, ws};
  hipError_t r = pw::dispatch_wg(pa, w, ldw, e, M, N, K, dma, slabs, st);
  if (r != hipSuccess || !dw) return r;
  return splitk_reduce(ws, slabs, static_cast<long long>(K) * N, dw, beta_w, st);
}
