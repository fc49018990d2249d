// Persistent halo-tiled 3x3 stride-1 convolution (forward, and the data gradient as the same
// convolution over flipped / transposed filters) with the producing BatchNorm fused in as an
// operand prologue — ResNet-50's 56x56 64->64 bottleneck convs (conv2_block*_2), their forward
// and data gradient.
//
// Why (tools/op_timing.py, profiles/r2_*): the tiled implicit-GEMM engine (gemm_conv.h) ran
// these at 370-430 TF/s: every output tile re-gathers its 9 taps through L2 (each input pixel
// is fetched 9 times), the 64-wide output tile gives little reuse per gathered byte, and the
// BN apply / backward-apply pass before each conv costs a full extra HBM round trip.
//
// Design (MI355X-first):
//  * one persistent 512-thread workgroup per CU keeps the whole filter (64 x 576 bf16 = 72 KiB)
//    resident in LDS, loaded once, and walks output tiles of TH full image rows (TH x W pixels);
//  * per tile the (TH+2) x (W+2) x C input halo (72.5 KiB) is loaded ONCE into LDS (each input
//    pixel is fetched 1.25x instead of 9x) through registers, so a prologue transforms it on the
//    way: PRO 1 = relu(x*scale + shift) (BN forward apply of the producing conv), PRO 2 =
//    a*g + b*y + c (BN backward apply); the halo's zero padding stays zero, and the transformed
//    interior is written back once (side / side_mask) for the weight gradient and the backward;
//  * the next tile's halo loads are issued before this tile's MFMAs, so they fly under them;
//  * the implicit GEMM reads A straight from the halo: output pixel p, tap (r, s) is halo pixel
//    q = p_row*(W+2) + p_col + r*(W+2) + s. The halo is stored channel-chunk-major — region c
//    (a 256-B multiple) holds 16-B chunk c of every halo pixel — so a 16-lane ds_read_b128 group
//    reads 16 consecutive pixels of one chunk (conflict-free but for row wraps: 4.6 LDS cycles
//    per 4 groups vs the ideal 4, measured by brute force over every tap shift), and every
//    (tap, k-step) is a compile-time offset from 7 per-lane base addresses: no address VALU in
//    the MFMA loop. Staging lanes are mapped 8 pixels x 8 chunks per wave (a wave still loads
//    1 KiB of contiguous NHWC memory), so each 8-lane ds_write_b128 group writes 128 contiguous
//    bytes;
//  * v_mfma_f32_16x16x32_bf16 with swapped operands, 8 waves as 4 (rows) x 2 (cols), 112 x 32
//    outputs per wave (7 x 2 MFMA blocks: each A fragment feeds 2 MFMAs, each B fragment 7);
//  * epilogue shared with the streaming pointwise kernel (stream_epi.h / epi_rows): BN partial
//    statistics per tile, or the next unit's ReLU-masked gradient + BN-backward sums (dgrad).
#include "stream_epi.h"

namespace ttdk {
namespace {
namespace c3 {

constexpr int THR = 512;
constexpr int NW = THR / 64;

struct Pro {
  const bf16_t* x;      // input [Nimg][H][W][C]
  const bf16_t* x2;     // PRO 2: y (BN input of x's unit), same layout
  const uint8_t* mask;  // PRO 2: ReLU bits of x (or null)
  const float* s;       // PRO 1: scale[C]; PRO 2: coef[3][C]
  const float* b;       // PRO 1: shift[C]
  bf16_t* side;         // transformed input written back (interior), or null
  uint8_t* side_mask;   // PRO 1: its ReLU bits, or null
};

__device__ __forceinline__ void load8f(const float* p, float (&d)[8]) {
  const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p), c = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    d[j] = a[j];
    d[4 + j] = c[j];
  }
}

// staging slot q (= tid + THR*i) -> (halo pixel, 16-B channel chunk): 8 pixels x 8 chunks per
// 64 slots, chunk fixed per thread
template <int CP>
__device__ __forceinline__ int slot_chunk(int q) { return (q >> 3) % CP; }
template <int CP>
__device__ __forceinline__ int slot_pix(int q) { return (q & 7) + 8 * (q / (8 * CP)); }

template <int C, int BN, int TH, int W, int PRO, bool FLIP, int WM>
__global__ __launch_bounds__(THR, 1) void conv3_kernel(Pro pa, const bf16_t* __restrict__ w, EpiParams E, int H,
                                                      int N, int tiles, int nslices) {
  constexpr int BM = TH * W;              // output pixels per tile
  constexpr int HR = TH + 2, HC = W + 2;  // halo rows / cols
  constexpr int CP = C / 8;               // 16-B chunks per pixel
  constexpr int KT = 9 * C;               // reduction length
  constexpr int WN = NW / WM;
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 16, TN = WC / 16;
  constexpr int NPIX = HR * HC;
  constexpr int NCH = ((NPIX + 7) / 8) * 8 * CP;   // staging slots per tile (8-pixel groups)
  constexpr int NA = (NCH + THR - 1) / THR;         // per thread
  constexpr int SB = BN * KT * 2;                   // resident filter slice
  constexpr int REG = ((NPIX * 16 + 255) / 256) * 256;  // bytes per channel-chunk region
  constexpr int SH = CP * REG;                      // halo
  constexpr int PITCH = BN * 2 + 16;
  constexpr int SE = BM * PITCH + NW * 3 * BN * 4;  // epilogue staging + statistics (aliases the halo)
  constexpr int SAE = SH > SE ? SH : SE;
  static_assert(C % 64 == 0 && BN % 32 == 0 && WR % 16 == 0 && WC % 16 == 0, "tile shape");
  static_assert(THR % (8 * CP) == 0, "fixed channel chunk per thread");
  static_assert(SB + SAE <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[SB + SAE];
  char* const sB = smem;
  char* const sA = smem + SB;

  const int b = blockIdx.x;
  const int G = gridDim.x / nslices;
  // adjacent tiles (which share two halo rows) go to workgroups of one XCD, so the overlap hits
  // that XCD's L2
  const int xcd = b & 7, rq = b >> 3;
  const int slice = rq % nslices;
  const int per_xcd = G / 8;
  const int g = xcd * per_xcd + rq / nslices;
  const int n0 = slice * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_per_img = H / TH;

  // resident filter slice: B[n][k], k = tap*C + c  (FLIP: data gradient, w = [Cout][3][3][Cin]
  // transposed filter read with the taps reversed)
  for (int q = tid; q < BN * (KT / 8); q += THR) {
    const int row = q / (KT / 8), kk = q % (KT / 8);
    const int tap = kk / CP, cc = kk % CP;
    const int n = n0 + row;
    const int src_tap = FLIP ? 8 - tap : tap;
    const uint4 v = n < N ? ldg16(w + (static_cast<long long>(n) * 9 + src_tap) * C + cc * 8) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(sB + (kk >> 3) * (BN * 128) + kmaj_off(row, kk & 7)) = v;
  }

  // this thread's fixed channel chunk (its prologue coefficients are re-read from L1/L2 at each
  // staging instead of being held in registers across the MFMA loop)
  const int ac = slot_chunk<CP>(tid);
  const bool write_side = slice == 0 && pa.side != nullptr;

  // lane's A-read base (halo pixel of tap (0,0), its k-chunk region) for each MFMA row block
  const char* abase[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const int i = wm * WR + a * 16 + (lane & 15);
    abase[a] = sA + (lane >> 4) * REG + ((i / W) * HC + (i % W)) * 16;
  }

  uint4 ra[NA], rx[PRO == 2 ? NA : 1];
  uint32_t rm[(NA + 3) / 4];  // PRO 2: ReLU mask bytes, four per register
  auto load_tile = [&](int t) {
    const int img = t / tiles_per_img, h0 = (t % tiles_per_img) * TH;
#pragma unroll
    for (int i = 0; i < (NA + 3) / 4; ++i) rm[i] = 0;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int pix = slot_pix<CP>(tid + THR * i);
      const int hr = pix / HC, hc = pix % HC;
      const int h = h0 - 1 + hr, x = hc - 1;
      const bool ok = pix < NPIX && h >= 0 && h < H && x >= 0 && x < W;
      const long long off = ((static_cast<long long>(img) * H + h) * W + x) * C + ac * 8;
      ra[i] = ok ? ldg16(pa.x + off) : make_uint4(0, 0, 0, 0);
      if constexpr (PRO == 2) {
        rx[i] = ok ? ldg16(pa.x2 + off) : make_uint4(0, 0, 0, 0);
        rm[i >> 2] |= static_cast<uint32_t>((ok && pa.mask) ? pa.mask[off >> 3] : 0xffu) << (8 * (i & 3));
      }
    }
  };
  auto stage_tile = [&](int t) {
    const int img = t / tiles_per_img, h0 = (t % tiles_per_img) * TH;
    float k0[8], k1[8], k2[8];
    if constexpr (PRO == 1) {
      load8f(pa.s + ac * 8, k0);
      load8f(pa.b + ac * 8, k1);
    } else if constexpr (PRO == 2) {
      load8f(pa.s + ac * 8, k0);
      load8f(pa.s + C + ac * 8, k1);
      load8f(pa.s + 2 * C + ac * 8, k2);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int pix = slot_pix<CP>(tid + THR * i);
      if (tid + THR * i >= NCH) break;
      const int hr = pix / HC, hc = pix % HC;
      const int h = h0 - 1 + hr, x = hc - 1;
      const bool ok = h >= 0 && h < H && x >= 0 && x < W;
      const bool interior = ok && hr >= 1 && hr <= TH;
      const long long off = ((static_cast<long long>(img) * H + h) * W + x) * C + ac * 8;
      uint4 v = ra[i];
      if constexpr (PRO == 1) {  // = apply_kernel (batchnorm.hip) with ReLU
        float f[8];
        unpack8(ra[i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = relu(f[j] * k0[j] + k1[j]);
        v = ok ? pack8(f) : make_uint4(0, 0, 0, 0);
        if (write_side && interior) {
          *reinterpret_cast<uint4*>(pa.side + off) = v;
          if (pa.side_mask) {
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            uint32_t mb = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t hb = (wv[j >> 1] >> (16 * (j & 1))) & 0xffffu;
              mb |= ((hb & 0x7fffu) != 0 && !(hb & 0x8000u) ? 1u : 0u) << j;
            }
            pa.side_mask[off >> 3] = static_cast<uint8_t>(mb);
          }
        }
      } else if constexpr (PRO == 2) {  // = bwd_apply_kernel
        float gq[8], yf[8];
        unpack8(ra[i], gq);
        const uint32_t mb = rm[i >> 2] >> (8 * (i & 3));
#pragma unroll
        for (int j = 0; j < 8; ++j) gq[j] = (mb >> j) & 1u ? gq[j] : 0.f;
        unpack8(rx[i], yf);
#pragma unroll
        for (int j = 0; j < 8; ++j) gq[j] = k0[j] * gq[j] + k1[j] * yf[j] + k2[j];
        v = ok ? pack8(gq) : make_uint4(0, 0, 0, 0);
        if (write_side && interior) *reinterpret_cast<uint4*>(pa.side + off) = v;
      }
      *reinterpret_cast<uint4*>(sA + ac * REG + pix * 16) = v;  // padding pixels (>= NPIX) are never read
    }
  };

  int t = g;
  if (t < tiles) load_tile(t);
  for (; t < tiles; t += G) {
    stage_tile(t);
    __syncthreads();
    if (t + G < tiles) load_tile(t + G);  // in flight under this tile's MFMAs and epilogue
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int c = 0; c < TN; ++c) acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int tq = (tap / 3) * HC + (tap % 3);
#pragma unroll
      for (int kc = 0; kc < C / 32; ++kc) {
        const int kglob = tap * C + kc * 32;  // first k of this 32-wide step
        const char* pB = sB + (kglob >> 6) * (BN * 128);
        const int kchunk = ((kglob & 63) >> 3) + (lane >> 4);
        bf16x8_t af[TM], bfr[TN];
#pragma unroll
        for (int c = 0; c < TN; ++c) bfr[c] = lds_read_b128(pB + kmaj_off(wn * WC + c * 16 + (lane & 15), kchunk));
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = lds_read_b128(abase[a] + kc * 4 * REG + tq * 16);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int c = 0; c < TN; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[c], af[a], acc[a][c], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done reading the halo: stage the tile over it
    sepi::stage_acc<TM, TN, WR, WC, PITCH>(sA, acc, wm, wn, lane, epi_alpha(E));
    __syncthreads();
    constexpr int ECPR = BN / 8;
    constexpr int RPP = THR / ECPR;
    const int m0 = t * BM;
    const int c = tid % ECPR, r0 = tid / ECPR;
    const int n = n0 + c * 8;
    const bool nfull = n + 8 <= N;
    const bool vst = nfull && (E.ldo & 7) == 0;
    float bias8[8], s8[8], q8[8], r8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bias8[j] = (E.bias && n + j < N) ? E.bias[n + j] : 0.f;
      s8[j] = q8[j] = r8[j] = 0.f;
    }
    const int M = tiles * BM;
    if (E.beta || E.residual || E.by)
      epi_rows<BM, RPP, PITCH, true, 2>(E, sA, c, r0, n, m0, M, N, vst, vst, bias8, s8, q8, r8);
    else
      epi_rows<BM, RPP, PITCH, false>(E, sA, c, r0, n, m0, M, N, vst, vst, bias8, s8, q8, r8);
    if (E.stat)
      sepi::tile_stats<BN, NW, THR, ECPR>(E, reinterpret_cast<float*>(sA + BM * PITCH), s8, q8, r8, c, lane, wave, tid,
                                          n0, N, t);
    else
      __syncthreads();  // staging reads done before the next tile overwrites the halo
  }
}

template <int C, int BN, int TH, int W, int PRO, bool FLIP, int WM>
hipError_t launch(const Pro& pa, const bf16_t* w, const EpiParams& E, int Nimg, int H, int N, hipStream_t st) {
  const int nsl = N / BN;
  const int tiles = Nimg * (H / TH);
  int per_xcd = big::device_cus() / (8 * nsl);  // one persistent workgroup per (free) CU in all
  if (per_xcd < 1) per_xcd = 1;
  const int need = ceil_div(tiles, 8);
  if (per_xcd > need) per_xcd = need;
  hipLaunchKernelGGL((conv3_kernel<C, BN, TH, W, PRO, FLIP, WM>), dim3(8 * nsl * per_xcd), dim3(THR), 0, st, pa, w, E, H, N,
                     tiles, nsl);
  return hipGetLastError();
}

// the shapes compiled in: (C, N, W, prologue) -> TH. The BN-backward prologue holds two
// prefetched halos (gradient + BN input) in registers, so it takes 4-row tiles (8 waves as
// 2 x 4): the 8-row configuration spilled them to scratch.
inline int pick_th(int C, int N, int W, int pro) {
  if (C == 64 && N == 64 && W == 56) return pro == 2 ? 4 : 8;
  return 0;
}

template <int PRO, bool FLIP>
hipError_t dispatch(const Pro& pa, const bf16_t* w, const EpiParams& E, int Nimg, int H, int W, int C, int N,
                    hipStream_t st) {
  if (C == 64 && N == 64 && W == 56) {
    if constexpr (PRO == 2) return launch<64, 64, 4, 56, PRO, FLIP, 2>(pa, w, E, Nimg, H, N, st);
    else return launch<64, 64, 8, 56, PRO, FLIP, 4>(pa, w, E, Nimg, H, N, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace c3

// ------------------------------------------------------------------------------------------
// Streamed-filter variant for the 28 x 28, 128 -> 128 convs (ResNet-50 stage-3 c2, forward and
// data gradient). Why: the implicit-GEMM engine runs them at ~530 TF/s, bound by L2 -> CU traffic
// (every 256 x 128 output tile re-gathers 256 x 1152 operand bytes: ~3.5 KB per output row), and
// the 56 x 56 kernel above cannot keep this filter resident (128 x 1152 bf16 = 288 KiB).
// Here one persistent workgroup per CU walks tiles of TR = 8 consecutive image rows of the
// flattened (image, row) sequence (224 output pixels, contiguous in NHWC; a tile may span two
// images: the halo then holds two row segments, each with its own zero-padded border rows), keeps
// the tile's (TR + 4) x 30 x 128 halo in LDS (channel-chunk-major, as above; PRO 1 applies the
// producing BN + ReLU on the way and writes the interior back once), and streams the filter one
// tap (128 x 128 bf16 = 32 KiB) at a time through two LDS buffers by LDS-DMA: tap t + 1 lands
// under tap t's 56 MFMAs per wave. L2 traffic per output row: ~1.7 KB (halo once, filter once
// per 224 rows). The next tile's halo is prefetched into registers under this tile's epilogue.
namespace c3s {

constexpr int THR = 512;
constexpr int NW = THR / 64;

// LDS-DMA of one 16-B piece per lane into a wave-uniform LDS base (lane l lands at base + 16 l).
// Inline asm: hipcc does not count it in its vmcnt bookkeeping (its own waits only get stronger);
// the kernel retires these pieces with explicit counted waits.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  typedef __attribute__((address_space(3))) const char lds_char_t;
  return (uint32_t)(size_t)(lds_char_t*)(p);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int C, int BN, int TR, int H, int W, int PRO, bool FLIP>
__global__ __launch_bounds__(THR, 1) void conv3s_kernel(c3::Pro pa, const bf16_t* __restrict__ w, EpiParams E,
                                                       int rows_total, int N, int tiles) {
  constexpr int WM = 2, WN = NW / WM;
  constexpr int BM = TR * W;                 // output pixels per tile
  constexpr int WR = BM / WM, WC = BN / WN;  // rows / cols per wave
  constexpr int TM = WR / 16, TN = WC / 16;
  constexpr int HS = TR + 4;                 // halo row slots: two segments with two border rows each
  constexpr int HC = W + 2;
  constexpr int NPIX = HS * HC;
  constexpr int CP = C / 8;
  constexpr int NCH = ((NPIX + 7) / 8) * 8 * CP;  // staging slots (8-pixel groups)
  constexpr int NA = (NCH + THR - 1) / THR;       // per thread (every thread issues NA loads)
  constexpr int REG = ((NPIX * 16 + 255) / 256) * 256;
  constexpr int SH = CP * REG;
  constexpr int SBT = BN * C * 2;            // one tap of the filter
  constexpr int PITCH = BN * 2 + 16;
  constexpr int SE = BM * PITCH + NW * 3 * BN * 4;
  constexpr int SAE = SH > SE ? SH : SE;
  constexpr int NDMA = SBT / 16 / THR;       // DMA pieces per thread per tap
  static_assert(PRO != 2 && C % 64 == 0 && BN % (16 * WN) == 0 && WR % 16 == 0 && TR <= H, "tile shape");
  static_assert(THR % (8 * CP) == 0 && SBT % (16 * THR) == 0, "staging / DMA mapping");
  static_assert(SAE + 2 * SBT <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[SAE + 2 * SBT];
  char* const sA = smem;
  char* const sBb = smem + SAE;

  const int b = blockIdx.x;
  const int G = gridDim.x;
  // consecutive tiles (sharing halo rows) on one XCD
  const int g = (b & 7) * (G / 8) + (b >> 3);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ac = c3::slot_chunk<CP>(tid);
  const bool write_side = pa.side != nullptr;
  const int nimg = rows_total / H;

  // one filter tap into buffer `buf` (K-major [BN][C], kmaj_off layout in 64-k sub-tiles: linear
  // LDS chunk L holds logical chunk (L % 8) ^ swz(row) of its row)
  auto dma_tap = [&](int tap, int buf) {
    const int stap = FLIP ? 8 - tap : tap;
    char* dst = sBb + buf * SBT;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int L = (i * NW + wave) * 64 + lane;
      const int sub = L / (BN * 8), p = L % (BN * 8), row = p >> 3, j = p & 7;
      const int sc = j ^ ((row >> 1) & 7);
      dma16(w + (static_cast<long long>(row) * 9 + stap) * C + (sub * 8 + sc) * 8,
            lds_addr(dst + (i * NW + wave) * 1024));
    }
  };
  // tile geometry: rows [R0, R0 + n0) of image i0 (from local row h0), then n1 rows of i0 + 1
  struct Geo {
    int i0, h0, n0, n1;
  };
  auto geo = [&](int t) {
    Geo q;
    const int R0 = t * TR, R1 = min(R0 + TR, rows_total);
    q.i0 = R0 / H;
    q.h0 = R0 - q.i0 * H;
    q.n0 = min(R1, (q.i0 + 1) * H) - R0;
    q.n1 = R1 - R0 - q.n0;
    return q;
  };
  // halo slot s -> (image, row, interior); valid = false for slots no segment uses
  auto slot_src = [&](const Geo& q, int s, int& img, int& h, bool& interior) {
    if (s < q.n0 + 2) {
      img = q.i0;
      h = q.h0 - 1 + s;
      interior = s >= 1 && s <= q.n0;
      return true;
    }
    const int u = s - (q.n0 + 2);
    img = q.i0 + 1;
    h = u - 1;
    interior = u >= 1 && u <= q.n1;
    return q.n1 > 0 && u < q.n1 + 2;
  };

  uint4 ra[NA];
  auto load_tile = [&](int t) {
    const Geo q = geo(t);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int qq = tid + THR * i;
      const int pix = c3::slot_pix<CP>(qq);
      const int s = pix / HC, x = pix % HC - 1;
      int img, h;
      bool interior;
      const bool ok = qq < NCH && slot_src(q, s, img, h, interior) && h >= 0 && h < H && x >= 0 && x < W;
      const long long off = ((static_cast<long long>(img) * H + h) * W + x) * C + ac * 8;
      // always one load per slot (the zero page otherwise): the counted waits below rely on it
      ra[i] = ldg16(ok ? pa.x + off : reinterpret_cast<const bf16_t*>(big::g_zero));
    }
  };
  auto stage_tile = [&](int t) {
    const Geo q = geo(t);
    float k0[8], k1[8];
    if constexpr (PRO == 1) {
      c3::load8f(pa.s + ac * 8, k0);
      c3::load8f(pa.b + ac * 8, k1);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int qq = tid + THR * i;
      if (qq >= NCH) break;
      const int pix = c3::slot_pix<CP>(qq);
      const int s = pix / HC, x = pix % HC - 1;
      int img, h;
      bool interior;
      const bool ok = slot_src(q, s, img, h, interior) && h >= 0 && h < H && x >= 0 && x < W;
      uint4 v = ok ? ra[i] : make_uint4(0, 0, 0, 0);
      if constexpr (PRO == 1) {  // = apply_kernel (batchnorm.hip) with ReLU
        const long long off = ((static_cast<long long>(img) * H + h) * W + x) * C + ac * 8;
        float f[8];
        unpack8(ra[i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = relu(f[j] * k0[j] + k1[j]);
        v = ok ? pack8(f) : make_uint4(0, 0, 0, 0);
        if (write_side && ok && interior) {
          *reinterpret_cast<uint4*>(pa.side + off) = v;
          if (pa.side_mask) {
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            uint32_t mb = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t hb = (wv[j >> 1] >> (16 * (j & 1))) & 0xffffu;
              mb |= ((hb & 0x7fffu) != 0 && !(hb & 0x8000u) ? 1u : 0u) << j;
            }
            pa.side_mask[off >> 3] = static_cast<uint8_t>(mb);
          }
        }
      }
      *reinterpret_cast<uint4*>(sA + ac * REG + pix * 16) = v;
    }
  };

  int bcur = 0;
  int t = g;
  if (t < tiles) {
    dma_tap(0, 0);
    load_tile(t);
  }
  for (; t < tiles; t += G) {
    const Geo q = geo(t);
    int abase[TM];  // lane's halo offset of tap (0, 0) for each MFMA row block (+ its k-chunk region)
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int i = wm * WR + a * 16 + (lane & 15);
      const int j = i / W, col = i % W;
      abase[a] = (lane >> 4) * REG + ((j + (j >= q.n0 ? 2 : 0)) * HC + col) * 16;
    }
    stage_tile(t);
    wait_vm<0>();  // this tile's tap 0 (and every earlier store) landed
    __syncthreads();
    const bool more = t + G < tiles;
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int c = 0; c < TN; ++c) acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int bnext = bcur ^ 1;
      if (tap < 8) dma_tap(tap + 1, bnext);
      else if (more) dma_tap(0, bnext);
      const char* sBc = sBb + bcur * SBT;
      const int tq = ((tap / 3) * HC + (tap % 3)) * 16;
#pragma unroll
      for (int kc = 0; kc < C / 32; ++kc) {
        const int kglob = kc * 32;
        const char* pB = sBc + (kglob >> 6) * (BN * 128);
        const int kchunk = ((kglob & 63) >> 3) + (lane >> 4);
        bf16x8_t af[TM], bfr[TN];
#pragma unroll
        for (int c = 0; c < TN; ++c) bfr[c] = lds_read_b128(pB + kmaj_off(wn * WC + c * 16 + (lane & 15), kchunk));
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = lds_read_b128(sA + abase[a] + kc * 4 * REG + tq);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int c = 0; c < TN; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[c], af[a], acc[a][c], 0, 0, 0);
      }
      wait_vm<0>();  // the next tap's DMA landed
      __syncthreads();
      bcur = bnext;
    }
    // (the last barrier above: every wave is done reading the halo) stage the tile over it
    sepi::stage_acc<TM, TN, WR, WC, PITCH>(sA, acc, wm, wn, lane, epi_alpha(E));
    // the next tile's halo into registers now that the accumulators are dead: it flies under this
    // tile's epilogue (prefetching it across the tap loop held 48 more VGPRs there and spilled)
    if (more) load_tile(t + G);
    __syncthreads();
    constexpr int ECPR = BN / 8;
    constexpr int RPP = THR / ECPR;
    const int m0 = t * BM;
    const int c = tid % ECPR, r0 = tid / ECPR;
    const int n = c * 8;
    const bool vst = (E.ldo & 7) == 0;
    float bias8[8], s8[8], q8[8], r8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bias8[j] = E.bias ? E.bias[n + j] : 0.f;
      s8[j] = q8[j] = r8[j] = 0.f;
    }
    const int M = rows_total * W;
    if (E.beta || E.residual || E.by)
      epi_rows<BM, RPP, PITCH, true, 2>(E, sA, c, r0, n, m0, M, N, vst, vst, bias8, s8, q8, r8);
    else
      epi_rows<BM, RPP, PITCH, false>(E, sA, c, r0, n, m0, M, N, vst, vst, bias8, s8, q8, r8);
    if (E.stat)
      sepi::tile_stats<BN, NW, THR, ECPR>(E, reinterpret_cast<float*>(sA + BM * PITCH), s8, q8, r8, c, lane, wave, tid,
                                          0, N, t);
    else
      __syncthreads();  // staging reads done before the next tile overwrites the halo
    (void)nimg;
  }
}

template <int PRO, bool FLIP>
hipError_t launch(const c3::Pro& pa, const bf16_t* w, const EpiParams& E, int Nimg, int N, hipStream_t st) {
  const int rows = Nimg * 28;
  const int tiles = ceil_div(rows, 8);
  int G = big::device_cus() / 8 * 8;  // one persistent workgroup per (free) CU, a multiple of 8
  if (G < 8) G = 8;
  const int need = ceil_div(tiles, 8) * 8;
  if (G > need) G = need;
  hipLaunchKernelGGL((conv3s_kernel<128, 128, 8, 28, 28, PRO, FLIP>), dim3(G), dim3(THR), 0, st, pa, w, E, rows, N,
                     tiles);
  return hipGetLastError();
}

inline bool fits(int H, int W, int C, int N, int pro) { return C == 128 && N == 128 && H == 28 && W == 28 && pro != 2; }

}  // namespace c3s
}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Output rows per tile (= BN partial-statistics row count divisor) of ttdk_conv3_halo for a
// [*, H, W, C] -> N 3x3/s1/p1 conv, or 0 when the shape is not compiled in.
namespace {
int& conv3_s3_flag() {
  static int on = getenv_int("TTD_CONV3_S3", 1);  // stage-3 streamed-filter variant (0: off)
  return on;
}
}  // namespace

// Runtime switch of the stage-3 streamed-filter variant; returns the previous setting.
TTDK_EXPORT int ttdk_set_conv3_s3(int on) {
  const int old = conv3_s3_flag();
  conv3_s3_flag() = on;
  return old;
}

TTDK_EXPORT int ttdk_conv3_rows(int H, int W, int C, int N, int pro) {
  if (conv3_s3_flag() && c3s::fits(H, W, C, N, pro)) return 8 * W;  // tiles of 8 rows of the flattened (image, row) sequence
  const int th = c3::pick_th(C, N, W, pro);
  return (th && H % th == 0) ? th * W : 0;
}

// out[Nimg, H, W, N] = epilogue( conv3x3_s1_p1( A'(x), w ) ), A' from the prologue:
//   pro 0: x; pro 1: relu(x*s + b); pro 2: s[0]*(x . mask) + s[1]*x2 + s[2] (s = coef[3][C]).
// flip = 0: w is the forward filter [N][3][3][C]; flip = 1: w is the transposed filter
// [N][3][3][C] of the conv whose data gradient this is (taps reversed here).
TTDK_EXPORT int ttdk_conv3_halo(const bf16_t* x, const bf16_t* x2, const uint8_t* mask_in, const float* s,
                                const float* b, bf16_t* side, uint8_t* side_mask, int pro, int flip, const bf16_t* w,
                                int Nimg, int H, int W, int C, int N, const TtdkEpilogue* epi, hipStream_t st) {
  if (ttdk_conv3_rows(H, W, C, N, pro) == 8 * W && c3s::fits(H, W, C, N, pro)) {
    if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15)) return hipErrorInvalidValue;
    const EpiParams e = to_epi(epi);
    if (e.mode != 0 || e.remap || e.bH || e.ldo != N || e.residual || e.by2) return hipErrorInvalidValue;
    if (pro == 1 && (!s || !b)) return hipErrorInvalidValue;
    if (side_mask && pro != 1) return hipErrorInvalidValue;
    const c3::Pro pa{x, nullptr, nullptr, s, b, side, side_mask};
    if (pro == 0 && !flip) return c3s::launch<0, false>(pa, w, e, Nimg, N, st);
    if (pro == 0 && flip) return c3s::launch<0, true>(pa, w, e, Nimg, N, st);
    if (pro == 1 && !flip) return c3s::launch<1, false>(pa, w, e, Nimg, N, st);
    return hipErrorInvalidValue;
  }
  const int th = c3::pick_th(C, N, W, pro);
  if (!th || H % th || (reinterpret_cast<uintptr_t>(x) & 15) || pro < 0 || pro > 2) return hipErrorInvalidValue;
  const EpiParams e = to_epi(epi);
  if (e.mode != 0 || e.remap || e.bH || e.ldo != N || e.residual || e.by2) return hipErrorInvalidValue;
  if (pro == 1 && (!s || !b)) return hipErrorInvalidValue;
  if (pro == 2 && (!s || !x2)) return hipErrorInvalidValue;
  if (side_mask && pro != 1) return hipErrorInvalidValue;
  const c3::Pro pa{x, x2, mask_in, s, b, side, side_mask};
#define C3_CASE(P_, F_) \
  if (pro == P_ && (flip != 0) == F_) return c3::dispatch<P_, F_>(pa, w, e, Nimg, H, W, C, N, st);
  C3_CASE(0, false)
  C3_CASE(1, false)
  C3_CASE(0, true)
  C3_CASE(2, true)
#undef C3_CASE
  return hipErrorInvalidValue;
}
