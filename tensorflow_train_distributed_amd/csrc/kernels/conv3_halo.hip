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
}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Output rows per tile (= BN partial-statistics row count divisor) of ttdk_conv3_halo for a
// [*, H, W, C] -> N 3x3/s1/p1 conv, or 0 when the shape is not compiled in.
TTDK_EXPORT int ttdk_conv3_rows(int H, int W, int C, int N, int pro) {
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
