// Weight gradient of the ResNet stem (7x7 stride-2 pad-3 conv over the RGB image stored with 8
// channels) with the stem BatchNorm's backward applied on the fly:
//     dW[k][r][s][c] = sum_{n,p,q} dz[n,p,q,k] * x[n, 2p-3+r, 2q-3+s, c],
//     dz = coef[0][k]*g + coef[1][k]*y + coef[2][k]           (c < 3; the padded channels get 0)
//
// Why (tools/op_timing.py): the generic im2col-gather GEMM ran this at 2.4 ms/step at batch
// 1024 — it computes all 8 stored channels (5 of them zero padding, 62 % of its MFMA work),
// its 392-wide column space leaves a 128-wide tile almost empty, and it is the last kernel of
// the backward pass with nothing to overlap.
//
// Design (MI355X-first): persistent workgroups (4 waves, 3 per CU) walk bands of 8 half output
// rows (56 pixels) of the 112x112 stem output. The row loop keeps its addressing in registers
// (formed once per thread: coefficients, dz^T destinations, im2col source offsets). The 7 input rows a half row touches live in an
// LDS ring, so each further output row of the band loads only its 2 new input rows (prefetched
// into registers with the row's g / y one row ahead); the 56x64 dz block is formed from g and y in registers and stored
// channel-major (the MFMA A operand, k = pixel), and the 147 real im2col columns (r, s, c<3)
// are built channel-major from the staged rows (the B operand); 2 k-steps x 10 column blocks
// of v_mfma_f32_16x16x32_bf16 per wave accumulate a 64 x 160 partial in registers across all
// of the workgroup's rows. Partials go to a [workgroups][64][160] slab that a deterministic
// split-K fold reduces, and a scatter writes dW in the [K][7][7][8] filter layout.
#include "gemm_conv.h"

namespace ttdk {
namespace {
namespace stem {

constexpr int THR = 256;
constexpr int QB = 56;            // output pixels per work item (half of a 112-pixel row)
constexpr int KP = 64;            // k (pixels) padded to the MFMA step
constexpr int XW = 2 * QB + 5;    // staged input columns per row
constexpr int NC = 160;           // im2col columns: 7*7*3 = 147, padded to 10 MFMA blocks
constexpr int KO = 64;            // output channels

constexpr int BAND = 8;          // output rows per work unit (a ring of input rows is kept across them)
constexpr int RING = 8;          // input-row slots (7 in use)

// CIN: channel stride of x (8: RGB padded with zeros, one 16-B load per pixel; 3: packed RGB,
// three 2-B loads per pixel, no padding pass)
template <int CIN>
__global__ __launch_bounds__(THR, 3) void stem_wgrad_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
                                                            const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                                            float* __restrict__ ws, int N, int H, int W, int P, int Q,
                                                            int units) {
  static_assert((RING & (RING - 1)) == 0 && QB % 8 == 0 && (NC * (KP / 8)) % THR == 0, "stem tiling");
  __shared__ __attribute__((aligned(16))) char xs[RING * XW * 16];  // input rows h % RING: [col][8 ch] bf16
  __shared__ __attribute__((aligned(16))) char sA[KO * 128];        // dz^T: [k_out][64 pixels] (kmaj)
  __shared__ __attribute__((aligned(16))) char sB[NC * 128];        // im2col^T: [col][64 pixels] (kmaj)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int halves = (Q + QB - 1) / QB;
  const int bands = (P + BAND - 1) / BAND;
  // Everything that does not change from row to row is formed once per thread: the loop body is
  // VALU-bound otherwise (the im2col index divisions and the per-element coefficient reads cost
  // more than the row's 20 MFMAs per wave).
  // dz^T: thread = (8-channel chunk cc, pixel pair pj); 28 pairs x 8 chunks = 224 threads, each
  // writing 8 packed bf16 pairs (channel k: pixels 2pj, 2pj+1)
  const int cc = tid & 7, pj = tid >> 3;
  const bool dz_on = pj < QB / 2;
  // the BN coefficients stay in LDS (registers spilled): six 16-B reads per row
  __shared__ __attribute__((aligned(16))) float cf[3 * KO];
  for (int i = tid; i < 3 * KO; i += THR) cf[i] = coef[i];
  // dz^T destination of channel cc*8+t: kmaj_off(cc*8+t, pj/4) + (2pj % 8)*2 = da0 + 128t + swizzle
  const int da0 = cc * 1024 + ((2 * pj) & 7) * 2, dchunk = (2 * pj) >> 3, dsw = (cc & 1) << 2;
  for (int c = tid; c < KO; c += THR)  // the padded pixel chunk (k = 56..63) of every dz^T row stays zero
    *reinterpret_cast<uint4*>(sA + kmaj_off(c, QB / 8)) = make_uint4(0, 0, 0, 0);
  // im2col^T items: c = tid + THR*m -> pixel chunk kc = c / NC, column col = c % NC = (r, s, ch);
  // columns >= 147 and the padded pixel chunk are zero for good (written once here)
  constexpr int NI = NC * (KP / 8) / THR;
  int ib[NI], id[NI];  // ib: source byte offset | r << 16 (-1: dead item)
#pragma unroll
  for (int m = 0; m < NI; ++m) {
    const int c = tid + THR * m, kc = c / NC, col = c % NC;
    id[m] = kmaj_off(col, kc);
    if (col < 147 && kc < QB / 8) {
      const int r = col / 21, rem = col % 21, sx = rem / 3, ch = rem % 3;
      ib[m] = ((sx * 8 + ch) * 2 + 256 * kc) | (r << 16);  // bytes: pixel column 2j+s of j = 8kc (+2t, +1 below)
    } else {
      ib[m] = -1;
      *reinterpret_cast<uint4*>(sB + id[m]) = make_uint4(0, 0, 0, 0);
    }
  }
  f32x4_t acc[NC / 16];
#pragma unroll
  for (int b = 0; b < NC / 16; ++b) acc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // cf is read before the row loop's first barrier

  // one input row (XW 16-B pixels starting at column 2*q0-3, zero outside the image)
  auto load_xpix = [&](int n, int h, int q0, int t) -> uint4 {
    const int w = 2 * q0 - 3 + t;
    if (!(h >= 0 && h < H && w >= 0 && w < W)) return make_uint4(0, 0, 0, 0);
    const bf16_t* px = x + ((static_cast<long long>(n) * H + h) * W + w) * CIN;
    if constexpr (CIN == 8) return ldg16(px);
    return make_uint4(static_cast<uint32_t>(px[0]) | (static_cast<uint32_t>(px[1]) << 16), px[2], 0, 0);
  };
  // per output row: the thread's g / y pixel pair and the two input rows that row adds to the
  // ring, prefetched into registers one row ahead
  constexpr int NX2 = (2 * XW + THR - 1) / THR;
  uint4 pg[2], py[2], px[NX2];
  auto prefetch = [&](int n, int p, int q0) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 2 * pj + e;
      const bool ok = dz_on && q0 + j < Q;
      const long long off = ((static_cast<long long>(n) * P + p) * Q + q0 + j) * KO + cc * 8;
      pg[e] = ok ? ldg16(g + off) : make_uint4(0, 0, 0, 0);
      py[e] = ok ? ldg16(y + off) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NX2; ++i) {
      const int c = tid + THR * i;
      const int rr = c / XW, t = c % XW;
      px[i] = c < 2 * XW ? load_xpix(n, 2 * p + 2 + rr, q0, t) : make_uint4(0, 0, 0, 0);  // rows 2p+2, 2p+3
    }
  };

  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int half = u % halves, band = (u / halves) % bands, n = u / (halves * bands);
    const int q0 = half * QB, p0 = band * BAND, p1 = min(P, p0 + BAND);
    // first output row of the band: input rows 2p0-3 .. 2p0+1 directly (the last two come with
    // the row's prefetch like every later row's two new rows)
    for (int c = tid; c < 5 * XW; c += THR) {
      const int rr = c / XW, t = c % XW;
      const int h = 2 * p0 - 3 + rr;
      *reinterpret_cast<uint4*>(xs + ((h & (RING - 1)) * XW + t) * 16) = load_xpix(n, h, q0, t);
    }
    prefetch(n, p0, q0);
    for (int p = p0; p < p1; ++p) {
      // 1. stage: the row's two new input rows, dz^T (BN backward applied on the way)
#pragma unroll
      for (int i = 0; i < NX2; ++i) {
        const int c = tid + THR * i;
        if (c < 2 * XW) {
          const int rr = c / XW, t = c % XW;
          *reinterpret_cast<uint4*>(xs + (((2 * p + 2 + rr) & (RING - 1)) * XW + t) * 16) = px[i];
        }
      }
      if (dz_on) {
        float g0[8], y0[8], g1[8], y1[8], c0[8], c1[8], c2[8];
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          *reinterpret_cast<f32x4_t*>(c0 + j) = *reinterpret_cast<const f32x4_t*>(cf + cc * 8 + j);
          *reinterpret_cast<f32x4_t*>(c1 + j) = *reinterpret_cast<const f32x4_t*>(cf + KO + cc * 8 + j);
          *reinterpret_cast<f32x4_t*>(c2 + j) = *reinterpret_cast<const f32x4_t*>(cf + 2 * KO + cc * 8 + j);
        }
        unpack8(pg[0], g0);
        unpack8(py[0], y0);
        unpack8(pg[1], g1);
        unpack8(py[1], y1);
#pragma unroll
        for (int t = 0; t < 8; ++t)
          *reinterpret_cast<uint32_t*>(sA + da0 + 128 * t + ((dchunk ^ (dsw + (t >> 1))) << 4)) =
              pack_bf16x2(c0[t] * g0[t] + c1[t] * y0[t] + c2[t], c0[t] * g1[t] + c1[t] * y1[t] + c2[t]);
      }
      __syncthreads();
      if (p + 1 < p1) prefetch(n, p + 1, q0);  // in flight under this row's im2col build and MFMAs
      // 2. im2col^T: column (r, s, c<3) -> B[col][j] = input row 2p-3+r, column 2j+s (relative), channel c
#pragma unroll
      for (int m = 0; m < NI; ++m) {
        if (ib[m] < 0) continue;
        const char* src = xs + ((2 * p - 3 + (ib[m] >> 16)) & (RING - 1)) * (XW * 16) + (ib[m] & 0xffff);
        uint32_t w4[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t lo = *reinterpret_cast<const bf16_t*>(src + 64 * t);
          const uint32_t hi = *reinterpret_cast<const bf16_t*>(src + 64 * t + 32);
          w4[t] = lo | (hi << 16);
        }
        *reinterpret_cast<uint4*>(sB + id[m]) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      __syncthreads();
      // 3. wave w: output channels 16w..16w+15 x all 160 columns, K = 64 pixels
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t a = lds_read_b128(sA + kmaj_off(wave * 16 + (lane & 15), ks * 4 + (lane >> 4)));
#pragma unroll
        for (int b = 0; b < NC / 16; ++b) {
          const bf16x8_t bb = lds_read_b128(sB + kmaj_off(b * 16 + (lane & 15), ks * 4 + (lane >> 4)));
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[b], 0, 0, 0);
        }
      }
      __syncthreads();
    }
  }
  // D[i][j]: i = output channel (A rows), j = column; lane holds rows 4*(lane>>4)+v, column lane&15
  float* o = ws + static_cast<long long>(blockIdx.x) * KO * NC;
#pragma unroll
  for (int b = 0; b < NC / 16; ++b)
#pragma unroll
    for (int v = 0; v < 4; ++v) o[(wave * 16 + 4 * (lane >> 4) + v) * NC + b * 16 + (lane & 15)] = acc[b][v];
}

// dW[k][r][s][c] (fp32, filter layout [64][7][7][8]) from the folded [64][160] sums
__global__ void stem_scatter_kernel(const float* __restrict__ sums, float* __restrict__ dw, int beta) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= KO * 49 * 8) return;
  const int c = i % 8, rs = (i / 8) % 49, k = i / (8 * 49);
  const float v = c < 3 ? sums[k * NC + (rs / 7) * 21 + (rs % 7) * 3 + c] : 0.f;
  dw[i] = v + (beta ? dw[i] : 0.f);
}

}  // namespace stem
}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Workgroups of ttdk_stem_wgrad (the caller's workspace holds workgroups*64*160 + 64*160 floats).
TTDK_EXPORT int ttdk_stem_wgrad_blocks(int N, int P, int Q) {
  const long long units = static_cast<long long>(N) * ((P + stem::BAND - 1) / stem::BAND) * ((Q + stem::QB - 1) / stem::QB);
  const int want = 3 * 256;
  return static_cast<int>(units < want ? units : want);
}

// x [N][H][W][cin] (cin = 3, or 8 with 3 real channels), g / y [N][P][Q][64], coef [3][64] -> dw [64][7][7][8] fp32.
TTDK_EXPORT int ttdk_stem_wgrad(const bf16_t* x, const bf16_t* g, const bf16_t* y, const float* coef, float* dw,
                                float* ws, int N, int H, int W, int P, int Q, int beta, int cin, hipStream_t st) {
  if (cin != 3 && cin != 8) return hipErrorInvalidValue;
  if (P != (H + 6 - 7) / 2 + 1 || Q != (W + 6 - 7) / 2 + 1 || N <= 0) return hipErrorInvalidValue;
  const int units = N * ((P + stem::BAND - 1) / stem::BAND) * ((Q + stem::QB - 1) / stem::QB);
  const int G = ttdk_stem_wgrad_blocks(N, P, Q);
  if (cin == 3)
    hipLaunchKernelGGL(stem::stem_wgrad_kernel<3>, dim3(G), dim3(stem::THR), 0, st, x, g, y, coef, ws, N, H, W, P, Q, units);
  else
    hipLaunchKernelGGL(stem::stem_wgrad_kernel<8>, dim3(G), dim3(stem::THR), 0, st, x, g, y, coef, ws, N, H, W, P, Q, units);
  float* sums = ws + static_cast<long long>(G) * stem::KO * stem::NC;
  hipError_t e = splitk_reduce(ws, G, static_cast<long long>(stem::KO) * stem::NC, sums, 0, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(stem::stem_scatter_kernel, dim3((stem::KO * 49 * 8 + 255) / 256), dim3(256), 0, st, sums, dw, beta);
  return hipGetLastError();
}
