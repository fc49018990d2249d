// Forward of the ResNet stem convolution (7x7, stride 2, pad 3, 64 filters) over the RGB image
// (packed [N][H][W][3], or stored with 8 channels, 3..7 zero), with the per-workgroup BatchNorm
// statistics of the stored bf16 output:
//     y[n][p][q][k] = sum_{r,s,c<3} x[n][2p-3+r][2q-3+s][c] * w[k][r][s][c]
//
// Why (tools/op_timing.py, b1024): the implicit-GEMM conv ran this at 1.8 ms — its K of 7*7*8 =
// 392 spends 62 % of the MFMA work on the 5 zero channels, and it gathers the im2col rows
// through the operand loader. Here the reduction per filter row r is (s, c) with c < 4 and
// s < 8: 32 = one v_mfma_f32_16x16x32_bf16 K-step, so K = 7 x 32 = 224 (147 real) — and the A
// fragment of a lane (output pixel q, K chunk g = (s = 2g, 2g+1) x c 0..3) is 16 contiguous bytes
// of the staged input row (columns 2q-3+2g, 2q-2+2g, 4 channels each): no im2col is built at all.
//
// Design (MI355X-first): persistent workgroups of 8 waves walk bands of 8 output rows of
// their images (one output row of 112 pixels x 64 channels per wave: 7 x 4 x 7 = 196 MFMAs).
// The 21 input rows a band reads live in an LDS ring (input row h in slot h % 21, 4 channels,
// 3 zero columns each side), so each further band of the image adds 16 rows, prefetched into
// registers under the previous band's MFMAs. The filter is staged once per workgroup as
// [k][r][s][c4] rows and held as MFMA B fragments in registers (112 VGPRs) for the whole launch.
// A wave computes its row one 16-pixel block at a time (28 MFMAs) and stores that block right
// away (lane pairs swap halves: 16 pixels x 64 contiguous bytes per store), so the stores drain
// under the next block's MFMAs; BN sum / sum of squares accumulate per lane (packed fp32
// pairs) and are reduced once per workgroup into part[block][2][64].
#include "gemm_conv.h"

namespace ttdk {
namespace {
namespace stemf {

constexpr int THR = 512;
constexpr int NW = THR / 64;
constexpr int BAND = NW;               // output rows per band (one per wave)
constexpr int RING = 2 * BAND + 5;     // input rows a band reads
constexpr int NEWR = 2 * BAND;         // input rows each further band adds
constexpr int Q = 112, W = 224;        // output / input width (ResNet stem at 224 x 224)
constexpr int QB = Q / 16;             // 16-pixel MFMA blocks per output row
constexpr int XC = W + 6;              // staged columns: input columns -3 .. W+2
constexpr int XP = XC * 8;             // bytes per staged row (4 bf16 channels per column)
constexpr int KO = 64;
constexpr int WP = 7 * 64 + 16;        // bytes per staged filter row k: 7 taps x 32 bf16 (+16: odd slot pitch)
constexpr int NLD = (NEWR * W + THR - 1) / THR;  // prefetched pixels per thread per band (8-channel input)
constexpr int RC3 = W * 3 * 2 / 16;              // 16-B chunks per input row (3-channel input)
constexpr int NLD3 = (NEWR * RC3 + THR - 1) / THR;

__device__ __forceinline__ int ring_slot(int h) { return (h + 4 * RING) % RING; }

// CIN: channel stride of x — 8 (RGB padded with zeros, one 16-B load per pixel) or 3 (packed
// RGB, 16-B loads over the row, scattered into the ring as 2-B writes; no padding pass)
template <int CIN>
__global__ __launch_bounds__(THR, 1) void stem_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ y, float* __restrict__ part, int N,
                                                          int H, int P, int imgs_per_wg) {
  __shared__ __attribute__((aligned(16))) char xs[RING * XP];
  __shared__ __attribute__((aligned(16))) char ws[KO * WP];
  __shared__ float red[NW][2][KO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int n_begin = blockIdx.x * imgs_per_wg, n_end = min(N, n_begin + imgs_per_wg);

  // filter -> [k][r][s*4 + c] (s < 7, c < 3; the other K slots stay zero)
  for (int i = tid; i < KO * 7 * 32; i += THR) {
    const int k = i / (7 * 32), rem = i % (7 * 32), r = rem / 32, s = (rem % 32) / 4, c = rem % 4;
    const bf16_t v = (s < 7 && c < 3) ? w[((k * 7 + r) * 7 + s) * 8 + c] : static_cast<bf16_t>(0);
    *reinterpret_cast<bf16_t*>(ws + k * WP + (r * 32 + s * 4 + c) * 2) = v;
  }
  // the ring starts zero: the pad columns and (3-channel input) channel 3 are never written
  for (int i = tid; i < RING * XP / 16; i += THR) reinterpret_cast<uint4*>(xs)[i] = make_uint4(0, 0, 0, 0);

  __syncthreads();
  // the filter as MFMA B fragments, resident in registers for the whole launch (28 x 16 B)
  bf16x8_t bw[7][4];
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) bw[r][cb] = lds_read_b128(ws + (cb * 16 + i16) * WP + (r * 4 + g) * 16);

  // 8-channel input: pixel loads (channels 0..3 kept)
  auto xpix = [&](int n, int h, int col) -> uint2 {
    if (h < 0 || h >= H) return make_uint2(0, 0);
    const uint4 v = ldg16(x + ((static_cast<long long>(n) * H + h) * W + col) * 8);
    return make_uint2(v.x, v.y);
  };
  auto put = [&](int h, int col, uint2 v) { *reinterpret_cast<uint2*>(xs + ring_slot(h) * XP + (col + 3) * 8) = v; };
  // 3-channel input: 16-B chunk j of row h (elements 8j .. 8j+7 of its packed [W][3] values)
  auto xchunk = [&](int n, int h, int j) -> uint4 {
    if (h < 0 || h >= H) return make_uint4(0, 0, 0, 0);
    return ldg16(x + (static_cast<long long>(n) * H + h) * W * 3 + j * 8);
  };
  auto put3 = [&](int h, int j, uint4 v) {
    char* row = xs + ring_slot(h) * XP;
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int el = 8 * j + e, px = el / 3, ch = el - 3 * px;
      *reinterpret_cast<bf16_t*>(row + (px + 3) * 8 + ch * 2) = static_cast<bf16_t>((wd[e >> 1] >> (16 * (e & 1))) & 0xffff);
    }
  };

  // BN partial sums of this lane's channels cb*16 + 4g + 2h + {0,1}, as packed fp32 pairs
  // (v_pk_add_f32 / v_pk_fma_f32)
  typedef __attribute__((ext_vector_type(2))) float f32x2_t;
  f32x2_t st[4][2], sq[4][2];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int h = 0; h < 2; ++h) st[cb][h] = sq[cb][h] = f32x2_t{0.f, 0.f};

  const int bands = P / BAND;
  for (int n = n_begin; n < n_end; ++n) {
    // first band of the image: all of its input rows 2p0-3 .. 2p0+2*BAND+1 (p0 = 0)
    __syncthreads();
    if constexpr (CIN == 8) {
      for (int i = tid; i < RING * W; i += THR) {
        const int rr = i / W, col = i % W, h = rr - 3;
        put(h, col, xpix(n, h, col));
      }
    } else {
      for (int i = tid; i < RING * RC3; i += THR) {
        const int rr = i / RC3, j = i % RC3, h = rr - 3;
        put3(h, j, xchunk(n, h, j));
      }
    }
    __syncthreads();
    for (int band = 0; band < bands; ++band) {
      const int p0 = band * BAND;
      const bool pre = band + 1 < bands;
      // next band's new input rows 2p0+2*BAND+2 .. +NEWR-1 into registers (in flight under the MFMAs)
      constexpr int NPF = CIN == 8 ? NLD : NLD3;
      uint2 nx[CIN == 8 ? NLD : 1];
      uint4 nx3[CIN == 8 ? 1 : NLD3];
#pragma unroll
      for (int i = 0; i < NPF; ++i) {
        const int idx = tid + THR * i;
        if constexpr (CIN == 8) {
          const int rr = idx / W, col = idx % W;
          nx[i] = (pre && idx < NEWR * W) ? xpix(n, 2 * p0 + 2 * BAND + 2 + rr, col) : make_uint2(0, 0);
        } else {
          const int rr = idx / RC3, j = idx % RC3;
          nx3[i] = (pre && idx < NEWR * RC3) ? xchunk(n, 2 * p0 + 2 * BAND + 2 + rr, j) : make_uint4(0, 0, 0, 0);
        }
      }
      // wave: output row p = p0 + wave, one 16-pixel block at a time (7 taps x 4 channel blocks
      // of MFMAs, then that block's stores, which drain under the next block's MFMAs)
      const int p = p0 + wave;
      int roff[7];
#pragma unroll
      for (int r = 0; r < 7; ++r) roff[r] = ring_slot(2 * p - 3 + r) * XP + 2 * g * 8;
      bf16_t* yrow = y + (static_cast<long long>(n) * P + p) * Q * KO;
      const bool odd = g & 1;
#pragma unroll 1
      for (int pb = 0; pb < QB; ++pb) {
        const int q = pb * 16 + i16;
        f32x4_t acc[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 7; ++r) {
          // columns 2q-3+2g, 2q-2+2g = staged columns 2q+2g, 2q+2g+1
          const bf16x8_t afr = lds_read_b128(xs + roff[r] + 2 * q * 8);
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[r][cb], afr, acc[cb], 0, 0, 0);
        }
        // lane holds pixel q, channels cb*16 + 4g + v. Lane pairs (g, g^1) swap so the even lane
        // stores channels cb0*16 + 4g .. +7 and the odd lane those of cb0 + 1.
#pragma unroll
        for (int cp = 0; cp < 2; ++cp) {
          uint2 pk[2];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int cb = 2 * cp + h2;
            const f32x4_t v = acc[cb];
            pk[h2] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
            // statistics of the values actually stored (bf16-rounded)
            const f32x2_t v01 = {bf2f(static_cast<bf16_t>(pk[h2].x & 0xffff)), bf2f(static_cast<bf16_t>(pk[h2].x >> 16))};
            const f32x2_t v23 = {bf2f(static_cast<bf16_t>(pk[h2].y & 0xffff)), bf2f(static_cast<bf16_t>(pk[h2].y >> 16))};
            st[cb][0] += v01;
            st[cb][1] += v23;
            sq[cb][0] += v01 * v01;
            sq[cb][1] += v23 * v23;
          }
          const uint2 snd = odd ? pk[0] : pk[1];
          const uint2 rcv = make_uint2(__shfl_xor(snd.x, 16, 64), __shfl_xor(snd.y, 16, 64));
          const uint4 o = odd ? make_uint4(rcv.x, rcv.y, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, rcv.x, rcv.y);
          const int ch = odd ? (2 * cp + 1) * 16 + 4 * (g - 1) : 2 * cp * 16 + 4 * g;
          *reinterpret_cast<uint4*>(yrow + static_cast<long long>(q) * KO + ch) = o;
        }
      }
      __syncthreads();  // every wave done with the ring rows the prefetched ones replace
      if (pre) {
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
          const int idx = tid + THR * i;
          if constexpr (CIN == 8) {
            if (idx < NEWR * W) put(2 * p0 + 2 * BAND + 2 + idx / W, idx % W, nx[i]);
          } else {
            if (idx < NEWR * RC3) put3(2 * p0 + 2 * BAND + 2 + idx / RC3, idx % RC3, nx3[i]);
          }
        }
      }
      __syncthreads();
    }
  }
  // BN partial sums: over the 16 pixel lanes of each channel group, then over the waves
  float fs[4][4], fq[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fs[cb][j] = st[cb][j >> 1][j & 1];
      fq[cb][j] = sq[cb][j >> 1][j & 1];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        fs[cb][j] += __shfl_xor(fs[cb][j], o, 64);
        fq[cb][j] += __shfl_xor(fq[cb][j], o, 64);
      }
    }
  if (i16 == 0) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[wave][0][cb * 16 + 4 * g + j] = fs[cb][j];
        red[wave][1][cb * 16 + 4 * g + j] = fq[cb][j];
      }
  }
  __syncthreads();
  if (tid < 2 * KO) {
    const int which = tid / KO, c = tid % KO;
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) s += red[v][which][c];
    part[(static_cast<long long>(blockIdx.x) * 2 + which) * KO + c] = s;
  }
}

}  // namespace stemf
}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Workgroups (= BN partial-sum rows) of ttdk_stem_fwd for a batch of N images.
TTDK_EXPORT int ttdk_stem_fwd_blocks(int N) {
  const int per = (N + 255) / 256;
  return (N + per - 1) / per;
}

// x [N][224][224][cin] bf16 (cin = 3, or 8 with channels 3..7 zero), w [64][7][7][8] bf16 ->
// y [N][112][112][64] bf16, part [blocks][2][64] fp32 (per-workgroup sum / sum of squares of y).
TTDK_EXPORT int ttdk_stem_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, float* part, int N, int H, int Wd, int cin,
                              hipStream_t st) {
  if (cin != 3 && cin != 8) return hipErrorInvalidValue;
  if (N <= 0 || H != stemf::W || Wd != stemf::W) return hipErrorInvalidValue;
  const int P = (H + 6 - 7) / 2 + 1;
  if (P % stemf::BAND != 0) return hipErrorInvalidValue;
  const int G = ttdk_stem_fwd_blocks(N);
  const int per = (N + G - 1) / G;
  if (cin == 3)
    hipLaunchKernelGGL(stemf::stem_fwd_kernel<3>, dim3(G), dim3(stemf::THR), 0, st, x, w, y, part, N, H, P, per);
  else
    hipLaunchKernelGGL(stemf::stem_fwd_kernel<8>, dim3(G), dim3(stemf::THR), 0, st, x, w, y, part, N, H, P, per);
  return hipGetLastError();
}
