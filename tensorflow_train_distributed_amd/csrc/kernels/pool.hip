// Pooling on NHWC bf16: MaxPool (forward records the window argmax as one byte, backward
// is a gather — no atomics) and global average pooling (ResNet-50 stem / head).
#include "common.h"

namespace ttdk {
namespace {

// One thread per (n, p, q, 8-channel group).
__global__ void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                   int N, int H, int W, int C, int P, int Q, int R, int S, int sh, int sw, int ph,
                                   int pw) {
  const int cg = C >> 3;
  const long long total = static_cast<long long>(N) * P * Q * cg;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(i % cg);
    long long t = i / cg;
    const int q = static_cast<int>(t % Q);
    t /= Q;
    const int p = static_cast<int>(t % P);
    const int n = static_cast<int>(t / P);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    for (int r = 0; r < R; ++r) {
      const int h = p * sh - ph + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < S; ++s) {
        const int w = q * sw - pw + s;
        if (w < 0 || w >= W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + ((static_cast<long long>(n) * H + h) * W + w) * C + c8 * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > best[j] || (f[j] != f[j])) {  // NaN propagates
            best[j] = f[j];
            bi[j] = r * S + s;
          }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    if (arg) {
      uint2 a;
      a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      reinterpret_cast<uint2*>(arg)[i] = a;
    }
  }
}

// dx[n,h,w,c] = sum over windows (p,q) containing (h,w) whose argmax is (h,w) of dy[n,p,q,c].
__global__ void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                   bf16_t* __restrict__ dx, int N, int H, int W, int C, int P, int Q, int R, int S,
                                   int sh, int sw, int ph, int pw) {
  const int cg = C >> 3;
  const long long total = static_cast<long long>(N) * H * W * cg;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(i % cg);
    long long t = i / cg;
    const int w = static_cast<int>(t % W);
    t /= W;
    const int h = static_cast<int>(t % H);
    const int n = static_cast<int>(t / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows p with p*sh - ph <= h <= p*sh - ph + R - 1
    const int p_lo = max(0, (h + ph - R + sh) / sh), p_hi = min(P - 1, (h + ph) / sh);
    const int q_lo = max(0, (w + pw - S + sw) / sw), q_hi = min(Q - 1, (w + pw) / sw);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * sh - ph);
      if (r < 0 || r >= R) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * sw - pw);
        if (s < 0 || s >= S) continue;
        const long long o = ((static_cast<long long>(n) * P + p) * Q + q) * cg + c8;
        const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
        float g[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], g);
        const int me = r * S + s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t word = j < 4 ? a.x : a.y;
          if (static_cast<int>((word >> (8 * (j & 3))) & 0xff) == me) acc[j] += g[j];
        }
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
  }
}

// y[n,c] = mean over HW of x[n,h,w,c]; one block per (n, 256*8-channel chunk).
__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, float* __restrict__ yf,
                                   int HW, int C) {
  const int n = blockIdx.y;
  const int c8 = blockIdx.x * blockDim.x + threadIdx.x;
  if (c8 * 8 >= C) return;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16_t* p = x + static_cast<long long>(n) * HW * C + c8 * 8;
  for (int i = 0; i < HW; ++i) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(p + static_cast<long long>(i) * C), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += f[j];
  }
  const float inv = 1.f / HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] *= inv;
  if (y) *reinterpret_cast<uint4*>(y + static_cast<long long>(n) * C + c8 * 8) = pack8(s);
  if (yf)
#pragma unroll
    for (int j = 0; j < 8; ++j) yf[static_cast<long long>(n) * C + c8 * 8 + j] = s[j];
}

// dx[n,h,w,c] = dy[n,c] / HW
__global__ void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, long long total8, int HW,
                                   int C) {
  const int cg = C >> 3;
  const float inv = 1.f / HW;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total8;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(i % cg);
    const long long n = i / cg / HW;
    float g[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + n * C + c8 * 8), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= inv;
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
}


// ---- ResNet stem fusions (3x3 / stride 2 / pad 1 max pooling of a BN+ReLU output, H = 2P, W = 2Q)
// Window (p, q) covers input rows 2p-1..2p+1 and OWNS rows {2p, 2p+1} x cols {2q, 2q+1}: the
// owned 2x2 block partitions the input, so per-input-element work (ReLU mask bits, gradient
// stores, BN statistics) happens exactly once with no atomics.

// Forward: pooled = maxpool(relu(y*scale + shift)) (the BN+ReLU output is never stored: the
// pooling kernel reads y directly), window argmax (byte per element) and the ReLU bit mask of
// the (bf16-rounded) activation for the backward. Thread per (n, p, q, 8-channel group).
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(const bf16_t* __restrict__ y,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              bf16_t* __restrict__ out, uint8_t* __restrict__ arg,
                                                              uint8_t* __restrict__ mask, int N, int H, int W, int C,
                                                              int P, int Q) {
  const int cg = C >> 3;
  const int total = N * P * Q * cg;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % cg;
    int t = i / cg;
    const int q = t % Q;
    t /= Q;
    const int p = t % P;
    const int n = t / P;
    float sc[8], sh[8];
    {
      const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(scale + c8 * 8);
      const f32x4_t s1 = *reinterpret_cast<const f32x4_t*>(scale + c8 * 8 + 4);
      const f32x4_t h0 = *reinterpret_cast<const f32x4_t*>(shift + c8 * 8);
      const f32x4_t h1 = *reinterpret_cast<const f32x4_t*>(shift + c8 * 8 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sc[j] = s0[j];
        sc[4 + j] = s1[j];
        sh[j] = h0[j];
        sh[4 + j] = h1[j];
      }
    }
    uint4 v[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int h = 2 * p - 1 + r, w = 2 * q - 1 + s;
        v[r][s] = (h >= 0 && w >= 0)
                      ? *reinterpret_cast<const uint4*>(y + ((static_cast<long long>(n) * H + h) * W + w) * C + c8 * 8)
                      : make_uint4(0, 0, 0, 0);
      }
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    uint32_t mbits[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int h = 2 * p - 1 + r, w = 2 * q - 1 + s;
        if (h < 0 || w < 0) continue;
        float f[8];
        unpack8(v[r][s], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = relu(f[j] * sc[j] + sh[j]);
        const uint4 pk = pack8(f);  // the bf16 activation the unfused path would have stored
        float o[8];
        unpack8(pk, o);
        uint32_t mb = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          mb |= (o[j] > 0.f ? 1u : 0u) << j;
          if (o[j] > best[j] || (o[j] != o[j])) {
            best[j] = o[j];
            bi[j] = r * 3 + s;
          }
        }
        if (r >= 1 && s >= 1) mbits[r - 1][s - 1] = mb;
      }
    reinterpret_cast<uint4*>(out)[i] = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    reinterpret_cast<uint2*>(arg)[i] = a;
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
        mask[((static_cast<long long>(n) * H + 2 * p + a2) * W + 2 * q + b2) * cg + c8] =
            static_cast<uint8_t>(mbits[a2][b2]);
  }
}

// Backward: g = maxpool_bwd(dpooled) * relu_mask for the owned 2x2 input block of window
// (i, j) (contributions from windows {i, i+1} x {j, j+1}), stored as the BN-backward input,
// plus the per-block BN partial sums (sum g, sum g*y). grid-stride over (n, i, j, c8) with the
// channel group fixed per thread (256 % (C/8) == 0): partial[blockIdx.x][2][C].
__global__ __launch_bounds__(256) void maxpool_bwd_bnstat_kernel(const bf16_t* __restrict__ dy,
                                                                 const uint8_t* __restrict__ arg,
                                                                 const uint8_t* __restrict__ mask,
                                                                 const bf16_t* __restrict__ y, bf16_t* __restrict__ g,
                                                                 float* __restrict__ partial, int N, int H, int W,
                                                                 int C, int P, int Q) {
  __shared__ float red[2][256][8];
  const int cg = C >> 3;
  const int c8 = threadIdx.x % cg;
  const int lanes = 256 / cg;  // threads per block sharing one channel group
  const int blocks = N * P * Q;  // owned 2x2 blocks per channel group
  float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b = blockIdx.x * lanes + threadIdx.x / cg; b < blocks; b += gridDim.x * lanes) {
    const int j = b % Q;
    const int t = b / Q;
    const int i = t % P;
    const int n = t / P;
    float acc[2][2][8];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[a2][b2][k] = 0.f;
#pragma unroll
    for (int dp = 0; dp < 2; ++dp)
#pragma unroll
      for (int dq = 0; dq < 2; ++dq) {
        const int pp = i + dp, qq = j + dq;
        if (pp >= P || qq >= Q) continue;
        const long long o = ((static_cast<long long>(n) * P + pp) * Q + qq) * cg + c8;
        const uint2 av = reinterpret_cast<const uint2*>(arg)[o];
        float gv[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], gv);
        // window (pp, qq) tap (r, s) -> input (2pp-1+r, 2qq-1+s); owned pixel (2i+a2, 2j+b2) has
        // r = 2(i-pp) + 1 + a2, s = 2(j-qq) + 1 + b2
#pragma unroll
        for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
          for (int b2 = 0; b2 < 2; ++b2) {
            const int r = 1 + a2 - 2 * dp, s = 1 + b2 - 2 * dq;
            if (r < 0 || s < 0) continue;
            const int me = r * 3 + s;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const uint32_t word = k < 4 ? av.x : av.y;
              if (static_cast<int>((word >> (8 * (k & 3))) & 0xff) == me) acc[a2][b2][k] += gv[k];
            }
          }
      }
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2) {
        const long long pix = (static_cast<long long>(n) * H + 2 * i + a2) * W + 2 * j + b2;
        const uint32_t mb = mask[pix * cg + c8];
        float yv[8];
        unpack8(*reinterpret_cast<const uint4*>(y + pix * C + c8 * 8), yv);
        float gg[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) gg[k] = (mb >> k) & 1u ? acc[a2][b2][k] : 0.f;
        const uint4 pk = pack8(gg);
        *reinterpret_cast<uint4*>(g + pix * C + c8 * 8) = pk;
        float gs[8];
        unpack8(pk, gs);  // statistics of the stored gradient
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s8[k] += gs[k];
          q8[k] += gs[k] * yv[k];
        }
      }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = s8[k];
    red[1][threadIdx.x][k] = q8[k];
  }
  __syncthreads();
  if (threadIdx.x < cg) {
    for (int l = 1; l < lanes; ++l)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s8[k] += red[0][threadIdx.x + l * cg][k];
        q8[k] += red[1][threadIdx.x + l * cg][k];
      }
    float* pp = partial + static_cast<long long>(blockIdx.x) * 2 * C + c8 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pp[k] = s8[k];
      pp[C + k] = q8[k];
    }
  }
}

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return static_cast<int>(g < 16384 ? (g < 1 ? 1 : g) : 16384);
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

TTDK_EXPORT int ttdk_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q,
                                 int R, int S, int sh, int sw, int ph, int pw, hipStream_t st) {
  if (C % 8 || R * S > 255) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(N) * P * Q * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, y, arg, N, H, W, C, P, Q, R, S,
                     sh, sw, ph, pw);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_maxpool_bwd(const bf16_t* dy, const uint8_t* arg, bf16_t* dx, int N, int H, int W, int C, int P,
                                 int Q, int R, int S, int sh, int sw, int ph, int pw, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(N) * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, dy, arg, dx, N, H, W, C, P, Q, R, S,
                     sh, sw, ph, pw);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_avgpool_fwd(const bf16_t* x, bf16_t* y, float* yf, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int cg = C / 8;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((cg + 63) / 64, N), dim3(64), 0, st, x, y, yf, HW, C);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const long long total8 = static_cast<long long>(N) * HW * (C / 8);
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(total8)), dim3(256), 0, st, dy, dx, total8, HW, C);
  return hipGetLastError();
}

static bool stem_pool_ok(int N, int H, int W, int C, int P, int Q) {
  return C % 8 == 0 && 256 % (C / 8) == 0 && H == 2 * P && W == 2 * Q &&
         static_cast<long long>(N) * H * W * C < (1LL << 31) * 8;
}

// Fused BN-apply + ReLU + 3x3/s2/p1 max pooling (ResNet stem): see bn_relu_maxpool_kernel.
TTDK_EXPORT int ttdk_bn_relu_maxpool(const bf16_t* y, const float* scale, const float* shift, bf16_t* out,
                                     uint8_t* arg, uint8_t* mask, int N, int H, int W, int C, int P, int Q,
                                     hipStream_t st) {
  if (!stem_pool_ok(N, H, W, C, P, Q)) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(N) * P * Q * (C / 8);
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(grid_for(total)), dim3(256), 0, st, y, scale, shift, out, arg, mask,
                     N, H, W, C, P, Q);
  return hipGetLastError();
}

// Rows of `partial` ttdk_maxpool_bwd_bnstat writes (its grid size).
TTDK_EXPORT int ttdk_maxpool_bwd_bnstat_blocks(int N, int P, int Q, int C) {
  const long long per_block = 256 / (C / 8);
  long long b = (static_cast<long long>(N) * P * Q + per_block * 4 - 1) / (per_block * 4);  // ~4 blocks per thread
  return static_cast<int>(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

// Fused max-pool backward + ReLU mask + BN-backward partial sums (see maxpool_bwd_bnstat_kernel).
TTDK_EXPORT int ttdk_maxpool_bwd_bnstat(const bf16_t* dy, const uint8_t* arg, const uint8_t* mask, const bf16_t* y,
                                        bf16_t* g, float* partial, int N, int H, int W, int C, int P, int Q,
                                        hipStream_t st) {
  if (!stem_pool_ok(N, H, W, C, P, Q)) return hipErrorInvalidValue;
  const int grid = ttdk_maxpool_bwd_bnstat_blocks(N, P, Q, C);
  hipLaunchKernelGGL(maxpool_bwd_bnstat_kernel, dim3(grid), dim3(256), 0, st, dy, arg, mask, y, g, partial, N, H, W,
                     C, P, Q);
  return hipGetLastError();
}
