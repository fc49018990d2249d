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
