// Shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Conventions used by every kernel file:
//  * wave = 64 lanes; block sizes are multiples of 64;
//  * activations are NHWC (channels-last) bf16; parameters/optimizer state fp32;
//  * every exported launcher is `extern "C" int ttdk_*(..., hipStream_t)` and returns the
//    hipError_t of the launch, so PyTorch's current stream (and hipGraph capture) drives it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TTDK_EXPORT extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;

namespace ttdk {

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

// Round-to-nearest-even fp32 -> bf16 (NaN stays NaN: hipcc lowers the cast to v_cvt_pk_bf16_f32).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}

// Two fp32 -> one dword of two RNE bf16 in ONE v_cvt_pk_bf16_f32 (lo, hi). Packing two scalar
// casts instead emits one cvt_pk per element plus a shift and an or (4 VALU per pair): in the
// VALU-bound attention loops that was ~15 % of the instructions.
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// ReLU as ONE v_maximum3_f32 (gfx950; NaN-propagating like torch.relu / tf.nn.relu). fmaxf(x, 0)
// on a value the compiler cannot prove canonical (a bf16 load, an MFMA accumulator) costs a
// canonicalising v_max_f32 x, x, x first: two VALU per element in the GEMM / BN epilogues.
__device__ __forceinline__ float relu(float x) { return __builtin_elementwise_maximum(x, 0.f); }

__device__ __forceinline__ void unpack8(const uint4& v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  uint4 v;
  v.x = pack_bf16x2(f[0], f[1]);
  v.y = pack_bf16x2(f[2], f[3]);
  v.z = pack_bf16x2(f[4], f[5]);
  v.w = pack_bf16x2(f[6], f[7]);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}

// Philox-4x32-10 counter-based RNG (dropout masks, truncated-normal init).
struct Philox {
  static __device__ __forceinline__ void round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
  }
  static __device__ __forceinline__ void gen(uint64_t seed, uint64_t offset, uint64_t counter, uint32_t (&out)[4]) {
    uint32_t c[4] = {static_cast<uint32_t>(counter), static_cast<uint32_t>(counter >> 32),
                     static_cast<uint32_t>(offset), static_cast<uint32_t>(offset >> 32)};
    uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      round(c, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    out[0] = c[0];
    out[1] = c[1];
    out[2] = c[2];
    out[3] = c[3];
  }
  static __device__ __forceinline__ float uniform(uint32_t x) {  // [0,1)
    return (x >> 8) * (1.0f / 16777216.0f);
  }
};

inline int ceil_div(long long a, long long b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace ttdk
