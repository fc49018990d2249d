// Device-side random variable initialisation (tf.truncated_normal_initializer / random_normal /
// random_uniform run as device ops in the reference's graph, /root/reference/distribute_training.py:49):
// counter-based Philox-4x32-10, so every element is a pure function of (seed, offset, index)
// and the result does not depend on the launch shape. Big models (BERT-Large: 340 M
// parameters) initialise in milliseconds instead of seconds of host RNG + copy.
//
// dist 0: normal(a, b)   1: truncated normal(a, b), resampled outside +-2 b (TF semantics)
//      2: uniform[a, b)  3: constant a
#include "common.h"

namespace ttdk {
namespace {

__device__ __forceinline__ void box_muller(uint32_t x, uint32_t y, float& z0, float& z1) {
  // u1 in (0, 1] so the log is finite
  const float u1 = (static_cast<float>(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = static_cast<float>(y >> 8) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

__global__ void init_random_kernel(float* __restrict__ out, long long n, int dist, float a, float b,
                                   unsigned long long seed, unsigned long long offset) {
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    float v;
    if (dist == 3) {
      v = a;
    } else if (dist == 2) {
      uint32_t r[4];
      Philox::gen(seed, offset, static_cast<unsigned long long>(i), r);
      v = a + (b - a) * Philox::uniform(r[0]);
    } else {
      float z = 0.f;
      // round k draws from counter i of stream offset + k; two normals per round
      for (int k = 0; k < 64; ++k) {
        uint32_t r[4];
        Philox::gen(seed, offset + (static_cast<unsigned long long>(k) << 40), static_cast<unsigned long long>(i), r);
        float z0, z1;
        box_muller(r[0], r[1], z0, z1);
        if (dist == 0 || fabsf(z0) <= 2.f) { z = z0; break; }
        if (fabsf(z1) <= 2.f) { z = z1; break; }
        box_muller(r[2], r[3], z0, z1);
        if (fabsf(z0) <= 2.f) { z = z0; break; }
        if (fabsf(z1) <= 2.f) { z = z1; break; }
      }
      v = a + b * z;
    }
    out[i] = v;
  }
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

TTDK_EXPORT int ttdk_init_random(float* out, long long n, int dist, float a, float b, unsigned long long seed,
                                 unsigned long long offset, hipStream_t st) {
  if (n < 0 || dist < 0 || dist > 3) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  long long blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(init_random_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, out, n, dist, a, b, seed,
                     offset);
  return hipGetLastError();
}
