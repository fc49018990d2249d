// fp8 (OCP e4m3fn) scaling state for the fp8 training path (BASELINE.json config 5).
//
// Every fp8 tensor stream owns a slot float[SLOT] = {amax_prev, amax_cur, scale, inv_scale, -, -, -, -,
// 64 amax lanes}; producers with many workgroups (BN apply) spread their atomicMax over the 64
// lanes (blockIdx % 64) so they do not serialise on one address; rollover folds the lanes.
//   * activations use DELAYED scaling: the producer (BN apply) quantises with `scale` derived
//     from the previous step's amax and accumulates this step's amax into amax_cur;
//     ttdk_fp8_rollover (once per step, graph-capturable) moves amax_cur -> amax_prev and
//     recomputes scale = fmax * margin / amax_prev;
//   * weights use CURRENT scaling over a multi-tensor table (two launches for all tensors):
//     per-tensor amax, then quantisation with scale = fmax / amax.
// GEMM epilogues read inv_scale pointers (EpiParams::ascale0/1), so nothing here needs a host
// synchronisation.
#include "common.h"

namespace ttdk {
namespace {

constexpr int SLOT = 72;

__global__ void rollover_kernel(float* __restrict__ slots, int n, float fmax, float margin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* s = slots + SLOT * i;
  float cur = s[1];
  for (int l = 0; l < 64; ++l) {
    cur = fmaxf(cur, s[8 + l]);
    s[8 + l] = 0.f;
  }
  const float prev = cur > 0.f ? cur : s[0];
  s[0] = prev;
  s[1] = 0.f;
  const float sc = prev > 0.f ? fmax * margin / prev : 1.f;
  s[2] = sc;
  s[3] = 1.f / sc;
}

struct QEntry {
  long long offset;  // element offset into the bf16 source / uint8 destination buffers
  int len;
  int slot;
};

__global__ __launch_bounds__(256) void multi_amax_kernel(const bf16_t* __restrict__ src, const QEntry* __restrict__ tab,
                                                         float* __restrict__ slots) {
  const QEntry e = tab[blockIdx.y];
  float m = 0.f;
  for (long long i = (static_cast<long long>(blockIdx.x) * 256 + threadIdx.x) * 8; i < e.len;
       i += static_cast<long long>(gridDim.x) * 256 * 8) {
    if (i + 8 <= e.len) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(src + e.offset + i), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[j]));
    } else {
      for (long long j = i; j < e.len; ++j) m = fmaxf(m, fabsf(bf2f(src[e.offset + j])));
    }
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(slots + SLOT * e.slot + 1), __float_as_uint(m));
}

__global__ __launch_bounds__(256) void multi_quant_kernel(const bf16_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          const QEntry* __restrict__ tab, float* __restrict__ slots,
                                                          float fmax) {
  const QEntry e = tab[blockIdx.y];
  float* s = slots + SLOT * e.slot;
  const float amax = s[1];
  const float sc = amax > 0.f ? fmax / amax : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s[0] = amax;
    s[2] = sc;
    s[3] = 1.f / sc;
  }
  for (long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x; i < e.len;
       i += static_cast<long long>(gridDim.x) * 256) {
    const float v = fminf(fmaxf(bf2f(src[e.offset + i]) * sc, -fmax), fmax);
    dst[e.offset + i] = static_cast<uint8_t>(__builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false) & 0xff);
  }
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

TTDK_EXPORT int ttdk_fp8_rollover(float* slots, int n, float fmax, float margin, hipStream_t st) {
  hipLaunchKernelGGL(rollover_kernel, dim3((n + 255) / 256), dim3(256), 0, st, slots, n, fmax, margin);
  return hipGetLastError();
}

// table: device array of n_tensors {int64 offset, int32 len, int32 slot}; max_len bounds the grid.
TTDK_EXPORT int ttdk_fp8_quant_weights(const bf16_t* src, uint8_t* dst, const void* table, int n_tensors, int max_len,
                                       float* slots, int n_slots, hipStream_t st) {
  const QEntry* tab = static_cast<const QEntry*>(table);
  // amax_cur of the weight slots is rebuilt from scratch every call
  hipLaunchKernelGGL(rollover_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, st, slots, n_slots, 448.f, 1.f);
  int gx = (max_len + 256 * 8 - 1) / (256 * 8);
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(multi_amax_kernel, dim3(gx, n_tensors), dim3(256), 0, st, src, tab, slots);
  int gq = (max_len + 255) / 256;
  if (gq > 256) gq = 256;
  hipLaunchKernelGGL(multi_quant_kernel, dim3(gq, n_tensors), dim3(256), 0, st, src, dst, tab, slots, 448.f);
  return hipGetLastError();
}
