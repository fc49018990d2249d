// Fused sparse softmax cross-entropy: forward loss + backward dlogits + in_top_k(k=1) +
// batch-mean loss/accuracy in one pass per row.
//
// Reference ops: tf.nn.sparse_softmax_cross_entropy_with_logits (distribute_training.py:80-81),
// tf.reduce_mean (:82), tf.nn.in_top_k(logits, labels, 1) (:96) and the accuracy mean
// (:125) — SURVEY.md §2.6 F6-F8, G1. in_top_k follows TF: correct iff the number of classes
// whose logit is STRICTLY greater than the target's is < k; a non-finite target logit is
// never correct.
#include "common.h"

namespace ttdk {
namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) {
  return p[i];
}
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) {
  return bf2f(p[i]);
}

// One 256-thread block per row. grad_scale multiplies dlogits (e.g. 1/(rows*replicas)).
template <typename T, typename L>
__global__ __launch_bounds__(256) void xent_kernel(const T* __restrict__ logits, const L* __restrict__ labels, int V,
                                                   float grad_scale, float* __restrict__ loss_rows,
                                                   T* __restrict__ dlogits, uint8_t* __restrict__ correct,
                                                   float* __restrict__ part, float inv_rows) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
  const T* z = logits + row * V;
  const long long lab = static_cast<long long>(labels[row]);
  const bool lab_ok = lab >= 0 && lab < V;
  const float zt = lab_ok ? ld(z, lab) : NAN;
  float mx = -INFINITY;
  int greater = 0;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = ld(z, i);
    mx = fmaxf(mx, v);
    greater += v > zt;
  }
  mx = wave_max(mx);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = red[0];
  for (int i = 1; i < (blockDim.x >> 6); ++i) mx = fmaxf(mx, red[i]);
  float se = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) se += __expf(ld(z, i) - mx);
  se = block_sum(se, red + 8);
  const float gsum = block_sum(static_cast<float>(greater), red);
  const float lse = mx + __logf(se);
  const float loss = lse - zt;
  if (dlogits) {
    const float inv = 1.f / se;
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      float g = __expf(ld(z, i) - mx) * inv - (i == lab ? 1.f : 0.f);
      g *= grad_scale;
      if constexpr (sizeof(T) == 2)
        dlogits[row * V + i] = f2bf(g);
      else
        dlogits[row * V + i] = g;
    }
  }
  if (threadIdx.x == 0) {
    const bool ok = lab_ok && isfinite(zt) && gsum < 1.f;
    if (loss_rows) loss_rows[row] = loss;
    if (correct) correct[row] = ok;
    if (part) {  // per-row terms; xent_sums_kernel reduces them in a fixed order (deterministic)
      part[2 * row] = loss * inv_rows;
      part[2 * row + 1] = (ok ? 1.f : 0.f) * inv_rows;
    }
  }
}

// sums[0..1] = sum over rows of part[row][0..1], one block, fixed order.
__global__ __launch_bounds__(256) void xent_sums_kernel(const float* __restrict__ part, int rows,
                                                        float* __restrict__ sums) {
  __shared__ float red[16];
  float a = 0.f, b = 0.f;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    a += part[2 * r];
    b += part[2 * r + 1];
  }
  a = block_sum(a, red);
  b = block_sum(b, red + 8);
  if (threadIdx.x == 0) {
    sums[0] = a;
    sums[1] = b;
  }
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

// logits_dtype: 0 = fp32, 1 = bf16. label_dtype: 0 = int32, 1 = int64.
// sums (optional, fp32[2]) receives mean loss and mean accuracy; `part` (fp32[2*rows], needed
// with sums) holds the per-row terms, reduced in a fixed order (bitwise reproducible).
TTDK_EXPORT int ttdk_sparse_xent(const void* logits, int logits_dtype, const void* labels, int label_dtype, int rows,
                                 int V, float grad_scale, float* loss_rows, void* dlogits, uint8_t* correct,
                                 float* sums, float* part, hipStream_t st) {
  if (sums && !part) return hipErrorInvalidValue;
  const float inv = 1.f / rows;
  dim3 g(rows), b(256);
#define TTDK_X(T, L)                                                                                              \
  hipLaunchKernelGGL((xent_kernel<T, L>), g, b, 0, st, static_cast<const T*>(logits), static_cast<const L*>(labels), \
                     V, grad_scale, loss_rows, static_cast<T*>(dlogits), correct, sums ? part : nullptr, inv)
  if (logits_dtype == 0 && label_dtype == 0) TTDK_X(float, int32_t);
  else if (logits_dtype == 0) TTDK_X(float, int64_t);
  else if (label_dtype == 0) TTDK_X(bf16_t, int32_t);
  else TTDK_X(bf16_t, int64_t);
#undef TTDK_X
  if (sums) hipLaunchKernelGGL(xent_sums_kernel, dim3(1), dim3(256), 0, st, part, rows, sums);
  return hipGetLastError();
}
