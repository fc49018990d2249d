// Fused multi-tensor optimizers over flat fp32 parameter/gradient/state buffers.
//
// Reference: tf.train.GradientDescentOptimizer.apply_gradients -> ApplyGradientDescent x10
// (/root/reference/distribute_training.py:145,150,152) plus the north-star
// fused Adam/LAMB (BASELINE.json). All parameters of a model live in ONE flat fp32 buffer
// (and one flat gradient buffer, which is also what the bucketed all-reduce reduces), so a
// whole optimizer step is one launch over a chunk table:
//   chunk = (start, len, segment) with len <= 16384; segment = the variable it belongs to
//   (per-variable weight-decay factor; LAMB per-variable trust ratio).
// Hyper-parameters are read from a device array so a hipGraph-captured step picks up the
// learning-rate schedule without re-capture (ttdk_lr_schedule writes them in-graph).
// Every optimizer optionally refreshes a bf16 copy of the weights (the compute copy).
#include "common.h"

namespace ttdk {
namespace {

struct Chunk {
  long long start;
  int len;
  int seg;
};

// hyper layout (floats)
enum : int {
  kLr = 0,
  kMu = 1,      // momentum / beta1
  kBeta2 = 2,
  kEps = 3,
  kBc1 = 4,     // 1 - beta1^t
  kBc2 = 5,     // 1 - beta2^t
  kMaxNorm = 6, // global-norm clip (<= 0: off)
  kGradScale = 7,
};

__device__ __forceinline__ float clip_factor(const float* hyper, const float* sumsq) {
  float s = hyper[kGradScale];
  if (sumsq && hyper[kMaxNorm] > 0.f) {
    const float norm = sqrtf(*sumsq) * s;
    if (norm > hyper[kMaxNorm]) s *= hyper[kMaxNorm] / norm;
  }
  return s;
}

// kind: 0 = SGD, 1 = momentum, 2 = nesterov momentum
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                  float* __restrict__ mom, bf16_t* __restrict__ wbf,
                                                  const Chunk* __restrict__ chunks, const float* __restrict__ seg_wd,
                                                  const float* __restrict__ hyper, const float* __restrict__ sumsq,
                                                  int kind) {
  const Chunk ch = chunks[blockIdx.x];
  const float lr = hyper[kLr], mu = hyper[kMu];
  const float gs = clip_factor(hyper, sumsq);
  const float wd = seg_wd ? seg_wd[ch.seg] : 0.f;
  for (int i = threadIdx.x * 4; i < ch.len; i += blockDim.x * 4) {
    const long long o = ch.start + i;
    if (i + 3 < ch.len) {
      f32x4_t wv = *reinterpret_cast<f32x4_t*>(w + o);
      f32x4_t gv = *reinterpret_cast<const f32x4_t*>(g + o) * gs + wd * wv;
      if (kind == 0) {
        wv -= lr * gv;
      } else {
        f32x4_t m = *reinterpret_cast<f32x4_t*>(mom + o) * mu + gv;
        *reinterpret_cast<f32x4_t*>(mom + o) = m;
        wv -= lr * (kind == 2 ? gv + mu * m : m);
      }
      *reinterpret_cast<f32x4_t*>(w + o) = wv;
      if (wbf) {
        uint2 p;
        p.x = pack_bf16x2(wv[0], wv[1]);
        p.y = pack_bf16x2(wv[2], wv[3]);
        *reinterpret_cast<uint2*>(wbf + o) = p;
      }
    } else {
      for (int j = i; j < ch.len; ++j) {
        const long long oj = ch.start + j;
        float wv = w[oj];
        float gv = g[oj] * gs + wd * wv;
        if (kind == 0) {
          wv -= lr * gv;
        } else {
          const float m = mom[oj] * mu + gv;
          mom[oj] = m;
          wv -= lr * (kind == 2 ? gv + mu * m : m);
        }
        w[oj] = wv;
        if (wbf) wbf[oj] = f2bf(wv);
      }
    }
  }
}

// Adam / AdamW. decoupled=1: AdamW (w -= lr*wd*w), else L2 added to the gradient.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ wbf, const Chunk* __restrict__ chunks,
                                                   const float* __restrict__ seg_wd, const float* __restrict__ hyper,
                                                   const float* __restrict__ sumsq, int decoupled) {
  const Chunk ch = chunks[blockIdx.x];
  const float lr = hyper[kLr], b1 = hyper[kMu], b2 = hyper[kBeta2], eps = hyper[kEps];
  const float bc1 = hyper[kBc1] > 0.f ? hyper[kBc1] : 1.f, bc2 = hyper[kBc2] > 0.f ? hyper[kBc2] : 1.f;
  const float step = lr * sqrtf(bc2) / bc1;  // TF AdamOptimizer: lr_t = lr*sqrt(1-b2^t)/(1-b1^t)
  const float gs = clip_factor(hyper, sumsq);
  const float wd = seg_wd ? seg_wd[ch.seg] : 0.f;
  for (int i = threadIdx.x; i < ch.len; i += blockDim.x) {
    const long long o = ch.start + i;
    float wv = w[o];
    float gv = g[o] * gs;
    if (!decoupled) gv += wd * wv;
    const float mv = b1 * m[o] + (1.f - b1) * gv;
    const float vv = b2 * v[o] + (1.f - b2) * gv * gv;
    m[o] = mv;
    v[o] = vv;
    wv -= step * mv / (sqrtf(vv) + eps);
    if (decoupled) wv -= lr * wd * w[o];
    w[o] = wv;
    if (wbf) wbf[o] = f2bf(wv);
  }
}

// LAMB phase 1: update direction u = m_hat/(sqrt(v_hat)+eps) + wd*w into `u`, and per-CHUNK
// sums of w^2 and u^2 (chunk_norms[2*chunk]); lamb_segnorm_kernel folds the chunks of each
// variable in a fixed order. No float atomics: every replica of a data-parallel job computes
// bit-identical trust ratios from bit-identical all-reduced gradients, so the replicas never
// drift apart.
__global__ __launch_bounds__(256) void lamb_phase1_kernel(const float* __restrict__ w, const float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          float* __restrict__ u, const Chunk* __restrict__ chunks,
                                                          const float* __restrict__ seg_wd,
                                                          const float* __restrict__ hyper,
                                                          const float* __restrict__ sumsq, float* __restrict__ chunk_norms) {
  __shared__ float red[16];
  const Chunk ch = chunks[blockIdx.x];
  const float b1 = hyper[kMu], b2 = hyper[kBeta2], eps = hyper[kEps];
  const float bc1 = hyper[kBc1] > 0.f ? hyper[kBc1] : 1.f, bc2 = hyper[kBc2] > 0.f ? hyper[kBc2] : 1.f;
  const float gs = clip_factor(hyper, sumsq);
  const float wd = seg_wd ? seg_wd[ch.seg] : 0.f;
  float sw = 0.f, su = 0.f;
  auto one = [&](float wv, float gv, float& mo, float& vo) {
    const float mv = b1 * mo + (1.f - b1) * gv;
    const float vv = b2 * vo + (1.f - b2) * gv * gv;
    mo = mv;
    vo = vv;
    const float uu = (mv / bc1) / (sqrtf(vv / bc2) + eps) + wd * wv;
    sw += wv * wv;
    su += uu * uu;
    return uu;
  };
  // 16-B accesses (every variable starts 64-element aligned in the flat buffer, chunks are
  // 16384 long): 28 B per parameter, HBM-bound
  for (int i = threadIdx.x * 4; i < ch.len; i += blockDim.x * 4) {
    const long long o = ch.start + i;
    if (i + 3 < ch.len) {
      const f32x4_t wv = *reinterpret_cast<const f32x4_t*>(w + o);
      const f32x4_t gv = *reinterpret_cast<const f32x4_t*>(g + o) * gs;
      f32x4_t mv = *reinterpret_cast<const f32x4_t*>(m + o), vv = *reinterpret_cast<const f32x4_t*>(v + o);
      f32x4_t uv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float mo = mv[j], vo = vv[j];
        uv[j] = one(wv[j], gv[j], mo, vo);
        mv[j] = mo;
        vv[j] = vo;
      }
      *reinterpret_cast<f32x4_t*>(m + o) = mv;
      *reinterpret_cast<f32x4_t*>(v + o) = vv;
      *reinterpret_cast<f32x4_t*>(u + o) = uv;
    } else {
      for (int j = i; j < ch.len; ++j) {
        const long long oj = ch.start + j;
        float mo = m[oj], vo = v[oj];
        u[oj] = one(w[oj], g[oj] * gs, mo, vo);
        m[oj] = mo;
        v[oj] = vo;
      }
    }
  }
  sw = block_sum(sw, red);
  su = block_sum(su, red + 8);
  if (threadIdx.x == 0) {
    chunk_norms[2 * blockIdx.x] = sw;
    chunk_norms[2 * blockIdx.x + 1] = su;
  }
}

// seg_norms[2*seg + {0,1}] = sum of chunk_norms over the (consecutive) chunks of segment `seg`
// (block per segment; the chunk range is found by binary search on the sorted seg ids).
__global__ __launch_bounds__(256) void lamb_segnorm_kernel(const Chunk* __restrict__ chunks, int n_chunks,
                                                           const float* __restrict__ chunk_norms,
                                                           float* __restrict__ seg_norms) {
  __shared__ float red[16];
  const int seg = blockIdx.x;
  int lo = 0, hi = n_chunks;  // first chunk with seg >= this
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (chunks[mid].seg < seg) lo = mid + 1; else hi = mid;
  }
  const int first = lo;
  hi = n_chunks;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (chunks[mid].seg <= seg) lo = mid + 1; else hi = mid;
  }
  const int last = lo;
  float sw = 0.f, su = 0.f;
  for (int c = first + threadIdx.x; c < last; c += blockDim.x) {
    sw += chunk_norms[2 * c];
    su += chunk_norms[2 * c + 1];
  }
  sw = block_sum(sw, red);
  su = block_sum(su, red + 8);
  if (threadIdx.x == 0) {
    seg_norms[2 * seg] = sw;
    seg_norms[2 * seg + 1] = su;
  }
}

__global__ __launch_bounds__(256) void lamb_phase2_kernel(float* __restrict__ w, const float* __restrict__ u,
                                                          bf16_t* __restrict__ wbf, const Chunk* __restrict__ chunks,
                                                          const float* __restrict__ hyper,
                                                          const float* __restrict__ seg_norms) {
  const Chunk ch = chunks[blockIdx.x];
  const float wn = sqrtf(seg_norms[2 * ch.seg]), un = sqrtf(seg_norms[2 * ch.seg + 1]);
  const float trust = (wn > 0.f && un > 0.f) ? wn / un : 1.f;
  const float step = hyper[kLr] * trust;
  for (int i = threadIdx.x * 4; i < ch.len; i += blockDim.x * 4) {
    const long long o = ch.start + i;
    if (i + 3 < ch.len) {
      const f32x4_t wv = *reinterpret_cast<const f32x4_t*>(w + o) - step * *reinterpret_cast<const f32x4_t*>(u + o);
      *reinterpret_cast<f32x4_t*>(w + o) = wv;
      if (wbf) {
        uint2 p;
        p.x = pack_bf16x2(wv[0], wv[1]);
        p.y = pack_bf16x2(wv[2], wv[3]);
        *reinterpret_cast<uint2*>(wbf + o) = p;
      }
    } else {
      for (int j = i; j < ch.len; ++j) {
        const long long oj = ch.start + j;
        const float wv = w[oj] - step * u[oj];
        w[oj] = wv;
        if (wbf) wbf[oj] = f2bf(wv);
      }
    }
  }
}

// Global sum of squares (gradient clipping): per-block partials, then one block folds them in
// a fixed order (deterministic, no atomics).
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, long long n,
                                                    float* __restrict__ partial) {
  __shared__ float red[16];
  float s = 0.f;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    s += x[i] * x[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partial, int n,
                                                           float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) *out = s;
}

// In-graph learning-rate schedule + step counter.
//   kind 0: constant; 1: exponential decay (staircase flag); 2: polynomial decay with linear warmup;
//   3: piecewise-linear warmup then cosine.
// sched = [base_lr, decay_steps, decay_rate, staircase, warmup_steps, end_lr, power, total_steps]
// The step used is the value BEFORE the increment (as tf.train.exponential_decay reading
// global_step inside the same run that increments it).
__global__ void lr_schedule_kernel(long long* __restrict__ step, const float* __restrict__ sched, int kind,
                                   float* __restrict__ hyper, float beta1, float beta2, int increment) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long s = *step;
  const float base = sched[0];
  float lr = base;
  const float fs = static_cast<float>(s);
  if (kind == 1) {
    float p = fs / sched[1];
    if (sched[3] != 0.f) p = floorf(p);
    lr = base * powf(sched[2], p);
  } else if (kind == 2) {
    const float warm = sched[4];
    if (warm > 0.f && fs < warm) {
      lr = base * (fs + 1.f) / warm;
    } else {
      const float total = sched[7];
      const float t = fminf(fs, total);
      lr = (base - sched[5]) * powf(1.f - t / total, sched[6]) + sched[5];
    }
  } else if (kind == 3) {
    const float warm = sched[4], total = sched[7];
    if (warm > 0.f && fs < warm)
      lr = base * (fs + 1.f) / warm;
    else
      lr = sched[5] + 0.5f * (base - sched[5]) * (1.f + cosf(3.14159265358979f * fminf(1.f, (fs - warm) / fmaxf(1.f, total - warm))));
  }
  hyper[kLr] = lr;
  const float t1 = static_cast<float>(s + 1);
  hyper[kBc1] = 1.f - powf(beta1, t1);
  hyper[kBc2] = 1.f - powf(beta2, t1);
  if (increment) *step = s + 1;
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

TTDK_EXPORT int ttdk_opt_sgd(float* w, const float* g, float* mom, bf16_t* wbf, const void* chunks, int n_chunks,
                             const float* seg_wd, const float* hyper, const float* sumsq, int kind, hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(n_chunks), dim3(256), 0, st, w, g, mom, wbf, static_cast<const Chunk*>(chunks),
                     seg_wd, hyper, sumsq, kind);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_opt_adam(float* w, const float* g, float* m, float* v, bf16_t* wbf, const void* chunks,
                              int n_chunks, const float* seg_wd, const float* hyper, const float* sumsq, int decoupled,
                              hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(n_chunks), dim3(256), 0, st, w, g, m, v, wbf, static_cast<const Chunk*>(chunks),
                     seg_wd, hyper, sumsq, decoupled);
  return hipGetLastError();
}

// u: scratch of the flat size; seg_norms: fp32[2*n_segments]; chunk_norms: fp32[2*n_chunks].
TTDK_EXPORT int ttdk_opt_lamb(float* w, const float* g, float* m, float* v, float* u, bf16_t* wbf, const void* chunks,
                              int n_chunks, int n_segments, const float* seg_wd, const float* hyper, const float* sumsq,
                              float* seg_norms, float* chunk_norms, hipStream_t st) {
  if (!chunk_norms) return hipErrorInvalidValue;
  const Chunk* c = static_cast<const Chunk*>(chunks);
  hipLaunchKernelGGL(lamb_phase1_kernel, dim3(n_chunks), dim3(256), 0, st, w, g, m, v, u, c, seg_wd, hyper, sumsq,
                     chunk_norms);
  hipLaunchKernelGGL(lamb_segnorm_kernel, dim3(n_segments), dim3(256), 0, st, c, n_chunks, chunk_norms, seg_norms);
  hipLaunchKernelGGL(lamb_phase2_kernel, dim3(n_chunks), dim3(256), 0, st, w, u, wbf, c, hyper, seg_norms);
  return hipGetLastError();
}

// out (fp32 scalar) = sum x^2; `partial`: scratch of >= 2048 floats.
TTDK_EXPORT int ttdk_sumsq(const float* x, long long n, float* out, float* partial, hipStream_t st) {
  if (!partial) return hipErrorInvalidValue;
  long long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sumsq_kernel, dim3(static_cast<int>(blocks)), dim3(256), 0, st, x, n, partial);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, st, partial, static_cast<int>(blocks), out);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_lr_schedule(long long* step, const float* sched, int kind, float* hyper, float beta1, float beta2,
                                 int increment, hipStream_t st) {
  hipLaunchKernelGGL(lr_schedule_kernel, dim3(1), dim3(64), 0, st, step, sched, kind, hyper, beta1, beta2, increment);
  return hipGetLastError();
}
