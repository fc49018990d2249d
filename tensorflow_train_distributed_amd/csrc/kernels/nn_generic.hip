// Shape-general kernels behind the functional `ttd.nn` ops (tf.nn / tf.layers surface, SURVEY.md
// §2.2 T22-T25, §7.5) for the shapes and dtypes the fused model engines never see: any channel /
// feature count, fp32 or bf16 tensors. The model engines (ResNet, BERT, MLP) use the vectorised,
// fused kernels in batchnorm/pool/transformer/xent.hip; these exist so that a ttd.nn op on a GPU
// tensor always runs a HIP kernel instead of silently falling back to an eager torch op.
//
// Everything is one scalar element per lane with 64-wide column groups (coalesced along the
// contiguous channel axis), fp32 accumulation, and deterministic reductions (per-block column
// partials folded in a fixed order) except the embedding gradient, which scatters with fp32
// global atomics like tf.math.unsorted_segment_sum on GPU.
//
// dt: 0 = fp32, 1 = bf16 (every tensor argument of one call shares it; statistics are fp32).
#include "common.h"

namespace ttdk {
namespace {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, long long i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }

template <typename T>
__device__ __forceinline__ void stf(T* p, long long i, float v);
template <>
__device__ __forceinline__ void stf<float>(float* p, long long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void stf<bf16_t>(bf16_t* p, long long i, float v) { p[i] = f2bf(v); }

__device__ __forceinline__ long long gidx() { return static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; }
__device__ __forceinline__ long long gstride() { return static_cast<long long>(gridDim.x) * blockDim.x; }

inline unsigned grid_for(long long n) {
  long long b = (n + 255) / 256;
  return static_cast<unsigned>(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

// ------------------------------------------------------------------ column statistics
// part[t][0][c] = sum_r a, part[t][1][c] = sum_r a*b   (mode 1)
//                                       = sum_r a*a    (mode 0)
//                                       = sum_r a*(b - mu[r])*rs[r]   (mode 2, LayerNorm dgamma)
// over the rows [t*rpb, (t+1)*rpb). Block = 64 columns x 4 row groups.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void col_stats_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                        const float* __restrict__ mu, const float* __restrict__ rs,
                                                        long long M, int C, long long rpb, float* __restrict__ part) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long long r0 = blockIdx.y * rpb;
  const long long r1 = r0 + rpb < M ? r0 + rpb : M;
  float s = 0.f, q = 0.f;
  if (c < C) {
    for (long long r = r0 + rg; r < r1; r += 4) {
      const float va = ldf(a, r * C + c);
      s += va;
      if (MODE == 0) q += va * va;
      else if (MODE == 1) q += va * ldf(b, r * C + c);
      else q += va * (ldf(b, r * C + c) - mu[r]) * rs[r];
    }
  }
  red[0][rg][cl] = s;
  red[1][rg][cl] = q;
  __syncthreads();
  if (rg != 0 || c >= C) return;
  s = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
  q = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  part[(2LL * blockIdx.y) * C + c] = s;
  part[(2LL * blockIdx.y + 1) * C + c] = q;
}

// o0[c] = sum_t part[t][0][c] (+ o0 if acc), o1[c] likewise; fixed order -> deterministic
__global__ void col_reduce2_kernel(const float* __restrict__ part, int T, int C, float* __restrict__ o0,
                                   float* __restrict__ o1, int acc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, q = 0.f;
  for (int t = 0; t < T; ++t) {
    s += part[(2LL * t) * C + c];
    q += part[(2LL * t + 1) * C + c];
  }
  if (o0) o0[c] = s + (acc ? o0[c] : 0.f);
  if (o1) o1[c] = q + (acc ? o1[c] : 0.f);
}

// out = a*c0[c] + (b ? b*c1[c] : 0) + (c2 ? c2[c] : 0)
template <typename T>
__global__ void col_affine_kernel(const T* __restrict__ a, const T* __restrict__ b, const float* __restrict__ c0,
                                  const float* __restrict__ c1, const float* __restrict__ c2, T* __restrict__ out,
                                  long long n, int C) {
  for (long long i = gidx(); i < n; i += gstride()) {
    const int c = static_cast<int>(i % C);
    float v = ldf(a, i) * c0[c];
    if (b) v += ldf(b, i) * c1[c];
    if (c2) v += c2[c];
    stf(out, i, v);
  }
}

// inference-mode BN coefficients from the moving statistics
__global__ void bn_infer_coef_kernel(const float* __restrict__ mm, const float* __restrict__ mv,
                                     const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int C,
                                     float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float r = rsqrtf(mv[c] + eps);
  const float sc = (gamma ? gamma[c] : 1.f) * r;
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - mm[c] * sc;
  rstd[c] = r;
}

// inference-mode BN backward parameter gradients from (sum g, sum g*x) partials:
// dgamma = rstd * (sum g*x - mm * sum g), dbeta = sum g
__global__ void bn_infer_bwd_kernel(const float* __restrict__ part, int T, int C, const float* __restrict__ mm,
                                    const float* __restrict__ rstd, float* __restrict__ dgamma,
                                    float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, q = 0.f;
  for (int t = 0; t < T; ++t) {
    s += part[(2LL * t) * C + c];
    q += part[(2LL * t + 1) * C + c];
  }
  if (dgamma) dgamma[c] = rstd[c] * (q - mm[c] * s);
  if (dbeta) dbeta[c] = s;
}

// ------------------------------------------------------------------ pooling (NHWC, any C)
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ arg, int N, int H,
                                   int W, int C, int P, int Q, int R, int S, int sh, int sw, int ph, int pw) {
  const long long total = static_cast<long long>(N) * P * Q * C;
  for (long long i = gidx(); i < total; i += gstride()) {
    const int c = static_cast<int>(i % C);
    long long t = i / C;
    const int q = static_cast<int>(t % Q);
    t /= Q;
    const int p = static_cast<int>(t % P);
    const int n = static_cast<int>(t / P);
    float best = -__builtin_huge_valf();
    int bi = 0;
    bool any = false;
    for (int r = 0; r < R; ++r) {
      const int h = p * sh - ph + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < S; ++s) {
        const int w = q * sw - pw + s;
        if (w < 0 || w >= W) continue;
        const float v = ldf(x, ((static_cast<long long>(n) * H + h) * W + w) * C + c);
        // first strict maximum wins; a NaN propagates (TF MaxPool semantics)
        if (!any || v > best || (v != v && best == best)) {
          best = v;
          bi = r * S + s;
          any = true;
        }
      }
    }
    stf(y, i, best);
    arg[i] = static_cast<uint8_t>(bi);
  }
}

// gather formulation: every input element sums the output gradients whose window chose it
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ arg, T* __restrict__ dx, int N,
                                   int H, int W, int C, int P, int Q, int R, int S, int sh, int sw, int ph, int pw) {
  const long long total = static_cast<long long>(N) * H * W * C;
  for (long long i = gidx(); i < total; i += gstride()) {
    const int c = static_cast<int>(i % C);
    long long t = i / C;
    const int w = static_cast<int>(t % W);
    t /= W;
    const int h = static_cast<int>(t % H);
    const int n = static_cast<int>(t / H);
    // p with p*sh - ph <= h <= p*sh - ph + R - 1
    int p_lo = h + ph - R + 1;
    p_lo = p_lo <= 0 ? 0 : (p_lo + sh - 1) / sh;
    int p_hi = (h + ph) / sh;
    if (p_hi > P - 1) p_hi = P - 1;
    int q_lo = w + pw - S + 1;
    q_lo = q_lo <= 0 ? 0 : (q_lo + sw - 1) / sw;
    int q_hi = (w + pw) / sw;
    if (q_hi > Q - 1) q_hi = Q - 1;
    float acc = 0.f;
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * sh - ph);
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * sw - pw);
        const long long o = ((static_cast<long long>(n) * P + p) * Q + q) * C + c;
        if (arg[o] == r * S + s) acc += ldf(dy, o);
      }
    }
    stf(dx, i, acc);
  }
}

// global average pool: y[n][c] = mean over HW; block = 64 channels x 4 row groups
template <typename T>
__global__ __launch_bounds__(256) void gap_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int HW, int C) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int n = blockIdx.y;
  float s = 0.f;
  if (c < C)
    for (int r = rg; r < HW; r += 4) s += ldf(x, (static_cast<long long>(n) * HW + r) * C + c);
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < C)
    stf(y, static_cast<long long>(n) * C + c, (red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]) / HW);
}

template <typename T>
__global__ void gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, long long total, int HW, int C) {
  const float inv = 1.f / HW;
  for (long long i = gidx(); i < total; i += gstride()) {
    const int c = static_cast<int>(i % C);
    const long long n = i / (static_cast<long long>(HW) * C);
    stf(dx, i, ldf(dy, n * C + c) * inv);
  }
}

// ------------------------------------------------------------------ LayerNorm (any width)
// one wave per row, 4 rows per block; two-pass statistics (mean, then centred variance)
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ g,
                                                     const float* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean, float* __restrict__ rstd, long long rows,
                                                     int H, float eps) {
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* xr = x + row * H;
  float s = 0.f;
  for (int j = lane; j < H; j += 64) s += ldf(xr, j);
  const float mu = wave_sum(s) / H;
  float v = 0.f;
  for (int j = lane; j < H; j += 64) {
    const float d = ldf(xr, j) - mu;
    v += d * d;
  }
  const float r = rsqrtf(wave_sum(v) / H + eps);
  for (int j = lane; j < H; j += 64) stf(y + row * H, j, (ldf(xr, j) - mu) * r * g[j] + b[j]);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = r;
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat))
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_dx_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                        const float* __restrict__ g, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, T* __restrict__ dx,
                                                        long long rows, int H) {
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float mu = mean[row], r = rstd[row];
  const T* dr = dy + row * H;
  const T* xr = x + row * H;
  float s1 = 0.f, s2 = 0.f;
  for (int j = lane; j < H; j += 64) {
    const float dg = ldf(dr, j) * g[j];
    s1 += dg;
    s2 += dg * (ldf(xr, j) - mu) * r;
  }
  s1 = wave_sum(s1) / H;
  s2 = wave_sum(s2) / H;
  for (int j = lane; j < H; j += 64) {
    const float xh = (ldf(xr, j) - mu) * r;
    stf(dx + row * H, j, r * (ldf(dr, j) * g[j] - s1 - xh * s2));
  }
}

// ------------------------------------------------------------------ embedding / metrics / unary
template <typename T, typename I>
__global__ void gather_kernel(const T* __restrict__ table, const I* __restrict__ ids, T* __restrict__ out, long long n,
                              int H, long long V) {
  for (long long i = gidx(); i < n * H; i += gstride()) {
    const long long id = static_cast<long long>(ids[i / H]);
    // out-of-range ids read as zeros (the GPU behaviour of tf.gather)
    stf(out, i, (id >= 0 && id < V) ? ldf(table, id * H + i % H) : 0.f);
  }
}

template <typename T, typename I>
__global__ void scatter_add_kernel(const T* __restrict__ dy, const I* __restrict__ ids, float* __restrict__ dtable,
                                   long long n, int H, long long V) {
  for (long long i = gidx(); i < n * H; i += gstride()) {
    const long long id = static_cast<long long>(ids[i / H]);
    if (id >= 0 && id < V) atomicAdd(dtable + id * H + i % H, ldf(dy, i));
  }
}

// tf.nn.in_top_k: correct iff fewer than k logits are strictly greater than the target's and
// the target logit is finite; one wave per row
template <typename T, typename I>
__global__ __launch_bounds__(256) void in_top_k_kernel(const T* __restrict__ z, const I* __restrict__ tgt,
                                                       uint8_t* __restrict__ out, long long rows, int V, int k) {
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long long t = static_cast<long long>(tgt[row]);
  const bool valid = t >= 0 && t < V;
  const float zt = valid ? ldf(z + row * V, t) : 0.f;
  int cnt = 0;
  for (int j = lane; j < V; j += 64) cnt += ldf(z + row * V, j) > zt ? 1 : 0;
  cnt = wave_sum(cnt);
  if (lane == 0) out[row] = (valid && cnt < k && __builtin_isfinite(zt)) ? 1 : 0;
}

template <typename T>
__global__ void unary_kernel(const T* __restrict__ x, T* __restrict__ y, long long n, int op) {
  for (long long i = gidx(); i < n; i += gstride()) {
    const float v = ldf(x, i);
    stf(y, i, op == 0 ? tanhf(v) : 1.f / (1.f + __expf(-v)));
  }
}

// gradient from the op's output y: tanh' = 1 - y^2, sigmoid' = y (1 - y)
template <typename T>
__global__ void unary_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, long long n,
                                 int op) {
  for (long long i = gidx(); i < n; i += gstride()) {
    const float v = ldf(y, i);
    stf(dx, i, ldf(dy, i) * (op == 0 ? 1.f - v * v : v * (1.f - v)));
  }
}

// ------------------------------------------------------------------ reductions / scaling glue
// stage 1: ws[b] = sum of block b's grid-stride slice (fixed order within and across blocks)
template <typename T>
__global__ __launch_bounds__(256) void sum_partial_kernel(const T* __restrict__ x, long long n, float* __restrict__ ws) {
  __shared__ float red[16];
  float s = 0.f;
  for (long long i = gidx(); i < n; i += gstride()) s += ldf(x, i);
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// stage 2: out[0] = scale * sum(ws[0..nb))
template <typename T>
__global__ __launch_bounds__(256) void sum_final_kernel(const float* __restrict__ ws, int nb, float scale,
                                                        T* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += ws[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) stf(out, 0, s * scale);
}

// dx[i] = g[0] * scale (gradient of a scaled full reduction)
template <typename T>
__global__ void fill_scaled_kernel(T* __restrict__ dx, long long n, const T* __restrict__ g, float scale) {
  const float v = ldf(g, 0) * scale;
  for (long long i = gidx(); i < n; i += gstride()) stf(dx, i, v);
}

// out[r][c] = a[r][c] * g[r] (per-example loss gradient into the logits gradient)
template <typename T>
__global__ void row_scale_kernel(const T* __restrict__ a, const float* __restrict__ g, T* __restrict__ out, long long n,
                                 int C) {
  for (long long i = gidx(); i < n; i += gstride()) stf(out, i, ldf(a, i) * g[i / C]);
}

// empty kernel that delimits a region in a kernel trace (tools/nn_step_trace.py)
__global__ void trace_marker_kernel(int) {}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

// launch KER<float> or KER<bf16_t> by dt, casting the untyped pointers
#define TTDK_LAUNCH_DT(dt, KER, grid, block, ...)                                                    \
  do {                                                                                              \
    if ((dt) == 0) {                                                                                \
      typedef float TT;                                                                             \
      hipLaunchKernelGGL(KER<TT>, grid, block, 0, st, __VA_ARGS__);                                 \
    } else if ((dt) == 1) {                                                                         \
      typedef bf16_t TT;                                                                            \
      hipLaunchKernelGGL(KER<TT>, grid, block, 0, st, __VA_ARGS__);                                 \
    } else {                                                                                        \
      return hipErrorInvalidValue;                                                                  \
    }                                                                                               \
  } while (0)

// number of row blocks the column-statistics kernel splits M rows into
TTDK_EXPORT int ttdk_col_stats_parts(long long M, int C) {
  const long long cb = (C + 63) / 64;
  long long t = (M + 255) / 256;
  const long long cap = 2048 / cb > 1 ? 2048 / cb : 1;
  if (t > cap) t = cap;
  return static_cast<int>(t < 1 ? 1 : t);
}

// mode 0: (sum a, sum a^2); mode 1: (sum a, sum a*b); mode 2: (sum a, sum a*(b-mu[r])*rs[r])
TTDK_EXPORT int ttdk_col_stats(const void* a, const void* b, const float* mu, const float* rs, int dt, int mode,
                               long long M, int C, float* part, int T, hipStream_t st) {
  if (C <= 0 || M <= 0 || T <= 0 || (mode != 0 && !b) || (mode == 2 && (!mu || !rs))) return hipErrorInvalidValue;
  const long long rpb = (M + T - 1) / T;
  dim3 grid((C + 63) / 64, T), block(256);
#define TTDK_CS(TT)                                                                                                    \
  switch (mode) {                                                                                                      \
    case 0: hipLaunchKernelGGL((col_stats_kernel<TT, 0>), grid, block, 0, st, (const TT*)a, (const TT*)b, mu, rs, M, C, \
                               rpb, part); break;                                                                      \
    case 1: hipLaunchKernelGGL((col_stats_kernel<TT, 1>), grid, block, 0, st, (const TT*)a, (const TT*)b, mu, rs, M, C, \
                               rpb, part); break;                                                                      \
    case 2: hipLaunchKernelGGL((col_stats_kernel<TT, 2>), grid, block, 0, st, (const TT*)a, (const TT*)b, mu, rs, M, C, \
                               rpb, part); break;                                                                      \
    default: return hipErrorInvalidValue;                                                                              \
  }
  if (dt == 0) { TTDK_CS(float) } else if (dt == 1) { TTDK_CS(bf16_t) } else return hipErrorInvalidValue;
#undef TTDK_CS
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_col_reduce2(const float* part, int T, int C, float* o0, float* o1, int acc, hipStream_t st) {
  hipLaunchKernelGGL(col_reduce2_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, T, C, o0, o1, acc);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_col_affine(const void* a, const void* b, int dt, const float* c0, const float* c1, const float* c2,
                                void* out, long long n, int C, hipStream_t st) {
  if (C <= 0 || (b && !c1)) return hipErrorInvalidValue;
  if (dt == 0)
    hipLaunchKernelGGL(col_affine_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)a, (const float*)b,
                       c0, c1, c2, (float*)out, n, C);
  else if (dt == 1)
    hipLaunchKernelGGL(col_affine_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16_t*)a,
                       (const bf16_t*)b, c0, c1, c2, (bf16_t*)out, n, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_bn_infer_coef(const float* mm, const float* mv, const float* gamma, const float* beta, float eps,
                                   int C, float* scale, float* shift, float* rstd, hipStream_t st) {
  hipLaunchKernelGGL(bn_infer_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, mm, mv, gamma, beta, eps, C, scale,
                     shift, rstd);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_bn_infer_bwd(const float* part, int T, int C, const float* mm, const float* rstd, float* dgamma,
                                  float* dbeta, hipStream_t st) {
  hipLaunchKernelGGL(bn_infer_bwd_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, T, C, mm, rstd, dgamma, dbeta);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_maxpool_generic_fwd(const void* x, void* y, uint8_t* arg, int dt, int N, int H, int W, int C, int P,
                                         int Q, int R, int S, int sh, int sw, int ph, int pw, hipStream_t st) {
  if (R * S > 255 || ph >= R || pw >= S || P <= 0 || Q <= 0) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(N) * P * Q * C;
  if (dt == 0)
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x, (float*)y,
                       arg, N, H, W, C, P, Q, R, S, sh, sw, ph, pw);
  else if (dt == 1)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)y, arg, N, H, W, C, P, Q, R, S, sh, sw, ph, pw);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_maxpool_generic_bwd(const void* dy, const uint8_t* arg, void* dx, int dt, int N, int H, int W,
                                         int C, int P, int Q, int R, int S, int sh, int sw, int ph, int pw,
                                         hipStream_t st) {
  const long long total = static_cast<long long>(N) * H * W * C;
  if (dt == 0)
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)dy, arg,
                       (float*)dx, N, H, W, C, P, Q, R, S, sh, sw, ph, pw);
  else if (dt == 1)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16_t*)dy, arg,
                       (bf16_t*)dx, N, H, W, C, P, Q, R, S, sh, sw, ph, pw);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_gap_fwd(const void* x, void* y, int dt, int N, int HW, int C, hipStream_t st) {
  if (N <= 0 || N > 65535 || HW <= 0 || C <= 0) return hipErrorInvalidValue;
  dim3 grid((C + 63) / 64, N);
  TTDK_LAUNCH_DT(dt, gap_fwd_kernel, grid, dim3(256), (const TT*)x, (TT*)y, HW, C);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_gap_bwd(const void* dy, void* dx, int dt, int N, int HW, int C, hipStream_t st) {
  const long long total = static_cast<long long>(N) * HW * C;
  TTDK_LAUNCH_DT(dt, gap_bwd_kernel, dim3(grid_for(total)), dim3(256), (const TT*)dy, (TT*)dx, total, HW, C);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_ln_generic_fwd(const void* x, const float* g, const float* b, void* y, float* mean, float* rstd,
                                    int dt, long long rows, int H, float eps, hipStream_t st) {
  if (H <= 0 || rows <= 0) return hipErrorInvalidValue;
  dim3 grid(static_cast<unsigned>((rows + 3) / 4));
  TTDK_LAUNCH_DT(dt, ln_fwd_kernel, grid, dim3(256), (const TT*)x, g, b, (TT*)y, mean, rstd, rows, H, eps);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_ln_generic_bwd_dx(const void* dy, const void* x, const float* g, const float* mean,
                                       const float* rstd, void* dx, int dt, long long rows, int H, hipStream_t st) {
  if (H <= 0 || rows <= 0) return hipErrorInvalidValue;
  dim3 grid(static_cast<unsigned>((rows + 3) / 4));
  TTDK_LAUNCH_DT(dt, ln_bwd_dx_kernel, grid, dim3(256), (const TT*)dy, (const TT*)x, g, mean, rstd, (TT*)dx, rows, H);
  return hipGetLastError();
}

// ids: int32 (id64 = 0) or int64 (id64 = 1)
TTDK_EXPORT int ttdk_gather_generic(const void* table, const void* ids, int id64, void* out, int dt, long long n, int H,
                                    long long V, hipStream_t st) {
  const unsigned g = grid_for(n * H);
  if (dt == 0 && id64) hipLaunchKernelGGL((gather_kernel<float, long long>), dim3(g), dim3(256), 0, st, (const float*)table, (const long long*)ids, (float*)out, n, H, V);
  else if (dt == 0) hipLaunchKernelGGL((gather_kernel<float, int>), dim3(g), dim3(256), 0, st, (const float*)table, (const int*)ids, (float*)out, n, H, V);
  else if (dt == 1 && id64) hipLaunchKernelGGL((gather_kernel<bf16_t, long long>), dim3(g), dim3(256), 0, st, (const bf16_t*)table, (const long long*)ids, (bf16_t*)out, n, H, V);
  else if (dt == 1) hipLaunchKernelGGL((gather_kernel<bf16_t, int>), dim3(g), dim3(256), 0, st, (const bf16_t*)table, (const int*)ids, (bf16_t*)out, n, H, V);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// dtable (fp32 [V][H]) += scatter(dy) — accumulates, so zero it first for a fresh gradient
TTDK_EXPORT int ttdk_scatter_add_generic(const void* dy, const void* ids, int id64, float* dtable, int dt, long long n,
                                         int H, long long V, hipStream_t st) {
  const unsigned g = grid_for(n * H);
  if (dt == 0 && id64) hipLaunchKernelGGL((scatter_add_kernel<float, long long>), dim3(g), dim3(256), 0, st, (const float*)dy, (const long long*)ids, dtable, n, H, V);
  else if (dt == 0) hipLaunchKernelGGL((scatter_add_kernel<float, int>), dim3(g), dim3(256), 0, st, (const float*)dy, (const int*)ids, dtable, n, H, V);
  else if (dt == 1 && id64) hipLaunchKernelGGL((scatter_add_kernel<bf16_t, long long>), dim3(g), dim3(256), 0, st, (const bf16_t*)dy, (const long long*)ids, dtable, n, H, V);
  else if (dt == 1) hipLaunchKernelGGL((scatter_add_kernel<bf16_t, int>), dim3(g), dim3(256), 0, st, (const bf16_t*)dy, (const int*)ids, dtable, n, H, V);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_in_top_k(const void* z, const void* tgt, int id64, uint8_t* out, int dt, long long rows, int V,
                              int k, hipStream_t st) {
  if (V <= 0 || rows <= 0) return hipErrorInvalidValue;
  const dim3 g(static_cast<unsigned>((rows + 3) / 4));
  if (dt == 0 && id64) hipLaunchKernelGGL((in_top_k_kernel<float, long long>), g, dim3(256), 0, st, (const float*)z, (const long long*)tgt, out, rows, V, k);
  else if (dt == 0) hipLaunchKernelGGL((in_top_k_kernel<float, int>), g, dim3(256), 0, st, (const float*)z, (const int*)tgt, out, rows, V, k);
  else if (dt == 1 && id64) hipLaunchKernelGGL((in_top_k_kernel<bf16_t, long long>), g, dim3(256), 0, st, (const bf16_t*)z, (const long long*)tgt, out, rows, V, k);
  else if (dt == 1) hipLaunchKernelGGL((in_top_k_kernel<bf16_t, int>), g, dim3(256), 0, st, (const bf16_t*)z, (const int*)tgt, out, rows, V, k);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// op 0 = tanh, 1 = sigmoid
TTDK_EXPORT int ttdk_unary(const void* x, void* y, int dt, long long n, int op, hipStream_t st) {
  if (op < 0 || op > 1) return hipErrorInvalidValue;
  TTDK_LAUNCH_DT(dt, unary_kernel, dim3(grid_for(n)), dim3(256), (const TT*)x, (TT*)y, n, op);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_unary_bwd(const void* dy, const void* y, void* dx, int dt, long long n, int op, hipStream_t st) {
  if (op < 0 || op > 1) return hipErrorInvalidValue;
  TTDK_LAUNCH_DT(dt, unary_bwd_kernel, dim3(grid_for(n)), dim3(256), (const TT*)dy, (const TT*)y, (TT*)dx, n, op);
  return hipGetLastError();
}

// out[0] = scale * sum(x); ws holds >= ttdk_sum_blocks(n) floats
TTDK_EXPORT int ttdk_sum_blocks(long long n) {
  long long b = (n + 4095) / 4096;
  return static_cast<int>(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

TTDK_EXPORT int ttdk_sum_all(const void* x, int dt, long long n, float* ws, float scale, void* out, hipStream_t st) {
  const int nb = ttdk_sum_blocks(n);
  TTDK_LAUNCH_DT(dt, sum_partial_kernel, dim3(nb), dim3(256), (const TT*)x, n, ws);
  TTDK_LAUNCH_DT(dt, sum_final_kernel, dim3(1), dim3(256), ws, nb, scale, (TT*)out);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_fill_scaled(void* dx, int dt, long long n, const void* g, float scale, hipStream_t st) {
  TTDK_LAUNCH_DT(dt, fill_scaled_kernel, dim3(grid_for(n)), dim3(256), (TT*)dx, n, (const TT*)g, scale);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_row_scale(const void* a, const float* g, void* out, int dt, long long rows, int C, hipStream_t st) {
  const long long n = rows * C;
  TTDK_LAUNCH_DT(dt, row_scale_kernel, dim3(grid_for(n)), dim3(256), (const TT*)a, g, (TT*)out, n, C);
  return hipGetLastError();
}

// zero a device buffer on the stream (the runtime's fill, not a framework elementwise kernel)
TTDK_EXPORT int ttdk_zero(void* p, long long bytes, hipStream_t st) { return hipMemsetAsync(p, 0, bytes, st); }
// Device-to-device copy on the stream (a runtime blit, capturable as a memcpy node): small
// parameter-row gathers without a torch cat / copy kernel in the step.
TTDK_EXPORT int ttdk_copy(void* dst, const void* src, long long bytes, hipStream_t st) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
}

TTDK_EXPORT int ttdk_trace_marker(int tag, hipStream_t st) {
  hipLaunchKernelGGL(trace_marker_kernel, dim3(1), dim3(64), 0, st, tag);
  return hipGetLastError();
}
