// Element-wise / layout kernels: dtype casts, channel padding, conv weight layout changes,
// bias + activation (+ Philox dropout) forward/backward, bias-gradient column sums, add.
//
// Reference ops covered: BiasAdd F2 / BiasAddGrad G2, Elu F3 / EluGrad G6,
// dropout F4 / G5 (tf.layers.dropout(rate=0.01, training=True),
// /root/reference/distribute_training.py:57-58). Dropout keeps with probability 1-rate and
// scales by 1/(1-rate); the mask comes from counter-based Philox4x32-10 (seed, offset) so the
// backward pass regenerates it instead of storing it.
// All bf16 streams are 16 B per lane (Guideline 13).
#include "common.h"

namespace ttdk {
namespace {

inline int grid_for(long long n, int cap = 16384) {
  long long g = (n + 255) / 256;
  return static_cast<int>(g < cap ? (g < 1 ? 1 : g) : cap);
}

#define GRID_STRIDE(i, n)                                                                     \
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < (n); \
       i += static_cast<long long>(gridDim.x) * blockDim.x)

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  GRID_STRIDE(i, (n + 3) / 4) {
    const long long o = i * 4;
    if (o + 3 < n) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(x + o);
      uint2 p;
      p.x = pack_bf16x2(v[0], v[1]);
      p.y = pack_bf16x2(v[2], v[3]);
      *reinterpret_cast<uint2*>(y + o) = p;
    } else {
      for (long long j = o; j < n; ++j) y[j] = f2bf(x[j]);
    }
  }
}

// The three fp32 -> bf16 roundings every kernel uses, side by side (tests pin them bitwise to
// torch's RNE conversion): f2bf (one element), pack_bf16x2 (a pair in one v_cvt_pk_bf16_f32),
// pack8 (16-B chunk of four pairs). n % 8 == 0.
__global__ void bf16_round_probe_kernel(const float* __restrict__ x, bf16_t* __restrict__ one,
                                        uint32_t* __restrict__ pair, uint4* __restrict__ eight, long long n8) {
  GRID_STRIDE(i, n8) {
    float f[8];
    const f32x4_t a = *reinterpret_cast<const f32x4_t*>(x + 8 * i), b = *reinterpret_cast<const f32x4_t*>(x + 8 * i + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = a[j];
      f[4 + j] = b[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) one[8 * i + j] = f2bf(f[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) pair[4 * i + j] = pack_bf16x2(f[2 * j], f[2 * j + 1]);
    eight[i] = pack8(f);
  }
}

__global__ void bf16_to_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long long n) {
  GRID_STRIDE(i, n) y[i] = bf2f(x[i]);
}

// x[rows][C] (any dtype via bf16 input) -> y[rows][Cp] with zero channels C..Cp-1.
__global__ void pad_channels_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long rows, int C,
                                    int Cp) {
  GRID_STRIDE(i, rows * Cp) {
    const long long r = i / Cp;
    const int c = static_cast<int>(i - r * Cp);
    y[i] = c < C ? x[r * C + c] : static_cast<bf16_t>(0);
  }
}

// 3 -> 8 channels (RGB image -> the stem's 16-B pixel vectors): 8 pixels per thread, three
// aligned 16-B loads (8 x 3 bf16 = 48 B) and eight 16-B stores.
__global__ void pad3to8_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long groups) {
  GRID_STRIDE(i, groups) {
    const uint4* src = reinterpret_cast<const uint4*>(x) + i * 3;
    const uint4 v0 = src[0], v1 = src[1], v2 = src[2];
    const uint32_t w[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
    uint4* dst = reinterpret_cast<uint4*>(y) + i * 8;
#pragma unroll
    for (int px = 0; px < 8; ++px) {
      uint32_t e[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int k = px * 3 + c;  // bf16 index within the 24-element group
        e[c] = (w[k >> 1] >> (16 * (k & 1))) & 0xffffu;
      }
      dst[px] = make_uint4(e[0] | (e[1] << 16), e[2], 0u, 0u);
    }
  }
}

__global__ void unpad_channels_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long rows, int Cp,
                                      int C) {
  GRID_STRIDE(i, rows * C) {
    const long long r = i / C;
    const int c = static_cast<int>(i - r * C);
    y[i] = x[r * Cp + c];
  }
}

// src [A][B][C] -> dst [C][B][A] (bf16), used for conv filters [K][RS][C] -> [C][RS][K].
__global__ void transpose_aca_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int A, int B, int C) {
  __shared__ bf16_t tile[32][33];
  const int b = blockIdx.z;
  const int a0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int a = a0 + k, c = c0 + tx;
    tile[k][tx] = (a < A && c < C) ? src[(static_cast<long long>(a) * B + b) * C + c] : static_cast<bf16_t>(0);
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, a = a0 + tx;
    if (a < A && c < C) dst[(static_cast<long long>(c) * B + b) * A + a] = tile[tx][k];
  }
}

// bf16 [A][C] -> [C][A] in 8 x 8 register blocks: each thread loads 8 rows x 16 B (lanes along
// C: every load instruction of a wave reads 1 KiB of one source row), transposes in registers
// (one v_perm_b32 per output dword) and stores 8 x 16 B. The 32 x 32 LDS-tile kernel above moves
// 2 B per lane per access: at BERT-Large's weight copies (96 per step, 0.67 GB) it ran at
// ~180 GB/s on the side stream (7.4 ms per step of kernel time next to the forward).
__global__ __launch_bounds__(256) void transpose8_bf16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                            int A, int C) {
  const int cb = C / 8, ab = A / 8;
  const long long nblk = static_cast<long long>(ab) * cb;
  for (long long q = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; q < nblk;
       q += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int ai = static_cast<int>(q / cb), ci = static_cast<int>(q - static_cast<long long>(ai) * cb);
    uint32_t r[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 v = src[(static_cast<long long>(ai) * 8 + i) * cb + ci];
      r[i][0] = v.x;
      r[i][1] = v.y;
      r[i][2] = v.z;
      r[i][3] = v.w;
    }
    // output row j (source column 8 ci + j) = r[0..7][j]: dword d holds rows 2d (lo) and 2d + 1 (hi)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t o[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t lo = r[2 * d][j >> 1], hi = r[2 * d + 1][j >> 1];
        // bytes of (hi, lo): select the 16-bit half j & 1 of each
        o[d] = (j & 1) ? __builtin_amdgcn_perm(hi, lo, 0x07060302u) : __builtin_amdgcn_perm(hi, lo, 0x05040100u);
      }
      dst[(static_cast<long long>(ci) * 8 + j) * ab + ai] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

// bf16 [A][C] -> [C][A] for A, C multiples of 128: one workgroup per 128 x 128 tile. Thread
// (ai, ci) = (tid / 16, tid % 16) loads its 8 x 8 block as 8 source-row pieces of 16 B (16 lanes
// per 256-B row segment), transposes it in registers (v_perm_b32), and parks the 8 output pieces
// in an LDS image of the output tile ([128 rows][256 B], 16-B chunk c at slot c ^ ((row >> 3) &
// 15): the 8-lane ds_write_b128 groups hit 8 different slots); after one barrier every store
// instruction writes 4 whole 256-B output row segments. transpose8_bf16_kernel stores each
// lane's 16 B to a different output row (64 rows per instruction): 47 us for a 4096 x 1024 BERT
// weight, ~0.35 TB/s.
__device__ __forceinline__ void transpose128_tile(const uint4* __restrict__ src, uint4* __restrict__ dst, int A, int C,
                                                  int tile) {
  __shared__ __attribute__((aligned(16))) uint4 img[128 * 16];
  const int tiles_c = C / 128;
  const int ta = tile / tiles_c, tc = tile - ta * tiles_c;
  const int tid = threadIdx.x, ai = tid >> 4, ci = tid & 15;
  const int cb = C / 8, ab = A / 8;
  uint32_t r[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 v = src[(static_cast<long long>(ta) * 128 + ai * 8 + i) * cb + tc * 16 + ci];
    r[i][0] = v.x;
    r[i][1] = v.y;
    r[i][2] = v.z;
    r[i][3] = v.w;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t lo = r[2 * d][j >> 1], hi = r[2 * d + 1][j >> 1];
      o[d] = (j & 1) ? __builtin_amdgcn_perm(hi, lo, 0x07060302u) : __builtin_amdgcn_perm(hi, lo, 0x05040100u);
    }
    const int row = ci * 8 + j;  // output row within the tile; chunk = ai
    img[row * 16 + (ai ^ ci)] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int row = it * 16 + (tid >> 4), c = tid & 15;
    dst[(static_cast<long long>(tc) * 128 + row) * ab + ta * 16 + c] = img[row * 16 + (c ^ ((row >> 3) & 15))];
  }
}

__global__ __launch_bounds__(256) void transpose128_bf16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                              int A, int C) {
  transpose128_tile(src, dst, A, C, blockIdx.x);
}

// Many [A][C] -> [C][A] transposes (all multiples of 128) in ONE launch: block b takes tile
// b - tile_begin of the last entry whose tile_begin <= b (binary search). BERT refreshes 96
// transposed weight copies per step; as separate launches of 64-256 workgroups each they ran
// one after another between the forward GEMMs (each of which holds every CU's register file).
struct TransposeEntry {
  const uint4* src;
  uint4* dst;
  int A, C, tile_begin, pad;
};
__global__ __launch_bounds__(256) void transpose128_batch_kernel(const TransposeEntry* __restrict__ tab, int n) {
  const int bid = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].tile_begin <= bid) lo = mid;
    else hi = mid - 1;
  }
  const TransposeEntry e = tab[lo];
  transpose128_tile(e.src, e.dst, e.A, e.C, bid - e.tile_begin);
}

// fp32 [A][B][C] -> fp32 [C][B][A] (checkpoint layout conversions: KRSC <-> RSCK done as 2-D)
__global__ void transpose2d_f32_kernel(const float* __restrict__ src, float* __restrict__ dst, int R, int C) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < R && c < C) ? src[static_cast<long long>(r) * C + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (r < R && c < C) dst[static_cast<long long>(c) * R + r] = tile[tx][k];
  }
}

enum Act : int { kNone = 0, kRelu = 1, kGelu = 2, kElu = 3 };

__device__ __forceinline__ float act_fwd(float x, int act) {
  switch (act) {
    case kRelu: return relu(x);
    case kGelu: return 0.5f * x * (1.f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
    case kElu: return x > 0.f ? x : expm1f(x);
    default: return x;
  }
}

// derivative given pre-activation z (and post-activation a for ELU: d = a + 1 for z <= 0)
__device__ __forceinline__ float act_grad(float z, int act) {
  switch (act) {
    case kRelu: return z > 0.f ? 1.f : 0.f;
    case kGelu: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      const float u = k0 * (z + k1 * z * z * z);
      const float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * k0 * (1.f + 3.f * k1 * z * z);
    }
    case kElu: return z > 0.f ? 1.f : expf(z);
    default: return 1.f;
  }
}

__device__ __forceinline__ bool keep_bit(uint64_t seed, uint64_t offset, long long idx, float rate) {
  uint32_t r[4];
  Philox::gen(seed, offset, static_cast<uint64_t>(idx >> 2), r);
  return Philox::uniform(r[idx & 3]) >= rate;
}

// y = dropout(act(x + bias)), x/y [rows][C] (T = float or bf16). Also writes z = x + bias if
// zout (needed by the backward for GELU/ELU).
template <typename T>
__device__ __forceinline__ float ldv(const T* p, long long i) {
  if constexpr (sizeof(T) == 2)
    return bf2f(p[i]);
  else
    return p[i];
}
template <typename T>
__device__ __forceinline__ void stv(T* p, long long i, float v) {
  if constexpr (sizeof(T) == 2)
    p[i] = f2bf(v);
  else
    p[i] = v;
}

template <typename T>
__global__ void bias_act_dropout_fwd_kernel(const T* __restrict__ x, const float* __restrict__ bias,
                                            T* __restrict__ y, long long n, int C, int act, float rate, uint64_t seed,
                                            uint64_t offset) {
  const float scale = rate > 0.f ? 1.f / (1.f - rate) : 1.f;
  GRID_STRIDE(i, n) {
    float v = ldv(x, i) + (bias ? bias[i % C] : 0.f);
    v = act_fwd(v, act);
    if (rate > 0.f) v = keep_bit(seed, offset, i, rate) ? v * scale : 0.f;
    stv(y, i, v);
  }
}

// dx = dy * dropout_mask * act'(z) with z = x + bias recomputed from the pre-activation x.
template <typename T>
__global__ void bias_act_dropout_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                            const float* __restrict__ bias, T* __restrict__ dx, long long n, int C,
                                            int act, float rate, uint64_t seed, uint64_t offset) {
  const float scale = rate > 0.f ? 1.f / (1.f - rate) : 1.f;
  GRID_STRIDE(i, n) {
    float g = ldv(dy, i);
    if (rate > 0.f) g = keep_bit(seed, offset, i, rate) ? g * scale : 0.f;
    const float z = ldv(x, i) + (bias ? bias[i % C] : 0.f);
    stv(dx, i, g * act_grad(z, act));
  }
}

// Column sums out[c] (+)= sum_r x[r][c] (bias gradients). grid.x over column chunks, grid.y row
// slices; each slice writes its partial row ws[slice][C] and colsum_fold_kernel adds the
// slices in a fixed order (no float atomics: bitwise reproducible). With one slice the
// kernels write `out` directly (honouring beta).
template <typename T>
__global__ void colsum_kernel(const T* __restrict__ x, long long rows, int C, float* __restrict__ dst,
                              long long rows_per_slice, int beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long long r0 = blockIdx.y * rows_per_slice, r1 = min(rows, r0 + rows_per_slice);
  float s = 0.f;
  for (long long r = r0; r < r1; ++r) s += ldv(x, r * C + c);
  float* d = dst + static_cast<long long>(blockIdx.y) * C + c;
  *d = s + (beta ? *d : 0.f);
}

__global__ void colsum_fold_kernel(const float* __restrict__ ws, int slices, int C, float* __restrict__ out,
                                   int beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < slices; ++k) s += ws[static_cast<long long>(k) * C + c];
  out[c] = s + (beta ? out[c] : 0.f);
}

// The same fold for C % 4 == 0 with the slices spread over the block: 32 columns per block
// (8 threads x float4) x 32 slice lanes, fixed-order partial sums per lane then a fixed-order
// LDS reduction (bitwise reproducible). The one-thread-per-column fold above walks up to 256
// slices serially on a handful of CUs: ~40 us per BERT bias gradient.
__global__ __launch_bounds__(256) void colsum_fold4_kernel(const float* __restrict__ ws, int slices, int C,
                                                           float* __restrict__ out, int beta) {
  __shared__ f32x4_t red[32][9];
  const int cl = threadIdx.x & 7, sl = threadIdx.x >> 3;
  const int c = blockIdx.x * 32 + cl * 4;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
#pragma unroll 4
    for (int k = sl; k < slices; k += 32) s += *reinterpret_cast<const f32x4_t*>(ws + static_cast<long long>(k) * C + c);
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && c < C) {
    f32x4_t t = red[0][cl];
#pragma unroll
    for (int k = 1; k < 32; ++k) t += red[k][cl];
    if (beta) t += *reinterpret_cast<const f32x4_t*>(out + c);
    *reinterpret_cast<f32x4_t*>(out + c) = t;
  }
}

// Vectorised bf16 column sum (C % 8 == 0): a 256-thread block covers 256 columns (32 threads
// x 8 columns, 16-B loads, 512 contiguous bytes per row) x 8 row lanes over its row slice;
// the 8 row lanes reduce through LDS and each block writes its 256 sums to its slice row.
__global__ __launch_bounds__(256) void colsum_bf16x8_kernel(const bf16_t* __restrict__ x, long long rows, int C,
                                                            float* __restrict__ dst, long long rows_per_slice,
                                                            int beta) {
  __shared__ float red[8][257];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 256 + cl * 8;
  const long long r0 = blockIdx.y * rows_per_slice, r1 = min(rows, r0 + rows_per_slice);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    long long r = r0 + rl;
    for (; r + 24 < r1; r += 32) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(x + (r + 8 * u) * C + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    }
    for (; r < r1; r += 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + r * C + c), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cl * 8 + j] = s[j];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][threadIdx.x];
    float* d = dst + static_cast<long long>(blockIdx.y) * C + col;
    *d = t + (beta ? *d : 0.f);
  }
}

__global__ void add_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                long long n8, float alpha, float beta) {
  GRID_STRIDE(i, n8) {
    float fa[8], fb[8];
    unpack8(reinterpret_cast<const uint4*>(a)[i], fa);
    unpack8(reinterpret_cast<const uint4*>(b)[i], fb);
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] = alpha * fa[j] + beta * fb[j];
    reinterpret_cast<uint4*>(y)[i] = pack8(fa);
  }
}

// fp8 (OCP e4m3fn / e5m2, gfx950 native) quantisation with a per-tensor scale:
// q = sat(x * scale); amax (optional) accumulates max|x| for delayed scaling.
__global__ void amax_bf16_kernel(const bf16_t* __restrict__ x, long long n, float* __restrict__ amax) {
  float m = 0.f;
  GRID_STRIDE(i, n) m = fmaxf(m, fabsf(bf2f(x[i])));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(m));
}

__global__ void quant_fp8_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q, long long n,
                                 const float* __restrict__ scale, int e5m2) {
  const float s = *scale;
  const float lim = e5m2 ? 57344.f : 448.f;
  GRID_STRIDE(i, n) {
    const float v = fminf(fmaxf(bf2f(x[i]) * s, -lim), lim);
    // gfx950 v_cvt_pk_{fp8,bf8}_f32 produce OCP e4m3fn / e5m2 (round-to-nearest-even)
    const int packed = e5m2 ? __builtin_amdgcn_cvt_pk_bf8_f32(v, v, 0, false) : __builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
    q[i] = static_cast<uint8_t>(packed & 0xff);
  }
}

__global__ void dequant_fp8_kernel(const uint8_t* __restrict__ q, bf16_t* __restrict__ x, long long n,
                                   const float* __restrict__ scale, int e5m2) {
  const float inv = 1.f / *scale;
  GRID_STRIDE(i, n) {
    const int b = q[i];
    const float v = e5m2 ? __builtin_amdgcn_cvt_f32_bf8(b, 0) : __builtin_amdgcn_cvt_f32_fp8(b, 0);
    x[i] = f2bf(v * inv);
  }
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

TTDK_EXPORT int ttdk_f32_to_bf16(const float* x, bf16_t* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, x, y, n);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_bf16_round_probe(const float* x, bf16_t* one, uint32_t* pair, void* eight, long long n,
                                      hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bf16_round_probe_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, x, one, pair,
                     static_cast<uint4*>(eight), n / 8);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_bf16_to_f32(const bf16_t* x, float* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_pad_channels(const bf16_t* x, bf16_t* y, long long rows, int C, int Cp, hipStream_t st) {
  if (C == 3 && Cp == 8 && rows % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
    hipLaunchKernelGGL(pad3to8_kernel, dim3(grid_for(rows / 8)), dim3(256), 0, st, x, y, rows / 8);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pad_channels_kernel, dim3(grid_for(rows * Cp)), dim3(256), 0, st, x, y, rows, C, Cp);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_unpad_channels(const bf16_t* x, bf16_t* y, long long rows, int Cp, int C, hipStream_t st) {
  hipLaunchKernelGGL(unpad_channels_kernel, dim3(grid_for(rows * C)), dim3(256), 0, st, x, y, rows, Cp, C);
  return hipGetLastError();
}

// tab: n TransposeEntry rows (device memory, 32 B each; src / dst 16-B aligned, A and C
// multiples of 128, tile_begin the running sum of (A/128)*(C/128)); tiles: the total
TTDK_EXPORT int ttdk_transpose128_batch_bf16(const void* tab, int n, int tiles, hipStream_t st) {
  if (n <= 0 || tiles <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose128_batch_kernel, dim3(tiles), dim3(256), 0, st, static_cast<const TransposeEntry*>(tab), n);
  return hipGetLastError();
}

// [A][B][C] -> [C][B][A] bf16
TTDK_EXPORT int ttdk_transpose_aca_bf16(const bf16_t* src, bf16_t* dst, int A, int B, int C, hipStream_t st) {
  if (B == 1 && A % 128 == 0 && C % 128 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    hipLaunchKernelGGL(transpose128_bf16_kernel, dim3((A / 128) * (C / 128)), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), A, C);
    return hipGetLastError();
  }
  if (B == 1 && A % 8 == 0 && C % 8 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const long long nblk = static_cast<long long>(A / 8) * (C / 8);
    hipLaunchKernelGGL(transpose8_bf16_kernel, dim3(grid_for(nblk, 4096)), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), A, C);
    return hipGetLastError();
  }
  dim3 grid((C + 31) / 32, (A + 31) / 32, B);
  hipLaunchKernelGGL(transpose_aca_kernel, grid, dim3(256), 0, st, src, dst, A, B, C);
  return hipGetLastError();
}

// Every data-gradient filter operand of a network in ONE launch (instead of one transpose per
// conv on the backward's critical chain, plus s*s sub-pixel gathers per strided conv): entry e
// turns the bf16 filter [K][R][S][C] at src + src_off into [C][Tr][Ts][K] at dst + dst_off,
// taking taps r = r0 + tr*s, q = s0 + ts*s (s = 1, full R x S: the plain [C,R,S,K] transpose;
// s > 1: one sub-pixel phase of a strided dgrad, see conv_dgrad.hip). Blocks walk the
// concatenated 32x32 (K, C) tiles of all entries' taps; tile_begin is each entry's first tile.
struct WPrepEntry {
  long long src_off, dst_off;
  int K, R, S, C, s, r0, Tr, s0, Ts, tile_begin;
};

__global__ __launch_bounds__(256) void wprep_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                    const WPrepEntry* __restrict__ tab, int n) {
  __shared__ bf16_t tile[32][33];
  const int bid = blockIdx.x;
  int e = 0;
  while (e + 1 < n && tab[e + 1].tile_begin <= bid) ++e;
  const WPrepEntry t = tab[e];
  const int kt = (t.K + 31) / 32, ct = (t.C + 31) / 32;
  int rel = bid - t.tile_begin;
  const int tap = rel / (kt * ct);
  rel -= tap * kt * ct;
  const int k0 = (rel / ct) * 32, c0 = (rel % ct) * 32;
  const int tr = tap / t.Ts, ts = tap % t.Ts;
  const int r = t.r0 + tr * t.s, q = t.s0 + ts * t.s;
  const bf16_t* s_ = src + t.src_off + (static_cast<long long>(r) * t.S + q) * t.C;
  bf16_t* d_ = dst + t.dst_off + static_cast<long long>(tap) * t.K;
  const long long sld = static_cast<long long>(t.R) * t.S * t.C;  // src stride between k rows
  const long long dld = static_cast<long long>(t.Tr) * t.Ts * t.K;  // dst stride between c rows
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int k = k0 + i, c = c0 + tx;
    tile[i][tx] = (k < t.K && c < t.C) ? s_[k * sld + c] : static_cast<bf16_t>(0);
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, k = k0 + tx;
    if (k < t.K && c < t.C) d_[c * dld + k] = tile[tx][i];
  }
}

TTDK_EXPORT int ttdk_wprep(const bf16_t* src, bf16_t* dst, const void* tab, int n, int tiles, hipStream_t st) {
  if (n <= 0 || tiles <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wprep_kernel, dim3(tiles), dim3(256), 0, st, src, dst, static_cast<const WPrepEntry*>(tab), n);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_transpose2d_f32(const float* src, float* dst, int R, int C, hipStream_t st) {
  dim3 grid((C + 31) / 32, (R + 31) / 32);
  hipLaunchKernelGGL(transpose2d_f32_kernel, grid, dim3(256), 0, st, src, dst, R, C);
  return hipGetLastError();
}

// dtype 0 = fp32, 1 = bf16
TTDK_EXPORT int ttdk_bias_act_dropout_fwd(const void* x, const float* bias, void* y, long long n, int C, int act,
                                          float rate, unsigned long long seed, unsigned long long offset, int dtype,
                                          hipStream_t st) {
  if (dtype == 0)
    hipLaunchKernelGGL(bias_act_dropout_fwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st,
                       static_cast<const float*>(x), bias, static_cast<float*>(y), n, C, act, rate, seed, offset);
  else
    hipLaunchKernelGGL(bias_act_dropout_fwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st,
                       static_cast<const bf16_t*>(x), bias, static_cast<bf16_t*>(y), n, C, act, rate, seed, offset);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_bias_act_dropout_bwd(const void* dy, const void* x, const float* bias, void* dx, long long n,
                                          int C, int act, float rate, unsigned long long seed,
                                          unsigned long long offset, int dtype, hipStream_t st) {
  if (dtype == 0)
    hipLaunchKernelGGL(bias_act_dropout_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st,
                       static_cast<const float*>(dy), static_cast<const float*>(x), bias, static_cast<float*>(dx), n, C,
                       act, rate, seed, offset);
  else
    hipLaunchKernelGGL(bias_act_dropout_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st,
                       static_cast<const bf16_t*>(dy), static_cast<const bf16_t*>(x), bias, static_cast<bf16_t*>(dx), n,
                       C, act, rate, seed, offset);
  return hipGetLastError();
}

// out[C] = (beta ? out : 0) + column sums of x[rows][C]
static void colsum_plan(long long rows, int C, int dtype, bool vec, long long* slices, long long* per) {
  long long sl;
  if (vec) {
    const int cblocks = (C + 255) / 256;
    sl = (1024 + cblocks - 1) / cblocks;            // ~1024 blocks
    const long long max_slices = (rows + 63) / 64;  // >= 64 rows per slice
    if (sl > max_slices) sl = max_slices;
  } else {
    sl = (rows + 127) / 128;
    if (sl > 256) sl = 256;
  }
  if (sl < 1) sl = 1;
  *per = (rows + sl - 1) / sl;
  *slices = (rows + *per - 1) / *per;
  if (*slices < 1) *slices = 1;
}

// Floats of workspace ttdk_colsum needs (covers both the vector and the scalar plan).
TTDK_EXPORT long long ttdk_colsum_ws_floats(long long rows, int C, int dtype) {
  long long s1, s2, per;
  colsum_plan(rows, C, dtype, true, &s1, &per);
  colsum_plan(rows, C, dtype, false, &s2, &per);
  const long long sl = s1 > s2 ? s1 : s2;
  return sl > 1 ? sl * C : 0;
}

TTDK_EXPORT int ttdk_colsum(const void* x, long long rows, int C, float* out, int beta, int dtype, float* ws,
                            hipStream_t st) {
  const bool vec = dtype == 1 && C % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  long long slices, per;
  colsum_plan(rows, C, dtype, vec, &slices, &per);
  if (slices > 1 && !ws) return hipErrorInvalidValue;
  float* dst = slices > 1 ? ws : out;
  const int bt = slices > 1 ? 0 : beta;
  if (vec) {
    hipLaunchKernelGGL(colsum_bf16x8_kernel, dim3((C + 255) / 256, static_cast<int>(slices)), dim3(256), 0, st,
                       static_cast<const bf16_t*>(x), rows, C, dst, per, bt);
  } else {
    dim3 grid((C + 255) / 256, static_cast<int>(slices));
    if (dtype == 0)
      hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, static_cast<const float*>(x), rows, C, dst, per,
                         bt);
    else
      hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(x), rows, C, dst,
                         per, bt);
  }
  if (slices > 1) {
    if (C % 4 == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0)
      hipLaunchKernelGGL(colsum_fold4_kernel, dim3((C + 31) / 32), dim3(256), 0, st, ws, static_cast<int>(slices), C, out,
                         beta);
    else
      hipLaunchKernelGGL(colsum_fold_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, static_cast<int>(slices), C,
                         out, beta);
  }
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_add_bf16(const bf16_t* a, const bf16_t* b, bf16_t* y, long long n, float alpha, float beta,
                              hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(add_bf16_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, a, b, y, n / 8, alpha, beta);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_amax_bf16(const bf16_t* x, long long n, float* amax, int reset, hipStream_t st) {
  if (reset) {
    hipError_t e = hipMemsetAsync(amax, 0, sizeof(float), st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(amax_bf16_kernel, dim3(grid_for(n, 2048)), dim3(256), 0, st, x, n, amax);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_quant_fp8(const bf16_t* x, uint8_t* q, long long n, const float* scale, int e5m2, hipStream_t st) {
  hipLaunchKernelGGL(quant_fp8_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, q, n, scale, e5m2);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_dequant_fp8(const uint8_t* q, bf16_t* x, long long n, const float* scale, int e5m2,
                                 hipStream_t st) {
  hipLaunchKernelGGL(dequant_fp8_kernel, dim3(grid_for(n)), dim3(256), 0, st, q, x, n, scale, e5m2);
  return hipGetLastError();
}
