// Transformer (BERT) element-wise / normalisation kernels for gfx950 (SURVEY.md §2.6 [NS]
// BERT-Large set; BASELINE.json config 4):
//   * LayerNorm forward/backward fused with the residual add and the two dropouts of a
//     post-LN block:  s = res + drop_in(x);  y = drop_out(LN(s) * gamma + beta)
//     (drop_in = hidden dropout of a sub-layer output, drop_out = embedding dropout). One wave
//     per 1024-wide row, whole row in registers, one HBM pass each way; dgamma/dbeta as
//     per-workgroup partial rows + a column reduce (no float atomics);
//   * embedding gather (word + position + token-type) and its backward (word rows scatter-add
//     with fp32 atomics, position/type grads reduced without contention);
//   * row gather / scatter (masked-LM positions), valid-label count, vocabulary-wide
//     softmax cross-entropy with ignore-index and in-place gradient, and bias-free tanh.
// Dropout masks come from the counter hash in tile_common.h keyed by device (seed, step).
#include "tile_common.h"

namespace ttdk {
namespace {

__device__ __forceinline__ uint4 ldg16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

struct DropSpec {
  const long long* rng;
  uint32_t site_in, site_out;
  uint32_t thr_in, thr_out;
  float scale_in, scale_out;
};

// ------------------------------------------------------------------ LayerNorm forward
// H = NV * 512; wave w of a 256-thread block owns row blockIdx.x * 4 + w; lane holds 16-B
// chunks lane + 64 * v.
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                     bf16_t* __restrict__ s_out, bf16_t* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     int rows, float eps, DropSpec dsp) {
  constexpr int H = NV * 512;
  const int lane = threadIdx.x & 63;
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint32_t kin = dsp.thr_in ? drop_key(dsp.rng, dsp.site_in) : 0u;
  const uint32_t kout = dsp.thr_out ? drop_key(dsp.rng, dsp.site_out) : 0u;
  float f[NV][8];
  float sum = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = (lane + 64 * v) * 8;
    unpack8(ldg16(x + row * H + c), f[v]);
    if (dsp.thr_in) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        f[v][j] = drop_keep(kin, static_cast<unsigned long long>(row) * H + c + j, dsp.thr_in) ? f[v][j] * dsp.scale_in
                                                                                                  : 0.f;
    }
    if (res) {
      float r[8];
      unpack8(ldg16(res + row * H + c), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[v][j] += r[j];
    }
    // statistics of the bf16 value that backward will re-read
    const uint4 pk = pack8(f[v]);
    unpack8(pk, f[v]);
    if (s_out) *reinterpret_cast<uint4*>(s_out + row * H + c) = pk;
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += f[v][j];
  }
  const float mean = wave_sum(sum) * (1.f / H);
  float var = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = f[v][j] - mean;
      var += d * d;
    }
  const float rstd = rsqrtf(wave_sum(var) * (1.f / H) + eps);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = (lane + 64 * v) * 8;
    float o[8], gw[8], bw[8];
    *reinterpret_cast<f32x4_t*>(gw) = *reinterpret_cast<const f32x4_t*>(gamma + c);
    *reinterpret_cast<f32x4_t*>(gw + 4) = *reinterpret_cast<const f32x4_t*>(gamma + c + 4);
    *reinterpret_cast<f32x4_t*>(bw) = *reinterpret_cast<const f32x4_t*>(beta + c);
    *reinterpret_cast<f32x4_t*>(bw + 4) = *reinterpret_cast<const f32x4_t*>(beta + c + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (f[v][j] - mean) * rstd * gw[j] + bw[j];
      if (dsp.thr_out)
        o[j] = drop_keep(kout, static_cast<unsigned long long>(row) * H + c + j, dsp.thr_out) ? o[j] * dsp.scale_out
                                                                                               : 0.f;
    }
    *reinterpret_cast<uint4*>(y + row * H + c) = pack8(o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// ------------------------------------------------------------------ LayerNorm backward
// ds = dL/ds (goes to the residual branch), dx = ds * mask_in * scale_in (the sub-layer
// output gradient; null when there is no input dropout). part: [gridDim.x][2][H] partial
// (dgamma, dbeta) rows.
// Each row needs two dependent wave reductions between its loads and its stores, so one wave
// per SIMD working one row at a time (the first version) was latency-bound at ~0.6 TB/s.
// H = 512: 16 waves per block (4 per SIMD, < 128 VGPRs), one row each; H >= 1024: 8 waves
// per block (2 per SIMD, ~230 VGPRs at H = 1024) with two rows in flight per wave and their
// reductions interleaved (16 x 1 would spill at H = 1024).

__device__ __forceinline__ void wave_sum4(float& a, float& b, float& c, float& d) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c += __shfl_xor(c, o, 64);
    d += __shfl_xor(d, o, 64);
  }
}

template <int NV, int W, int U, bool PF = false>  // W waves per block, U rows in flight per wave, PF: prefetch
__global__ __launch_bounds__(W * 64) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                             const float* __restrict__ mean_in,
                                                             const float* __restrict__ rstd_in,
                                                             const float* __restrict__ gamma, bf16_t* __restrict__ ds_out,
                                                             bf16_t* __restrict__ dx_out, float* __restrict__ part,
                                                             int rows, int rows_per_block, DropSpec dsp) {
  constexpr int H = NV * 512, CH = 512;  // a wave's columns for one v: lane * 8 + j
  __shared__ __attribute__((aligned(16))) float red[W][2][CH];  // 64 KB
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t kin = dsp.thr_in ? drop_key(dsp.rng, dsp.site_in) : 0u;
  const uint32_t kout = dsp.thr_out ? drop_key(dsp.rng, dsp.site_out) : 0u;
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[v][j] = db[v][j] = 0.f;
  // gamma is re-read (L1/L2-resident) where used rather than held in 8*NV VGPRs
  auto load_g = [&](int c, float (&gm)[8]) {
    *reinterpret_cast<f32x4_t*>(gm) = *reinterpret_cast<const f32x4_t*>(gamma + c);
    *reinterpret_cast<f32x4_t*>(gm + 4) = *reinterpret_cast<const f32x4_t*>(gamma + c + 4);
  };
  const long long r0 = static_cast<long long>(blockIdx.x) * rows_per_block;
  const long long r1 = min(static_cast<long long>(rows), r0 + rows_per_block);
  // dy after the output dropout (recomputed in both passes; the mask is a hash, not stored)
  auto load_d = [&](const uint4& pk, long long row, int c, float (&d)[8]) {
    unpack8(pk, d);
    if (dsp.thr_out) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        d[j] = drop_keep(kout, static_cast<unsigned long long>(row) * H + c + j, dsp.thr_out) ? d[j] * dsp.scale_out : 0.f;
    }
  };
  // rows of the next iteration are loaded one iteration ahead (PF): a wave otherwise had no load
  // in flight while it reduced and stored its rows, and the kernel waited on memory 69 % of its
  // wave cycles at ~3.4 TB/s (rocprofv3 --pmc, tools/pmc_ln.sh)
  uint4 nd[U][NV], ns[U][NV];
  float nmean[U], nrstd[U];
  auto fetch = [&](long long ra) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = ra + u * W;
      const bool h = r < r1;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = (lane + 64 * v) * 8;
        nd[u][v] = h ? ldg16(dy + r * H + c) : make_uint4(0, 0, 0, 0);
        ns[u][v] = h ? ldg16(s + r * H + c) : make_uint4(0, 0, 0, 0);
      }
      nmean[u] = h ? mean_in[r] : 0.f;
      nrstd[u] = h ? rstd_in[r] : 0.f;
    }
  };
  if (PF && r0 + w < r1) fetch(r0 + w);
#pragma unroll 1
  for (long long ra = r0 + w; ra < r1; ra += U * W) {
    long long rw[U];
    bool has[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rw[u] = ra + u * W;
      has[u] = rw[u] < r1;
    }
    uint4 pd[U][NV], ps[U][NV];
    float mean[U], rstd[U];
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          pd[u][v] = nd[u][v];
          ps[u][v] = ns[u][v];
        }
        mean[u] = nmean[u];
        rstd[u] = nrstd[u];
      }
      if (ra + U * W < r1) fetch(ra + U * W);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int c = (lane + 64 * v) * 8;
          pd[u][v] = has[u] ? ldg16(dy + rw[u] * H + c) : make_uint4(0, 0, 0, 0);
          ps[u][v] = has[u] ? ldg16(s + rw[u] * H + c) : make_uint4(0, 0, 0, 0);
        }
        mean[u] = has[u] ? mean_in[rw[u]] : 0.f;
        rstd[u] = has[u] ? rstd_in[rw[u]] : 0.f;
      }
    }
    float c1[U], c2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c1[u] = c2[u] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = (lane + 64 * v) * 8;
        float d[8], sv[8], gm[8];
        load_d(pd[u][v], rw[u], c, d);
        unpack8(ps[u][v], sv);
        load_g(c, gm);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (sv[j] - mean[u]) * rstd[u];
          dg[v][j] += d[j] * xh;  // a missing second row has d == 0
          db[v][j] += d[j];
          const float g = d[j] * gm[j];
          c1[u] += g;
          c2[u] += g * xh;
        }
      }
    // opaque to the optimiser: pass 2 re-derives d / x-hat from the packed rows instead of
    // keeping pass 1's unpacked floats alive across the reductions (which spilled)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        asm volatile("" : "+v"(pd[u][v].x), "+v"(pd[u][v].y), "+v"(pd[u][v].z), "+v"(pd[u][v].w));
        asm volatile("" : "+v"(ps[u][v].x), "+v"(ps[u][v].y), "+v"(ps[u][v].z), "+v"(ps[u][v].w));
      }
    if constexpr (U == 2) {
      wave_sum4(c1[0], c2[0], c1[1], c2[1]);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c1[u] = wave_sum(c1[u]);
        c2[u] = wave_sum(c2[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!has[u]) break;
      const float m1 = c1[u] * (1.f / H), m2 = c2[u] * (1.f / H);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = (lane + 64 * v) * 8;
        float d[8], sv[8], o[8], gm[8];
        load_d(pd[u][v], rw[u], c, d);
        unpack8(ps[u][v], sv);
        load_g(c, gm);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (sv[j] - mean[u]) * rstd[u];
          o[j] = rstd[u] * (d[j] * gm[j] - m1 - xh * m2);
        }
        *reinterpret_cast<uint4*>(ds_out + rw[u] * H + c) = pack8(o);
        if (dx_out) {
          if (dsp.thr_in) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
              o[j] = drop_keep(kin, static_cast<unsigned long long>(rw[u]) * H + c + j, dsp.thr_in) ? o[j] * dsp.scale_in
                                                                                                    : 0.f;
          }
          *reinterpret_cast<uint4*>(dx_out + rw[u] * H + c) = pack8(o);
        }
      }
    }
  }
  // block reduce of (dg, db) over the W waves in fixed order, one 512-column slice (v) at a time
  float* out = part + static_cast<long long>(blockIdx.x) * 2 * H;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    __syncthreads();
    *reinterpret_cast<f32x4_t*>(&red[w][0][lane * 8]) = *reinterpret_cast<const f32x4_t*>(dg[v]);
    *reinterpret_cast<f32x4_t*>(&red[w][0][lane * 8 + 4]) = *reinterpret_cast<const f32x4_t*>(dg[v] + 4);
    *reinterpret_cast<f32x4_t*>(&red[w][1][lane * 8]) = *reinterpret_cast<const f32x4_t*>(db[v]);
    *reinterpret_cast<f32x4_t*>(&red[w][1][lane * 8 + 4]) = *reinterpret_cast<const f32x4_t*>(db[v] + 4);
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * CH; i += W * 64) {
      const int which = i / CH, col = i % CH;
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < W; ++k) t += red[k][which][col];
      out[which * H + v * CH + col] = t;
    }
  }
}

// out[c] (+)= sum_b part[b * stride + c] for c < C (C % 4 == 0, stride % 4 == 0).
__global__ __launch_bounds__(256) void colreduce_kernel(const float* __restrict__ part, int nb, int C, int stride,
                                                        float* __restrict__ out, int beta) {
  // 64 row lanes x 4 column vectors (16 columns) per block: C / 16 blocks (128 for BERT-Large's
  // [dgamma | dbeta] rows) with every lane's rows in flight at once; the previous 16 x 64-column
  // layout ran 32 blocks of 16 dependent loads per lane (53 us for a 2 MB slab, now latency ~ 1 load)
  __shared__ f32x4_t red[64][5];
  const int cv = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int c = blockIdx.x * 16 + cv * 4;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int b = rl;
    for (; b + 192 < nb; b += 256) {
      f32x4_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(part + static_cast<long long>(b + 64 * u) * stride + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; b < nb; b += 64) s += *reinterpret_cast<const f32x4_t*>(part + static_cast<long long>(b) * stride + c);
  }
  red[rl][cv] = s;
  __syncthreads();
#pragma unroll
  for (int h = 32; h > 0; h >>= 1) {  // fixed-order tree (deterministic)
    if (rl < h) red[rl][cv] += red[rl + h][cv];
    __syncthreads();
  }
  if (rl == 0 && c < C) {
    const f32x4_t t = red[0][cv];
    f32x4_t* o = reinterpret_cast<f32x4_t*>(out + c);
    *o = beta ? *o + t : t;
  }
}

// ------------------------------------------------------------------ embeddings
// s[row] = word[ids[row]] + pos[row % S] + type[tt[row]]   (bf16 tables [*, H])
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int* __restrict__ ids, const int* __restrict__ tt,
                                                        const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                                        const bf16_t* __restrict__ typ, bf16_t* __restrict__ s,
                                                        long long rows, int S, int H) {
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const long long id = ids[row];
  const int p = static_cast<int>(row % S);
  const int t = tt ? tt[row] : 0;
  for (int c = lane * 8; c < H; c += 512) {
    float a[8], b[8], d[8];
    unpack8(ldg16(word + id * H + c), a);
    unpack8(ldg16(pos + static_cast<long long>(p) * H + c), b);
    unpack8(ldg16(typ + static_cast<long long>(t) * H + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += b[j] + d[j];
    *reinterpret_cast<uint4*>(s + row * H + c) = pack8(a);
  }
}

// dword[ids[row]] += ds[row]  (fp32 atomics; rows of distinct tokens rarely collide). Lane l of
// a wave adds column c0 + l: every atomic instruction covers 256 contiguous bytes of one row.
// (Lane-owns-8-columns, as the loads would like, put each instruction's 64 lanes on 64
// different 32-B pieces: 2.1 ms for BERT-Large b128's 65536 x 1024 rows.)
__global__ __launch_bounds__(256) void embed_bwd_word_kernel(const bf16_t* __restrict__ ds, const int* __restrict__ ids,
                                                             float* __restrict__ dword, long long rows, int H) {
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const long long id = ids[row];
  const unsigned short* src = reinterpret_cast<const unsigned short*>(ds) + row * H;
  float* dst = dword + id * H;
  for (int c0 = 0; c0 < H; c0 += 512) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j * 64 + lane;
      a[j] = c < H ? __uint_as_float(static_cast<uint32_t>(src[c]) << 16) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j * 64 + lane;
      if (c < H) atomicAdd(dst + c, a[j]);
    }
  }
}

// dpos[p] (+)= sum_b ds[b*S + p]; dtype[t] (+)= sum over rows with tt == t (T <= 4), via
// per-thread register sums over a row slice and one atomic per (type, column, block).
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(const bf16_t* __restrict__ ds, float* __restrict__ dpos,
                                                            int B, int S, int H, int beta) {
  const long long gid = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;  // (p, chunk)
  const int chunks = H / 8;
  if (gid >= static_cast<long long>(S) * chunks) return;
  const int p = static_cast<int>(gid / chunks), c = static_cast<int>(gid % chunks) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
    float a[8];
    unpack8(ldg16(ds + (static_cast<long long>(b) * S + p) * H + c), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += a[j];
  }
  float* o = dpos + static_cast<long long>(p) * H + c;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = beta ? o[j] + acc[j] : acc[j];
}

__global__ __launch_bounds__(256) void embed_bwd_type_kernel(const bf16_t* __restrict__ ds, const int* __restrict__ tt,
                                                             float* __restrict__ dtype, long long rows, int H, int T,
                                                             int rows_per_block) {
  const int chunks = H / 8;
  const int c = (threadIdx.x % chunks) * 8;  // requires H / 8 <= 256 chunks handled per pass
  const int rsub = threadIdx.x / chunks, rstep = 256 / chunks;
  float acc[4][8];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  const long long r0 = static_cast<long long>(blockIdx.x) * rows_per_block;
  const long long r1 = min(rows, r0 + rows_per_block);
  for (long long row = r0 + rsub; row < r1; row += rstep) {
    const int t = tt ? tt[row] : 0;
    float a[8];
    unpack8(ldg16(ds + row * H + c), a);
#pragma unroll
    for (int tt2 = 0; tt2 < 4; ++tt2)
      if (tt2 == t)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[tt2][j] += a[j];
  }
  for (int t = 0; t < T && t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(dtype + static_cast<long long>(t) * H + c + j, acc[t][j]);
}

// ------------------------------------------------------------------ row gather / scatter
// Row r reads source row (idx ? idx[r] : 0) + (r / per) * gs: with per = positions per sequence
// and gs = the sequence length, the MLM / CLS gathers index [B*S, H] directly from the batch's
// per-sequence positions (no per-step offset tensor built by framework kernels).
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16_t* __restrict__ src, long long lds_,
                                                          const int* __restrict__ idx, int per, long long gs,
                                                          bf16_t* __restrict__ dst, int n, int H) {
  const long long r = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const long long from = (idx ? idx[r] : 0) + (r / per) * gs;
  for (int c = (threadIdx.x & 63) * 8; c < H; c += 512)
    *reinterpret_cast<uint4*>(dst + r * H + c) = ldg16(src + from * lds_ + c);
}

__global__ __launch_bounds__(256) void scatter_rows_kernel(const bf16_t* __restrict__ src, const int* __restrict__ idx,
                                                           int per, long long gs, bf16_t* __restrict__ dst,
                                                           long long ldd, int n, int H, int accumulate) {
  const long long r = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const long long to = (idx ? idx[r] : 0) + (r / per) * gs;
  for (int c = (threadIdx.x & 63) * 8; c < H; c += 512) {
    uint4 v = ldg16(src + r * H + c);
    if (accumulate) {
      float a[8], b[8];
      unpack8(v, a);
      unpack8(ldg16(dst + to * ldd + c), b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j];
      v = pack8(a);
    }
    *reinterpret_cast<uint4*>(dst + to * ldd + c) = v;
  }
}

// ------------------------------------------------------------------ vocabulary xent
// inv_count[0] = scale / max(1, #labels >= 0)
// inv_count[0] = scale / count; with both (the MLM step's metric and gradient scales from one
// launch instead of a torch multiply) inv_count[0] = 1 / count, inv_count[1] = scale / count
__global__ __launch_bounds__(256) void count_valid_kernel(const int* __restrict__ labels, int n, float scale,
                                                          float* __restrict__ inv_count, int both) {
  __shared__ float red[16];
  float c = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) c += labels[i] >= 0 ? 1.f : 0.f;
  c = block_sum(c, red);
  if (threadIdx.x == 0) {
    const float cc = fmaxf(c, 1.f);
    if (both) {
      inv_count[0] = 1.f / cc;
      inv_count[1] = scale / cc;
    } else {
      inv_count[0] = scale / cc;
    }
  }
}

// One block per row of bf16 logits [rows][ld] (first V columns valid). labels < 0 are
// ignored (zero loss and gradient). dlogits may alias logits. sums[0] += loss * inv,
// sums[1] += correct * inv (inv = inv_count[0] / scale_for_grad... see wrapper).
__global__ __launch_bounds__(256) void xent_vocab_kernel(const bf16_t* logits, long long ld, int V,
                                                         const int* __restrict__ labels, const float* __restrict__ gsc,
                                                         bf16_t* dlogits, float* __restrict__ sums,
                                                         const float* __restrict__ msc) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
  const bf16_t* z = logits + row * ld;
  const int lab = labels[row];
  const bool valid = lab >= 0 && lab < V;
  const float zt = valid ? bf2f(z[lab]) : 0.f;
  float mx = -INFINITY;
  int greater = 0;
  for (int i = threadIdx.x * 8; i < V; i += 256 * 8) {
    float a[8];
    if (i + 8 <= V) {
      unpack8(ldg16(z + i), a);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = i + j < V ? bf2f(z[i + j]) : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mx = fmaxf(mx, a[j]);
      greater += a[j] > zt;
    }
  }
  mx = wave_max(mx);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float se = 0.f;
  for (int i = threadIdx.x * 8; i < V; i += 256 * 8) {
    float a[8];
    if (i + 8 <= V) {
      unpack8(ldg16(z + i), a);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = i + j < V ? bf2f(z[i + j]) : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) se += __expf(a[j] - mx);
  }
  se = block_sum(se, red + 8);
  const float gt = block_sum(static_cast<float>(greater), red);
  const float g = valid ? gsc[0] : 0.f;
  if (dlogits) {  // also zero the padding columns [V, ld) so padded vocabulary rows get no gradient
    const float inv = 1.f / se;
    for (int i = threadIdx.x * 8; i < ld; i += 256 * 8) {
      float a[8];
      if (i + 8 <= V) {
        unpack8(ldg16(z + i), a);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = i + j < V ? bf2f(z[i + j]) : -INFINITY;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = (__expf(a[j] - mx) * inv - (i + j == lab ? 1.f : 0.f)) * g;
      *reinterpret_cast<uint4*>(dlogits + row * ld + i) = pack8(a);
    }
  }
  if (threadIdx.x == 0 && valid && sums) {
    const float loss = mx + __logf(se) - zt;
    const float ms = msc ? msc[0] : 1.f;
    atomicAdd(&sums[0], loss * ms);
    atomicAdd(&sums[1], (isfinite(zt) && gt < 1.f ? 1.f : 0.f) * ms);
  }
}

// dx = dy * act'(aux): kind 0 = tanh-GELU (aux = pre-activation), kind 1 = tanh (aux = output)
__global__ __launch_bounds__(256) void dact_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ aux,
                                                   bf16_t* __restrict__ dx, long long n8, int kind) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  float d[8], a[8];
  unpack8(ldg16(dy + i * 8), d);
  unpack8(ldg16(aux + i * 8), a);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (kind == 0) {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f, x = a[j];
      const float t = tanhf(k0 * (x + k1 * x * x * x));
      d[j] *= 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
    } else {
      d[j] *= 1.f - a[j] * a[j];
    }
  }
  *reinterpret_cast<uint4*>(dx + i * 8) = pack8(d);
}

__global__ void tanh_bf16_kernel(bf16_t* x, long long n) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) x[i] = f2bf(tanhf(bf2f(x[i])));
}

DropSpec make_drop(const long long* rng, unsigned site_in, float p_in, unsigned site_out, float p_out) {
  DropSpec d;
  d.rng = rng;
  d.site_in = site_in;
  d.site_out = site_out;
  d.thr_in = drop_threshold(p_in);
  d.thr_out = drop_threshold(p_out);
  d.scale_in = p_in > 0.f ? 1.f / (1.f - p_in) : 1.f;
  d.scale_out = p_out > 0.f ? 1.f / (1.f - p_out) : 1.f;
  return d;
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

#define TTDK_LN_DISPATCH(KER, ...)                                                      \
  switch (H) {                                                                          \
    case 512: hipLaunchKernelGGL(KER<1>, __VA_ARGS__); break;                           \
    case 1024: hipLaunchKernelGGL(KER<2>, __VA_ARGS__); break;                          \
    case 1536: hipLaunchKernelGGL(KER<3>, __VA_ARGS__); break;                          \
    case 2048: hipLaunchKernelGGL(KER<4>, __VA_ARGS__); break;                          \
    case 4096: hipLaunchKernelGGL(KER<8>, __VA_ARGS__); break;                          \
    default: return hipErrorInvalidValue;                                               \
  }

// TTD_LN_BWD_PREFETCH (default 1): the H = 1024 backward loads its next rows one iteration ahead
inline bool ln_bwd_prefetch() {
  static const bool on = [] {
    const char* e = getenv("TTD_LN_BWD_PREFETCH");
    return !(e && e[0] == '0');
  }();
  return on;
}

#define TTDK_LN_BWD_DISPATCH(...)                                                        \
  switch (H) {                                                                           \
    case 512: hipLaunchKernelGGL((ln_bwd_kernel<1, 16, 1>), dim3(nb), dim3(16 * 64), __VA_ARGS__); break; \
    case 1024:                                                                           \
      if (ln_bwd_prefetch())                                                             \
        hipLaunchKernelGGL((ln_bwd_kernel<2, 8, 1, true>), dim3(nb), dim3(8 * 64), __VA_ARGS__); \
      else                                                                               \
        hipLaunchKernelGGL((ln_bwd_kernel<2, 8, 2>), dim3(nb), dim3(8 * 64), __VA_ARGS__);       \
      break;                                                                             \
    case 1536: hipLaunchKernelGGL((ln_bwd_kernel<3, 8, 1>), dim3(nb), dim3(8 * 64), __VA_ARGS__); break;  \
    case 2048: hipLaunchKernelGGL((ln_bwd_kernel<4, 4, 1>), dim3(nb), dim3(4 * 64), __VA_ARGS__); break;  \
    case 4096: hipLaunchKernelGGL((ln_bwd_kernel<8, 4, 1>), dim3(nb), dim3(4 * 64), __VA_ARGS__); break;  \
    default: return hipErrorInvalidValue;                                                \
  }

TTDK_EXPORT int ttdk_ln_fwd(const bf16_t* x, const bf16_t* res, bf16_t* s_out, bf16_t* y, float* mean, float* rstd,
                            const float* gamma, const float* beta, int rows, int H, float eps, float p_in,
                            unsigned site_in, float p_out, unsigned site_out, const long long* rng, hipStream_t st) {
  if ((p_in > 0.f || p_out > 0.f) && !rng) return hipErrorInvalidValue;
  DropSpec d = make_drop(rng, site_in, p_in, site_out, p_out);
  dim3 grid((rows + 3) / 4), block(256);
  TTDK_LN_DISPATCH(ln_fwd_kernel, grid, block, 0, st, x, res, s_out, y, mean, rstd, gamma, beta, rows, eps, d);
  return hipGetLastError();
}

// Blocks of ln_bwd_kernel (= partial rows of the workspace): one 8-wave block per CU. Two per CU
// (4 waves per SIMD at the H = 1024 kernel's 120 VGPRs) measured the same standalone (146 vs 147
// us at 65536 x 1024) and in the BERT step, four slower (TTD_LN_BWD_BLOCKS: A/B).
TTDK_EXPORT int ttdk_ln_bwd_num_blocks(int rows) {
  static const int cap = [] {
    const char* e = getenv("TTD_LN_BWD_BLOCKS");
    const int v = e ? atoi(e) : 256;
    return v > 0 ? v : 256;
  }();
  return rows < cap * 16 ? (rows + 15) / 16 : cap;
}

// part: fp32 [nblocks][2][H] workspace; dgamma/dbeta written (beta=0) or accumulated.
TTDK_EXPORT int ttdk_ln_bwd(const bf16_t* dy, const bf16_t* s, const float* mean, const float* rstd,
                            const float* gamma, bf16_t* ds_out, bf16_t* dx_out, float* part, float* dgamma,
                            float* dbeta, int accumulate, int rows, int H, float p_in, unsigned site_in, float p_out,
                            unsigned site_out, const long long* rng, hipStream_t st) {
  if ((p_in > 0.f || p_out > 0.f) && !rng) return hipErrorInvalidValue;
  DropSpec d = make_drop(rng, site_in, p_in, site_out, p_out);
  const int nb = ttdk_ln_bwd_num_blocks(rows);
  const int rpb = (rows + nb - 1) / nb;
  TTDK_LN_BWD_DISPATCH(0, st, dy, s, mean, rstd, gamma, ds_out, dx_out, part, rows, rpb, d);
  // part rows are [dgamma(H) | dbeta(H)]; one launch when the outputs are adjacent (flat store)
  if (dbeta == dgamma + H) {
    hipLaunchKernelGGL(colreduce_kernel, dim3((2 * H + 15) / 16), dim3(256), 0, st, part, nb, 2 * H, 2 * H, dgamma,
                       accumulate);
  } else {
    hipLaunchKernelGGL(colreduce_kernel, dim3((H + 15) / 16), dim3(256), 0, st, part, nb, H, 2 * H, dgamma, accumulate);
    hipLaunchKernelGGL(colreduce_kernel, dim3((H + 15) / 16), dim3(256), 0, st, part + H, nb, H, 2 * H, dbeta,
                       accumulate);
  }
  return hipGetLastError();
}

// out[c] (+)= sum_b part[b * stride + c], c < C.
TTDK_EXPORT int ttdk_colreduce(const float* part, int nb, int C, int stride, float* out, int beta, hipStream_t st) {
  if (C % 4 || stride % 4 || (reinterpret_cast<uintptr_t>(part) & 15) || (reinterpret_cast<uintptr_t>(out) & 15))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(colreduce_kernel, dim3((C + 15) / 16), dim3(256), 0, st, part, nb, C, stride, out, beta);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_embed_fwd(const int* ids, const int* tt, const bf16_t* word, const bf16_t* pos, const bf16_t* typ,
                               bf16_t* s, long long rows, int S, int H, hipStream_t st) {
  if (H % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(static_cast<unsigned>((rows + 3) / 4)), dim3(256), 0, st, ids, tt, word, pos,
                     typ, s, rows, S, H);
  return hipGetLastError();
}

// dword must already hold (or be zeroed for) the other contributions (e.g. the tied decoder).
TTDK_EXPORT int ttdk_embed_bwd(const bf16_t* ds, const int* ids, const int* tt, float* dword, float* dpos, float* dtype,
                               int B, int S, int H, int T, int pos_beta, hipStream_t st) {
  if (H % 8 || H / 8 > 256 || T > 4) return hipErrorInvalidValue;
  const long long rows = static_cast<long long>(B) * S;
  hipLaunchKernelGGL(embed_bwd_word_kernel, dim3(static_cast<unsigned>((rows + 3) / 4)), dim3(256), 0, st, ds, ids,
                     dword, rows, H);
  hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(static_cast<unsigned>((static_cast<long long>(S) * (H / 8) + 255) / 256)),
                     dim3(256), 0, st, ds, dpos, B, S, H, pos_beta);
  if (dtype) {
    hipError_t e = hipMemsetAsync(dtype, 0, sizeof(float) * T * H, st);
    if (e != hipSuccess) return e;
    const int nb = 512;
    const int rpb = static_cast<int>((rows + nb - 1) / nb);
    hipLaunchKernelGGL(embed_bwd_type_kernel, dim3(nb), dim3(256), 0, st, ds, tt, dtype, rows, H, T, rpb);
  }
  return hipGetLastError();
}

// idx (nullable) + per / gs: see gather_rows_kernel; per = 1, gs = 0 is a plain index gather.
TTDK_EXPORT int ttdk_gather_rows(const bf16_t* src, long long ld_src, const int* idx, int per, long long gs, bf16_t* dst,
                                 int n, int H, hipStream_t st) {
  if (H % 8 || ld_src % 8 || per < 1 || (!idx && gs == 0 && n > 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, st, src, ld_src, idx, per, gs, dst, n, H);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_scatter_rows(const bf16_t* src, const int* idx, int per, long long gs, bf16_t* dst, long long ld_dst,
                                  int n, int H, int accumulate, hipStream_t st) {
  if (H % 8 || ld_dst % 8 || per < 1 || (!idx && gs == 0 && n > 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, st, src, idx, per, gs, dst, ld_dst, n, H,
                     accumulate);
  return hipGetLastError();
}

// dropout RNG state [seed, step]: step += 1 on the stream (a captured node in a graph replay)
__global__ void rng_advance_kernel(long long* __restrict__ t) {
  if (threadIdx.x == 0) t[1] = t[1] + 1;
}

TTDK_EXPORT int ttdk_rng_advance(long long* t, hipStream_t st) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(64), 0, st, t);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_count_valid(const int* labels, int n, float scale, float* inv_count, hipStream_t st) {
  hipLaunchKernelGGL(count_valid_kernel, dim3(1), dim3(256), 0, st, labels, n, scale, inv_count, 0);
  return hipGetLastError();
}

// out[0] = 1 / count, out[1] = scale / count (count = labels >= 0)
TTDK_EXPORT int ttdk_count_valid2(const int* labels, int n, float scale, float* out, hipStream_t st) {
  hipLaunchKernelGGL(count_valid_kernel, dim3(1), dim3(256), 0, st, labels, n, scale, out, 1);
  return hipGetLastError();
}

// grad scale = gsc[0] (device, e.g. from ttdk_count_valid); metric scale = msc[0] (device or
// null = 1). sums (fp32[2]) is accumulated, not zeroed.
TTDK_EXPORT int ttdk_xent_vocab(const bf16_t* logits, long long ld, int V, const int* labels, int rows, const float* gsc,
                                bf16_t* dlogits, float* sums, const float* msc, hipStream_t st) {
  if (ld % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_vocab_kernel, dim3(rows), dim3(256), 0, st, logits, ld, V, labels, gsc, dlogits, sums, msc);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_dact_bf16(const bf16_t* dy, const bf16_t* aux, bf16_t* dx, long long n, int kind,
                               hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  const long long n8 = n / 8;
  hipLaunchKernelGGL(dact_kernel, dim3(static_cast<unsigned>((n8 + 255) / 256)), dim3(256), 0, st, dy, aux, dx, n8, kind);
  return hipGetLastError();
}

TTDK_EXPORT int ttdk_tanh_bf16(bf16_t* x, long long n, hipStream_t st) {
  hipLaunchKernelGGL(tanh_bf16_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, st, x, n);
  return hipGetLastError();
}
