#pragma once
// MFMA (bf16, gfx950) GEMM engine + implicit-GEMM convolution (fwd / dgrad / wgrad): the
// kernel templates and host-side dispatch helpers shared by gemm_conv.hip (dense GEMM),
// conv_fwd.hip (forward conv, fp8), conv_dgrad.hip and conv_wgrad.hip — one translation
// unit per entry group so hipcc builds them in parallel.
//
// This is the MatMul/Conv2D hot path of the framework: the dense layers of the reference's
// MLP (tf.layers.dense, /root/reference/distribute_training.py:54,61 — fwd MatMul F1/F5 and
// the backward MatMuls G3/G4 of SURVEY.md §2.6) and every conv / FC / projection of the
// BASELINE.json north-star models (ResNet-50, BERT-Large).
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §3, §5):
//  * One templated kernel: BMxBN output tile (64/128 each), BK = 64, 256 threads = 4 waves in
//    a 2x2 arrangement, each wave owning (BM/2)x(BN/2) as 16x16 tiles of
//    v_mfma_f32_16x16x32_bf16 (fp32 accumulate).
//  * Operands are staged global -> registers -> LDS (double buffered, one barrier per K-step,
//    loads for step k+1 issued before the MFMAs of step k, LDS write after them: T14).
//    Register staging lets the A loader be an implicit-GEMM *gather* with zero padding.
//  * Each operand is either K-major (reduction dim contiguous: 16-B ds_read_b128 fragments,
//    XOR-swizzled rows) or MN-major (rows contiguous: stored [k][rows] and read with the
//    gfx950 transposing ds_read_b64_tr_b16, 32-B-slot XOR swizzle), so NN/NT/TN/TT GEMMs and
//    the conv weight-gradient (both operands pixel-strided) share one engine, conflict-free.
//  * The MFMA is issued with operands swapped (D = B·Aᵀ) so each lane ends up holding 4
//    consecutive output columns of one row: 8-/16-byte vector stores in the epilogue.
//  * XCD-aware bijective block remap (T1) so blocks sharing an A panel share an L2.
//  * Split-K (grid.y) writes fp32 slabs that a reduce kernel sums (no float atomics).
//  * Optional fused epilogue: bias, ReLU/GELU, residual add, accumulate-into-output,
//    strided output-row remap (stride-2 1x1 dgrad), per-tile BatchNorm partial sums.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

// process-wide runtime switches shared by every translation unit of libttd_hip (defined in
// gemm_conv.hip; everything below lives in an anonymous namespace, i.e. per TU)
namespace ttdk_rt {
int& pers_flag();
int& reserved_cus();
int& fold_flag();
}

namespace ttdk {
namespace {

constexpr int BK = 64;
constexpr int NTHR = 256;

// ------------------------------------------------------------------ LDS layouts
// K-major tile: ROWS x 64 bf16 (128 B per row, 8 chunks of 16 B), chunk ^= (row>>1)&7.
__device__ __forceinline__ int kmaj_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// MN-major tile: 64 k-rows x ROWS bf16; 32-B slots XOR-swizzled so that the 8 k-rows a
// half-wave touches in one ds_read_b64_tr_b16 land on distinct banks.
template <int ROWS>
__device__ __forceinline__ int mn_swz(int k) {
  if constexpr (ROWS == 128)
    return (k & 3) | ((k >> 1) & 4);
  else
    return ((k >> 1) & 1) | ((k >> 2) & 2);
}
template <int ROWS>
__device__ __forceinline__ int mnmaj_off(int k, int col) {
  return k * (ROWS * 2) + (((col >> 4) ^ mn_swz<ROWS>(k)) << 5) + ((col & 15) << 1);
}

__device__ __forceinline__ bf16x8_t lds_read_b128(const char* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

__device__ __forceinline__ s16x4_t lds_read_tr(const char* p) {
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p));
}

__device__ __forceinline__ uint4 ldg16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

// ------------------------------------------------------------------ operand loaders
// Every loader: Params; init(params, row0, tid); load(k0) -> regs; store(lds); frag(...).

struct DenseParams {  // K-major: element (row, k) at p[row*ld + k]; MN-major: (k, row) at p[k*ld + row]
  const bf16_t* p;
  long long ld;
  int rows;
  int K;
};

struct GatherParams {  // conv operand geometry (see KConvGather / MNConvGather)
  const bf16_t* x;
  int Hs, Ws, Cs;
  int P, Q;
  int R, S;
  int sh, sw, ph, pw, dh, dw;
  int rows;
  int K;
};

template <int ROWS, bool VEC = true>
struct KDense {  // element (row, k) at p[row * ld + k]; VEC: K % 8 == 0, ld % 8 == 0, 16-B aligned base
  using Params = DenseParams;
  static constexpr int N = ROWS / 32;
  static constexpr int BYTES = ROWS * BK * 2;
  const bf16_t* ptr[N];
  bool ok[N];
  int c, K;
  uint4 r[N];
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    c = tid & 7;
    K = P.K;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int row = row0 + (tid >> 3) + 32 * i;
      ok[i] = row < P.rows;
      ptr[i] = P.p + static_cast<long long>(ok[i] ? row : 0) * P.ld + c * 8;
    }
  }
  __device__ __forceinline__ void load(int k0) {
    if constexpr (VEC) {
      const bool kin = k0 + c * 8 < K;
#pragma unroll
      for (int i = 0; i < N; ++i) r[i] = (ok[i] && kin) ? ldg16(ptr[i] + k0) : make_uint4(0, 0, 0, 0);
    } else {
      const int kb = k0 + c * 8;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t lo = (ok[i] && kb + 2 * e < K) ? ptr[i][k0 + 2 * e] : 0u;
          const uint32_t hi = (ok[i] && kb + 2 * e + 1 < K) ? ptr[i][k0 + 2 * e + 1] : 0u;
          w[e] = lo | (hi << 16);
        }
        r[i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + kmaj_off((tid >> 3) + 32 * i, c)) = r[i];
  }
  static __device__ __forceinline__ bf16x8_t frag(const char* lds, int rowbase, int ks, int lane) {
    return lds_read_b128(lds + kmaj_off(rowbase + (lane & 15), ks * 4 + (lane >> 4)));
  }
};

// Implicit-GEMM gather of a conv input patch, K-major: row = output pixel (n, p, q),
// k = (r, s, c). DGRAD=false: forward conv, source pixel = p*stride - pad + r*dil.
// DGRAD=true: data gradient, source pixel of dY = (p + pad - r*dil) / stride when divisible.
// The k-steps run in order, so the tap (r, s) and channel group of a thread's 16-B chunk are
// tracked incrementally (no integer divisions per k-step) whenever C % 64 == 0 (the chunk's
// channel group advances by 8 and wraps into the next tap) or C divides 64 (the tap advances by
// 64/C); per-row work is then two adds, two unsigned range tests and one 64-bit add on a
// per-row base pointer. Other shapes (and strided dgrad) recompute with divisions.
template <int ROWS, bool DGRAD>
struct KConvGather {
  // x: source activations NHWC [Nimg, Hs, Ws, Cs]; (P, Q): pixel grid of the GEMM rows;
  // rows = Nimg*P*Q; K = R*S*Cs.
  using Params = GatherParams;
  static constexpr int N = ROWS / 32;
  static constexpr int BYTES = ROWS * BK * 2;
  const bf16_t* x;
  int Hs, Ws, Cs, cch, S, sh, sw, dh, dw, K, c;
  int img[N], hb[N], wb[N];
  const bf16_t* base[N];  // tap-(0,0) source pixel of each row (may point outside x; only valid taps load)
  bool ok[N];
  uint4 r[N];
  int knext, c8, rr, ss, mode, dss, drr;
  bool unit;
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    x = P.x;
    Hs = P.Hs;
    Ws = P.Ws;
    Cs = P.Cs;
    cch = P.Cs >> 3;
    S = P.S;
    sh = P.sh;
    sw = P.sw;
    dh = P.dh;
    dw = P.dw;
    K = P.K;
    c = tid & 7;
    unit = !DGRAD || (P.sh == 1 && P.sw == 1);
    mode = !unit ? 0 : (cch % 8 == 0 ? 1 : (8 % cch == 0 ? 2 : 0));
    const int dt = mode == 2 ? 8 / cch : 0;
    dss = mode == 2 ? dt % S : 0;
    drr = mode == 2 ? dt / S : 0;
    knext = -1;
    const int pq = P.P * P.Q;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int m = row0 + (tid >> 3) + 32 * i;
      ok[i] = m < P.rows;
      const int mm = ok[i] ? m : 0;
      const int n = mm / pq, rem = mm - n * pq;
      const int p = rem / P.Q, q = rem - p * P.Q;
      img[i] = n * P.Hs;
      if (DGRAD) {
        hb[i] = p + P.ph;
        wb[i] = q + P.pw;
      } else {
        hb[i] = p * P.sh - P.ph;
        wb[i] = q * P.sw - P.pw;
      }
      base[i] = x + (static_cast<long long>(img[i] + hb[i]) * Ws + wb[i]) * Cs;
    }
  }
  __device__ __forceinline__ void load(int k0) {
    if (k0 != knext) {  // (re)derive this thread's chunk position (first step / generic shapes)
      const int kc = (k0 >> 3) + c;
      const int tap = kc / cch;
      c8 = kc - tap * cch;
      rr = tap / S;
      ss = tap - rr * S;
    }
    const bool kin = ((k0 >> 3) + c) * 8 < K;
    if (unit) {
      const int dhh = DGRAD ? -rr * dh : rr * dh, dww = DGRAD ? -ss * dw : ss * dw;
      const long long off = (static_cast<long long>(dhh) * Ws + dww) * Cs + c8 * 8;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const bool v = ok[i] && kin && static_cast<unsigned>(hb[i] + dhh) < static_cast<unsigned>(Hs) &&
                       static_cast<unsigned>(wb[i] + dww) < static_cast<unsigned>(Ws);
        r[i] = v ? ldg16(base[i] + off) : make_uint4(0, 0, 0, 0);
      }
    } else {  // strided data gradient: source pixel only where the stride divides
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int hn = hb[i] - rr * dh, wn = wb[i] - ss * dw;
        const int h = hn / sh, w = wn / sw;
        const bool v = ok[i] && kin && hn >= 0 && wn >= 0 && h * sh == hn && w * sw == wn && h < Hs && w < Ws;
        r[i] = v ? ldg16(x + ((static_cast<long long>(img[i] + h) * Ws + w) * Cs + c8 * 8)) : make_uint4(0, 0, 0, 0);
      }
    }
    // advance to the next k-step (k0 + BK = 8 chunks further)
    if (mode == 1) {
      c8 += 8;
      if (c8 >= cch) {
        c8 -= cch;
        if (++ss == S) {
          ss = 0;
          ++rr;
        }
      }
      knext = k0 + BK;
    } else if (mode == 2) {
      ss += dss;
      rr += drr;
      if (ss >= S) {
        ss -= S;
        ++rr;
      }
      knext = k0 + BK;
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + kmaj_off((tid >> 3) + 32 * i, c)) = r[i];
  }
  static __device__ __forceinline__ bf16x8_t frag(const char* lds, int rowbase, int ks, int lane) {
    return KDense<ROWS>::frag(lds, rowbase, ks, lane);
  }
};

template <int ROWS>
__device__ __forceinline__ bf16x8_t mn_frag(const char* lds, int colbase, int ks, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int ka = ks * 32 + 8 * g + q;
  const int col = colbase + 4 * p;
  const s16x4_t lo = lds_read_tr(lds + mnmaj_off<ROWS>(ka, col));
  const s16x4_t hi = lds_read_tr(lds + mnmaj_off<ROWS>(ka + 4, col));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int ROWS, bool VEC = true>
struct MNDense {  // element (k, row) at p[k * ld + row]; VEC: rows % 8 == 0, ld % 8 == 0, aligned base
  using Params = DenseParams;
  static constexpr int CPR = ROWS / 8;           // 16-B chunks per k-row
  static constexpr int KPP = NTHR / CPR;         // k-rows per pass
  static constexpr int N = BK / KPP;             // passes
  static constexpr int BYTES = ROWS * BK * 2;
  const bf16_t* p;
  long long ld;
  int K, cc, kr, rows_left;
  bool cok;
  uint4 r[N];
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    cc = tid % CPR;
    kr = tid / CPR;
    ld = P.ld;
    K = P.K;
    cok = row0 + cc * 8 < P.rows;
    rows_left = P.rows - (row0 + cc * 8);
    p = P.p + row0 + cc * 8;
  }
  __device__ __forceinline__ void load(int k0) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int k = k0 + kr + KPP * i;
      if constexpr (VEC) {
        r[i] = (cok && k < K) ? ldg16(p + static_cast<long long>(k) * ld) : make_uint4(0, 0, 0, 0);
      } else {
        const bf16_t* q = p + static_cast<long long>(k) * ld;
        const bool kok = cok && k < K;
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t lo = (kok && 2 * e < rows_left) ? q[2 * e] : 0u;
          const uint32_t hi = (kok && 2 * e + 1 < rows_left) ? q[2 * e + 1] : 0u;
          w[e] = lo | (hi << 16);
        }
        r[i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + mnmaj_off<ROWS>(kr + KPP * i, cc * 8)) = r[i];
  }
  static __device__ __forceinline__ bf16x8_t frag(const char* lds, int colbase, int ks, int lane) {
    return mn_frag<ROWS>(lds, colbase, ks, lane);
  }
};

// MN-major operand produced on the fly from a BatchNorm backward: element (k, row) =
// a[row] * g[k][row] + b[row] * y[k][row] + c[row] (coef = [3][rows] fp32, rounded to bf16 as
// ttdk_bn_bwd_apply rounds dz). Lets a weight gradient consume the BN-backward output without
// that pass storing it (the stem: the last kernels of every backward). rows % 8 == 0.
struct DenseBNParams {
  const bf16_t* p;  // g: already ReLU-masked output gradient
  long long ld;
  int rows, K;
  const bf16_t* y;  // BN input, same layout as g
  const float* coef;
};

template <int ROWS>
struct MNDenseBN {
  using Params = DenseBNParams;
  static constexpr int CPR = ROWS / 8;
  static constexpr int KPP = NTHR / CPR;
  static constexpr int N = BK / KPP;
  static constexpr int BYTES = ROWS * BK * 2;
  const bf16_t* p;
  const bf16_t* y;
  long long ld;
  int K, cc, kr;
  bool cok;
  float ca[8], cb[8], c0[8];
  uint4 r[N];
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    cc = tid % CPR;
    kr = tid / CPR;
    ld = P.ld;
    K = P.K;
    const int m = row0 + cc * 8;
    cok = m < P.rows;
    p = P.p + m;
    y = P.y + m;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = cok ? P.coef[m + j] : 0.f;
      cb[j] = cok ? P.coef[P.rows + m + j] : 0.f;
      c0[j] = cok ? P.coef[2 * P.rows + m + j] : 0.f;
    }
  }
  __device__ __forceinline__ void load(int k0) {
    uint4 gv[N], yv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int k = k0 + kr + KPP * i;
      const bool ok = cok && k < K;
      gv[i] = ok ? ldg16(p + static_cast<long long>(k) * ld) : make_uint4(0, 0, 0, 0);
      yv[i] = ok ? ldg16(y + static_cast<long long>(k) * ld) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int k = k0 + kr + KPP * i;
      float g[8], yf[8];
      unpack8(gv[i], g);
      unpack8(yv[i], yf);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = ca[j] * g[j] + cb[j] * yf[j] + c0[j];
      r[i] = (cok && k < K) ? pack8(g) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + mnmaj_off<ROWS>(kr + KPP * i, cc * 8)) = r[i];
  }
  static __device__ __forceinline__ bf16x8_t frag(const char* lds, int colbase, int ks, int lane) {
    return mn_frag<ROWS>(lds, colbase, ks, lane);
  }
};

// Weight-gradient im2col operand, MN-major: k = output pixel (n, p, q), column = (r, s, c),
// element = x[n, p*sh - ph + r*dh, q*sw - pw + s*dw, c]. Each thread's k-rows advance by BK
// per step; their (n, p, q) are carried forward with adds and wraps instead of two integer
// divisions per chunk per step.
template <int ROWS>
struct MNConvGather {
  // x: conv input [Nimg, Hs, Ws, Cs]; (P, Q): output grid; rows = R*S*Cs; K = Nimg*P*Q.
  using Params = GatherParams;
  static constexpr int CPR = ROWS / 8;
  static constexpr int KPP = NTHR / CPR;
  static constexpr int N = BK / KPP;
  static constexpr int BYTES = ROWS * BK * 2;
  const bf16_t* x;
  int H, W, C, P, Q, pq, sh, sw, K, kr, cc, roff, soff, dq, dp, knext;
  int nn[N], pp[N], qq[N];
  bool cok;
  uint4 r[N];
  __device__ __forceinline__ void init(const Params& Pm, int row0, int tid) {
    cc = tid % CPR;
    kr = tid / CPR;
    x = Pm.x;
    H = Pm.Hs;
    W = Pm.Ws;
    C = Pm.Cs;
    P = Pm.P;
    Q = Pm.Q;
    pq = Pm.P * Pm.Q;
    sh = Pm.sh;
    sw = Pm.sw;
    K = Pm.K;
    dq = BK % Q;
    dp = BK / Q;
    knext = -1;
    const int col = row0 + cc * 8;
    cok = col < Pm.rows;
    const int cl = cok ? col : 0;
    const int tap = cl / C, c = cl - tap * C;
    const int rr = tap / Pm.S, ss = tap - rr * Pm.S;
    roff = rr * Pm.dh - Pm.ph;
    soff = ss * Pm.dw - Pm.pw;
    x += c;
  }
  __device__ __forceinline__ void load(int k0) {
    if (k0 != knext) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int k = k0 + kr + KPP * i;
        nn[i] = k / pq;
        const int rem = k - nn[i] * pq;
        pp[i] = rem / Q;
        qq[i] = rem - pp[i] * Q;
      }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int k = k0 + kr + KPP * i;
      const int h = pp[i] * sh + roff, w = qq[i] * sw + soff;
      const bool v = cok && k < K && static_cast<unsigned>(h) < static_cast<unsigned>(H) &&
                     static_cast<unsigned>(w) < static_cast<unsigned>(W);
      r[i] = v ? ldg16(x + (static_cast<long long>(nn[i] * H + h) * W + w) * C) : make_uint4(0, 0, 0, 0);
      // advance this k-row by BK pixels
      qq[i] += dq;
      pp[i] += dp;
      if (qq[i] >= Q) {
        qq[i] -= Q;
        ++pp[i];
      }
      while (pp[i] >= P) {
        pp[i] -= P;
        ++nn[i];
      }
    }
    knext = k0 + BK;
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + mnmaj_off<ROWS>(kr + KPP * i, cc * 8)) = r[i];
  }
  static __device__ __forceinline__ bf16x8_t frag(const char* lds, int colbase, int ks, int lane) {
    return mn_frag<ROWS>(lds, colbase, ks, lane);
  }
};

// ------------------------------------------------------------------ epilogues
// kActDGelu: backward of the tanh-GELU: out = acc * gelu'(residual) (residual = the
// pre-activation saved by the forward epilogue; not added).
enum Act : int { kActNone = 0, kActRelu = 1, kActGelu = 2, kActTanh = 3, kActDGelu = 4 };

// tanh(u) = 1 - 2 / (1 + 2^(2u log2 e)): one v_exp_f32 + one v_rcp_f32 instead of the
// libm tanhf (measured: the GELU epilogues of the BERT GEMMs were VALU-bound on it);
// saturates to +-1 through exp2 -> inf / 0, absolute error ~1e-7 near 0
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * 2.8853900817779268f));
}

// tanh-GELU as x * sigmoid(2u), u = k0 (x + k1 x^3): 0.5 x (1 + tanh u) = x / (1 + e^(-2u)), with
// 2u log2(e) = x (c1 + c2 x^2) — five plain VALU ops + v_exp_f32 + v_rcp_f32 per element (the
// 0.5 x (1 + tanh) form took ten plain ops; the GELU / dGELU GEMM epilogues run ~256 elements
// per lane after the main loop). Saturates through exp2 -> inf / 0 (x -> -inf: 0, +inf: x).
constexpr float kGeluC1 = 2.f * 0.7978845608028654f * 1.4426950408889634f;
constexpr float kGeluC2 = kGeluC1 * 0.044715f;
__device__ __forceinline__ float gelu_tanh(float x) {
  const float z = -x * __builtin_fmaf(kGeluC2, x * x, kGeluC1);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}

// d/dx x s(x), s = sigmoid(2u): s + x s (1 - s) 2u' = s (1 + x (1 - s) 2 k0 (1 + 3 k1 x^2))
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float t = x * x;
  const float sg = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * __builtin_fmaf(kGeluC2, t, kGeluC1)));
  const float q = __builtin_fmaf(6.f * k0 * k1, t, 2.f * k0);
  return __builtin_fmaf(sg, x * (1.f - sg) * q, sg);  // (1 - sg, not e * sg: inf * 0 at x -> -inf)
}

struct EpiParams {
  int mode;  // 0 = bf16 store, 1 = fp32 slab store (split-K), 2 = fp32 store
  void* out;
  long long ldo;
  long long slab_stride;  // elements between split-K slabs (mode 1)
  const float* bias;      // [N] or null
  const bf16_t* residual; // same layout as out, or null
  long long ldr;
  int act;
  int beta;               // accumulate: out = acc + out
  // strided output-row remap (dgrad of strided 1x1 convs): row m=(n,p,q) -> (n, p*rs, q*rs) of [OH,OW]
  int remap;
  int rP, rQ, rOH, rOW, rs;
  float* stat;  // BN partial sums: [tiles_m][2][N] (sum, sumsq) or null
  float alpha;  // scale applied to acc
  bf16_t* aux;  // optional: pre-activation copy (GELU backward input), row stride ldo
  const float* ascale0;  // optional device scalars multiplied into alpha (fp8 dequant scales)
  const float* ascale1;
  // BN-backward statistics of the produced gradient (dgrad feeding a conv+BN(+ReLU) unit):
  // with `by` set the stored value is g = v * mask (ReLU bit per element, `bmask`, optional)
  // and `stat` receives per-tile (sum g, sum g*y) with y = by (the unit's pre-BN conv output,
  // same layout as out) — the separate bwd-partial pass over dy and y disappears.
  const bf16_t* by;
  const uint8_t* bmask;
  // optional second BN fed by the same masked gradient (ResNet projection shortcut): stat2
  // receives per-tile (sum g, sum g*by2)
  const bf16_t* by2;
  float* stat2;
  // beta (accumulate) only at output rows m = (n, h, w) of an [bH, bW] grid with h and w even:
  // the other rows of `out` hold no data yet (the stride-2 1x1 projection dgrad wrote only the
  // pixels it samples), so the accumulated tensor needs no zero fill. 0 = every row.
  int bH, bW;
  int feed_pf;  // 256-row kernel: prefetched feeding-BN epilogue allowed (TTD_FEED_PREFETCH, default 1)
  // BN-backward operand prologue of the 256-row kernel (OpDenseKBN A operand, 1x1 dgrads): the A
  // tile read by DMA is the unit's masked output gradient g; in LDS it becomes
  // dz = a[k]*g + b[k]*py + c[k] (pcoef = [3][K] a | b | c, py = the unit's conv output, row
  // stride pld) before any fragment is read, and the workgroups of tile column 0 store dz to pdz
  // (the weight gradient's operand): the separate BN backward-apply pass and this GEMM's
  // re-read of its output disappear.
  // Forward modes (OpDenseKBN<.., 2 | 3>, the next unit's 1x1 conv consuming a raw conv output):
  // A tile = y3 (DMA); in LDS it becomes h = relu(sc[k]*y3 + sh[k] + r) with r = py (residual)
  // (mode 3: r*rsc[k] + rsh[k], the projection shortcut's BN), pcoef = [sc | sh (| rsc | rsh)];
  // tile column 0 stores h to pdz and its ReLU bits to pmask — the BN apply pass disappears.
  const bf16_t* py;
  const float* pcoef;
  bf16_t* pdz;
  uint8_t* pmask;
  long long pld;
  // mode 3 (256-row kernel): split-K with the fold inside the launch. Every split writes its fp32
  // slab as in mode 1; the workgroup that finishes a tile last (per-tile arrival counter kctr,
  // reset by that workgroup) sums the tile's slabs in split order and writes kout (+= with beta):
  // no separate fold launch re-reading every slab over the whole chip.
  float* kout;
  int* kctr;
  // Row sums of the A operand over this launch's K range (gemm256_kernel RS = 1: the weight
  // gradient dW = dY^T.X also yields the bias gradient colsum(dY) = rowsum(dY^T)): partial slab
  // rsum[(blockIdx.y * tiles_n + tile_n) * M + m], each (split, tile column) workgroup covering the
  // K-tiles kt with (kt - kt0) % tiles_n == tile_n; the host folds the slabs.
  float* rsum;
};

__device__ __forceinline__ bool beta_row(const EpiParams& E, int m) {
  if (!E.bH) return true;
  const int hw = m % (E.bH * E.bW);
  const int h = hw / E.bW, w = hw - h * E.bW;
  return !((h | w) & 1);
}

__device__ __forceinline__ float epi_alpha(const EpiParams& E) {
  float a = E.alpha;
  if (E.ascale0) a *= *E.ascale0;
  if (E.ascale1) a *= *E.ascale1;
  return a;
}

__device__ __forceinline__ long long out_row(const EpiParams& E, int m) {
  if (!E.remap) return m;
  const int pq = E.rP * E.rQ;
  const int n = m / pq, rem = m - n * pq;
  const int p = rem / E.rQ, q = rem - p * E.rQ;
  return (static_cast<long long>(n) * E.rOH + p * E.rs) * E.rOW + q * E.rs;
}

// Row loop of the bf16 epilogues (both kernels): one thread owns 16-B column chunk `c` of
// rows r0, r0+RPP, ... of the LDS-staged tile. Rows go in batches of EB with every
// residual / accumulate (beta) load of the batch issued before any of them is used: with one
// workgroup per CU (LDS-bound tiles) a load-use per row left the epilogue latency-bound,
// which is what capped the K <= 128 ResNet 1x1 GEMMs at ~50% of HBM bandwidth.
template <int BM, int RPP, int PITCH, bool PF, int EBMAX = 8>
__device__ __forceinline__ void epi_rows(const EpiParams& E, const char* smem, int c, int r0, int n, int m0, int M,
                                         int N, bool vst, bool vres, const float (&bias8)[8], float (&s8)[8],
                                         float (&q8)[8], float (&r8)[8]) {
  constexpr int NR = (BM + RPP - 1) / RPP;
  constexpr int EB = !PF ? 1 : (NR < EBMAX ? NR : EBMAX);  // 16 spills (measured +12 % step time)
  bf16_t* out = static_cast<bf16_t*>(E.out);
  if (n >= N) return;
  if (!PF && !E.bias && !E.residual && !E.aux && E.act == kActNone && !E.remap && vst) {
    // plain store (+ BN statistics): the staged tile already holds the rounded bf16 result, so
    // each 16-B chunk goes LDS -> global untouched (no unpack / bias / repack per element) and
    // the row pointer advances by a constant instead of a 64-bit multiply per row
    bf16_t* op = out + static_cast<long long>(m0 + r0) * E.ldo + n;
    const long long step = static_cast<long long>(RPP) * E.ldo;
    const int rmax = min(BM, M - m0);
#pragma unroll 4
    for (int r = r0; r < rmax; r += RPP, op += step) {
      const uint4 v = *reinterpret_cast<const uint4*>(smem + r * PITCH + c * 16);
      *reinterpret_cast<uint4*>(op) = v;
      if (E.stat) {
        float sv[8];
        unpack8(v, sv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s8[j] += sv[j];
          q8[j] += sv[j] * sv[j];
        }
      }
    }
    return;
  }
#pragma unroll 1
  for (int rb = r0; rb < BM; rb += RPP * EB) {
    uint4 pres[EB], pold[EB], pby[EB], pby2[EB];
    uint32_t pmb[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int r = rb + u * RPP, m = m0 + r;
      if (r < BM && m < M) {
        if (E.residual && vres) pres[u] = *reinterpret_cast<const uint4*>(E.residual + static_cast<long long>(m) * E.ldr + n);
        if (E.beta && vst) {
          pold[u] = beta_row(E, m) ? *reinterpret_cast<const uint4*>(out + out_row(E, m) * E.ldo + n)
                                   : make_uint4(0, 0, 0, 0);
        }
        if (E.by) {  // vst is guaranteed by the host (N % 8 == 0, ldo % 8 == 0)
          const long long o = out_row(E, m) * E.ldo + n;
          pby[u] = *reinterpret_cast<const uint4*>(E.by + o);
          if (E.by2) pby2[u] = *reinterpret_cast<const uint4*>(E.by2 + o);
          pmb[u] = E.bmask ? E.bmask[o >> 3] : 0xffu;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int r = rb + u * RPP, m = m0 + r;
      if (r >= BM || m >= M) break;
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(smem + r * PITCH + c * 16), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += bias8[j];
      if (E.residual) {
        const bf16_t* rp = E.residual + static_cast<long long>(m) * E.ldr + n;
        float rv[8];
        if (vres) {
          unpack8(pres[u], rv);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) rv[j] = n + j < N ? bf2f(rp[j]) : 0.f;
        }
        if (E.act == kActDGelu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] *= gelu_tanh_grad(rv[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] += rv[j];
        }
      }
      bf16_t* op = out + out_row(E, m) * E.ldo + n;
      if (E.beta) {
        float ov[8];
        if (vst) {
          unpack8(pold[u], ov);
        } else {
          const bool br = beta_row(E, m);
#pragma unroll
          for (int j = 0; j < 8; ++j) ov[j] = (br && n + j < N) ? bf2f(op[j]) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += ov[j];
      }
      if (E.aux) {
        bf16_t* ap = E.aux + out_row(E, m) * E.ldo + n;
        const uint4 pa = pack8(f);
        if (vst) {
          *reinterpret_cast<uint4*>(ap) = pa;
        } else {
          const uint32_t w[4] = {pa.x, pa.y, pa.z, pa.w};
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (n + j < N) ap[j] = static_cast<bf16_t>((w[j >> 1] >> (16 * (j & 1))) & 0xffff);
        }
      }
      if (E.act == kActRelu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = relu(f[j]);
      } else if (E.act == kActGelu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = gelu_tanh(f[j]);
      } else if (E.act == kActTanh) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = tanhf(f[j]);
      }
      if (E.by) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (pmb[u] >> j) & 1u ? f[j] : 0.f;
      }
      const uint4 packed = pack8(f);
      if (vst) {
        *reinterpret_cast<uint4*>(op) = packed;
      } else {
        const uint32_t w[4] = {packed.x, packed.y, packed.z, packed.w};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (n + j < N) op[j] = static_cast<bf16_t>((w[j >> 1] >> (16 * (j & 1))) & 0xffff);
      }
      if (E.by) {
        float sv[8], yv[8];
        unpack8(packed, sv);  // statistics of the gradient actually stored
        unpack8(pby[u], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s8[j] += sv[j];
          q8[j] += sv[j] * yv[j];
        }
        if (E.by2) {
          unpack8(pby2[u], yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) r8[j] += sv[j] * yv[j];
        }
      } else if (E.stat) {
        float sv[8];
        unpack8(packed, sv);  // statistics of the values actually stored
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s8[j] += sv[j];
          q8[j] += sv[j] * sv[j];
        }
      }
    }
  }
}

template <int BM, int BN>
__device__ __forceinline__ void epilogue(const EpiParams& E, f32x4_t (&acc)[BM / 32][BN / 32], int m0, int n0,
                                         int mwave, int nwave, int lane, int M, int N, int split, int tile_m,
                                         char* smem) {
  static_assert(BM * (BN * 2 + 16) + 4 * 3 * BN * 4 <= 2 * (BM + BN) * BK * 2, "staged epilogue must fit in LDS");
  constexpr int TM = BM / 32, TN = BN / 32;
  const int g = lane >> 4, i16 = lane & 15;
  const float alpha_e = epi_alpha(E);
  if (E.mode != 0) {
    float* out = static_cast<float*>(E.out) + (E.mode == 1 ? split * E.slab_stride : 0);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int m = mwave + tm * 16 + i16;
      if (m >= M) continue;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = nwave + tn * 16 + 4 * g;
        f32x4_t v = acc[tm][tn] * alpha_e;
        float* o = out + static_cast<long long>(m) * E.ldo + n;
        if (n + 3 < N && (E.ldo & 3) == 0) {
          if (E.beta) v += *reinterpret_cast<const f32x4_t*>(o);
          *reinterpret_cast<f32x4_t*>(o) = v;
        } else {
          #pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n + j < N) o[j] = v[j] + (E.beta ? o[j] : 0.f);
        }
      }
    }
    return;
  }
  // ---- bf16 output: stage the tile through LDS (the K loop ended on a barrier, so the
  // operand buffers are free), then every thread stores whole 16-B chunks of full rows:
  // one wave-instruction writes 4 x 256 contiguous bytes instead of 16 x 32-B segments.
  constexpr int PITCH = BN * 2 + 16;  // 16-B aligned rows; +16 B breaks the bank period
  const int tid = threadIdx.x;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int r = mwave - m0 + tm * 16 + i16, c = nwave - n0 + tn * 16 + 4 * g;
      const f32x4_t v = acc[tm][tn] * alpha_e;
      uint2 w;
      w.x = pack_bf16x2(v[0], v[1]);
      w.y = pack_bf16x2(v[2], v[3]);
      *reinterpret_cast<uint2*>(smem + r * PITCH + c * 2) = w;
    }
  __syncthreads();
  constexpr int CPR = BN / 8;       // 16-B chunks per row
  constexpr int RPP = NTHR / CPR;   // rows per pass
  const int c = tid % CPR, r0 = tid / CPR;
  const int n = n0 + c * 8;
  const bool nfull = n + 8 <= N;
  const bool vst = nfull && (E.ldo & 7) == 0;
  const bool vres = nfull && (E.ldr & 7) == 0;
  float bias8[8], s8[8], q8[8], r8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bias8[j] = (E.bias && n + j < N) ? E.bias[n + j] : 0.f;
    s8[j] = q8[j] = r8[j] = 0.f;
  }
  if (E.beta || E.residual || E.by)  // batched loads only where there are loads (no cost to plain stores)
    epi_rows<BM, RPP, PITCH, true>(E, smem, c, r0, n, m0, M, N, vst, vres, bias8, s8, q8, r8);
  else
    epi_rows<BM, RPP, PITCH, false>(E, smem, c, r0, n, m0, M, N, vst, vres, bias8, s8, q8, r8);
  if (E.stat) {
    // lanes sharing a chunk column: lane % CPR equal -> reduce over the wave, then over 4 waves.
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        s8[j] += __shfl_xor(s8[j], o, 64);
        q8[j] += __shfl_xor(q8[j], o, 64);
        if (E.stat2) r8[j] += __shfl_xor(r8[j], o, 64);
      }
    }
    float* red = reinterpret_cast<float*>(smem + BM * PITCH);  // [4 waves][3][BN]
    const int w = tid >> 6;
    if ((tid & 63) < CPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(w * 3 + 0) * BN + c * 8 + j] = s8[j];
        red[(w * 3 + 1) * BN + c * 8 + j] = q8[j];
        red[(w * 3 + 2) * BN + c * 8 + j] = r8[j];
      }
    }
    __syncthreads();
    for (int t = tid; t < BN; t += NTHR) {
      if (n0 + t < N) {
        float ss = 0.f, qq = 0.f, rr = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ss += red[(k * 3 + 0) * BN + t];
          qq += red[(k * 3 + 1) * BN + t];
          rr += red[(k * 3 + 2) * BN + t];
        }
        E.stat[(static_cast<long long>(tile_m) * 2 + 0) * N + n0 + t] = ss;
        E.stat[(static_cast<long long>(tile_m) * 2 + 1) * N + n0 + t] = qq;
        if (E.stat2) {
          E.stat2[(static_cast<long long>(tile_m) * 2 + 0) * N + n0 + t] = ss;
          E.stat2[(static_cast<long long>(tile_m) * 2 + 1) * N + n0 + t] = rr;
        }
      }
    }
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <int BM, int BN, class LA, class LB>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(typename LA::Params pa, typename LB::Params pb, EpiParams pe,
                                                      int M, int N, int K, int tiles_m, int tiles_n, int kt_per_split,
                                                      long long bsa = 0, long long bsb = 0, long long bso = 0) {
  __shared__ __attribute__((aligned(16))) char smem[2 * (LA::BYTES + LB::BYTES)];
  // strided batch on grid z (dense operands only; element strides, output stride in elements of
  // the epilogue's output type): one launch for a batched MatMul
  if constexpr (std::is_same_v<typename LA::Params, DenseParams> && std::is_same_v<typename LB::Params, DenseParams>) {
    if (gridDim.z > 1) {
      pa.p += blockIdx.z * bsa;
      pb.p += blockIdx.z * bsb;
      pe.out = static_cast<char*>(pe.out) + blockIdx.z * bso * (pe.mode == 0 ? 2 : 4);
    }
  }
  const int nblk = tiles_m * tiles_n;
  // split-K (gridDim.y > 1): the XCD-aware order runs over (tile, split) so the output tiles of
  // one K-split — which read the same K rows of both operands (a weight gradient's dy and
  // im2col slices) — share an XCD's L2; with few tiles (stem 7x7: 4) each slice was otherwise
  // fetched from HBM by up to 4 XCDs
  int t, split;
  if (gridDim.y == 1) {
    t = xcd_remap(blockIdx.x, nblk);
    split = 0;
  } else {
    const int w = xcd_remap(blockIdx.x + blockIdx.y * nblk, nblk * gridDim.y);
    t = w % nblk;
    split = w / nblk;
  }
  const int tile_n = t % tiles_n, tile_m = t / tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int TM = BM / 32, TN = BN / 32;

  char* const sA0 = smem;
  char* const sB0 = smem + 2 * LA::BYTES;

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ktiles = (K + BK - 1) / BK;
  const int kt0 = split * kt_per_split;
  const int kt1 = min(kt0 + kt_per_split, ktiles);

  LA la;
  LB lb;
  la.init(pa, m0, tid);
  lb.init(pb, n0, tid);
  if (kt0 < kt1) {
    la.load(kt0 * BK);
    lb.load(kt0 * BK);
    la.store(sA0, tid);
    lb.store(sB0, tid);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    const bool nxt = kt + 1 < kt1;
    if (nxt) {
      la.load((kt + 1) * BK);
      lb.load((kt + 1) * BK);
    }
    const char* sa = sA0 + cur * LA::BYTES;
    const char* sb = sB0 + cur * LB::BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = LA::frag(sa, wm * (BM / 2) + a * 16, ks, lane);
#pragma unroll
      for (int b = 0; b < TN; ++b) bfr[b] = LB::frag(sb, wn * (BN / 2) + b * 16, ks, lane);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
    }
    if (nxt) {
      la.store(sA0 + (cur ^ 1) * LA::BYTES, tid);
      lb.store(sB0 + (cur ^ 1) * LB::BYTES, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
  epilogue<BM, BN>(pe, acc, m0, n0, m0 + wm * (BM / 2), n0 + wn * (BN / 2), lane, M, N, split, tile_m, smem);
}

// Split-K reduction of fp32 slabs ws[splits][n] into out (+= when beta), deterministic, no
// atomics, no memset. One pass when the output alone gives enough threads; otherwise pass 1
// folds each group of `per` slabs into the group's first slab IN PLACE (every thread reads
// and writes only its own elements) with 4 independent loads in flight per thread, and
// pass 2 sums the group heads. The group count is chosen so pass 1 runs ~2^19 threads (the
// wgrad slabs are tens of MB; the old atomic reducer plus its memset ran at ~1.7 TB/s).
__global__ __launch_bounds__(256) void splitk_fold_kernel(float* __restrict__ ws, int splits, long long n, int per,
                                                          float* __restrict__ out, int beta) {
  const long long i4 = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  const int s0 = blockIdx.y * per, s1 = min(splits, s0 + per);
  // out == nullptr: write the group sum to slab s0 (pass 1); else out (+)= sum (single pass / pass 2,
  // where the "slabs" are the group heads: stride per*n)
  if (i4 + 3 < n) {
    f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    int k = s0;
    for (; k + 3 < s1; k += 4) {
      a0 += *reinterpret_cast<const f32x4_t*>(ws + k * n + i4);
      a1 += *reinterpret_cast<const f32x4_t*>(ws + (k + 1) * n + i4);
      a2 += *reinterpret_cast<const f32x4_t*>(ws + (k + 2) * n + i4);
      a3 += *reinterpret_cast<const f32x4_t*>(ws + (k + 3) * n + i4);
    }
    for (; k < s1; ++k) a0 += *reinterpret_cast<const f32x4_t*>(ws + k * n + i4);
    f32x4_t sum = (a0 + a1) + (a2 + a3);
    if (out) {
      if (beta) sum += *reinterpret_cast<const f32x4_t*>(out + i4);
      *reinterpret_cast<f32x4_t*>(out + i4) = sum;
    } else {
      *reinterpret_cast<f32x4_t*>(ws + s0 * n + i4) = sum;
    }
  } else {
    for (long long i = i4; i < n; ++i) {
      float t = 0.f;
      for (int k = s0; k < s1; ++k) t += ws[k * n + i];
      if (out)
        out[i] = t + (beta ? out[i] : 0.f);
      else
        ws[s0 * n + i] = t;
    }
  }
}

// pass 2: out[i] (+)= sum over g of ws[g*per*n + i]
__global__ __launch_bounds__(256) void splitk_heads_kernel(const float* __restrict__ ws, int groups, int per,
                                                           long long n, float* __restrict__ out, int beta) {
  const long long i4 = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  const long long gs = static_cast<long long>(per) * n;
  if (i4 + 3 < n) {
    f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
    int g = 0;
    for (; g + 1 < groups; g += 2) {
      a0 += *reinterpret_cast<const f32x4_t*>(ws + g * gs + i4);
      a1 += *reinterpret_cast<const f32x4_t*>(ws + (g + 1) * gs + i4);
    }
    if (g < groups) a0 += *reinterpret_cast<const f32x4_t*>(ws + g * gs + i4);
    f32x4_t sum = a0 + a1;
    if (beta) sum += *reinterpret_cast<const f32x4_t*>(out + i4);
    *reinterpret_cast<f32x4_t*>(out + i4) = sum;
  } else {
    for (long long i = i4; i < n; ++i) {
      float t = 0.f;
      for (int g = 0; g < groups; ++g) t += ws[g * gs + i];
      out[i] = t + (beta ? out[i] : 0.f);
    }
  }
}

hipError_t splitk_reduce(const float* ws_c, int splits, long long n, float* out, int beta, hipStream_t st) {
  float* ws = const_cast<float*>(ws_c);  // pass 1 folds in place (the slabs are the caller's scratch)
  // TTD_DIAG_SKIP_FOLD=1: diagnostic only (wrong gradients): measures what the fold passes cost a step
  static const bool diag_skip = [] { const char* e = getenv("TTD_DIAG_SKIP_FOLD"); return e && atoi(e) != 0; }();
  if (diag_skip) return hipSuccess;
  const long long vec = (n + 3) / 4;
  const int bx = ceil_div(vec, 256);
  long long want = ((1LL << 19) + vec - 1) / vec;  // groups for ~2^19 pass-1 threads
  int groups = static_cast<int>(want < 1 ? 1 : (want > splits ? splits : want));
  int per = ceil_div(splits, groups);
  if (per < 4 && splits >= 4) per = 4;  // at least 4 slabs per group (independent loads)
  groups = ceil_div(splits, per);
  if (groups <= 1) {
    hipLaunchKernelGGL(splitk_fold_kernel, dim3(bx, 1), dim3(256), 0, st, ws, splits, n, splits, out, beta);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(splitk_fold_kernel, dim3(bx, groups), dim3(256), 0, st, ws, splits, n, per,
                     static_cast<float*>(nullptr), 0);
  hipLaunchKernelGGL(splitk_heads_kernel, dim3(bx), dim3(256), 0, st, ws, groups, per, n, out, beta);
  return hipGetLastError();
}

// integer environment switch (A/B runs)
inline int getenv_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// ------------------------------------------------------------------ 256-row LDS-DMA GEMM
// Large-GEMM / large-conv path: 256 x BN x (128 B of K) tile, BN in {256, 128}, 8 waves,
// ~1 workgroup per CU. Operand tiles stream global -> LDS with global_load_lds_dwordx4 (no
// VGPR staging, no ds_write pass); the XOR swizzle is applied on the per-lane SOURCE address
// so the LDS image stays lane-linear. Operand policies (A: rows = M, B: rows = N):
//   OpDenseK   element (row, k) at p[row*ld + k]        (bf16, or fp8 e4m3/e5m2)
//   OpDenseMN  element (k, row) at p[k*ld + row]        (bf16)
//   OpConvK    implicit-GEMM conv row gather (fwd: x patch, dgrad: dy patch; C % (64|128))
//   OpWgradMN  implicit-GEMM im2col columns for the weight gradient (bf16)
// Padding / out-of-range rows read a zero page (DMA cannot zero-fill), so convolutions need
// no masking in the MFMA loop.
//
// Each operand tile is split in two halves (A0/A1: 128 rows each, B0/B1: BN/2 rows). Wave
// (wm, wn) owns rows {h*128 + wm*64 + [0,64)} and cols {h'*BN/2 + wn*BN/8 + [0,BN/8)}:
// four quadrants, one per phase, ordered (A0,B0) (A0,B1) (A1,B1) (A1,B0) so every fragment
// is read from LDS once per K-tile (B1 behind q0's MFMAs, A1 behind q1's, the next tile's
// A0/B0 behind q3's) and each phase reloads one half no wave reads any more:
//   q0 -> (T+1).A1, q1 -> (T+1).B0, q2 -> (T+2).A0, q3 -> (T+2).B1.
// Barriers only at q2 (WAR for A0) and q3 (after a counted s_waitcnt vmcnt that retires
// tile T+1 but leaves (T+2).A0 in flight; publishes T+1's DMA to every wave). All LDS lives
// in one __shared__ array; s_setprio(1) brackets each MFMA cluster.
// fp8: K-tile = 128 elements, v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales
// (2x the bf16 MFMA rate); A and B fragments take the same 32 contiguous k per lane group,
// so the product is independent of the instruction's internal k order.
namespace big {
constexpr int BM = 256, THR = 512;

// zero page for padded / out-of-range DMA sources (static device memory is zero-filled)
__device__ __attribute__((aligned(16))) unsigned char g_zero[256];

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((ext_vector_type(8))) int i32x8_t;

template <int HROWS>
__device__ __forceinline__ int swz_mn(int k) {
  if constexpr (HROWS == 128)
    return (k & 3) | ((k >> 1) & 4);
  else
    return ((k >> 1) & 1) | ((k >> 2) & 2);
}

__device__ __forceinline__ void glds(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(lds), 16, 0, 0);
}

// The same DMA as inline asm, for the MN-major operand policies: the compiler tracks the builtin
// as an LDS write it cannot disambiguate from the ds_read_b64_tr_b16 fragment reads, so every
// MN-major main loop got an s_waitcnt vmcnt(0) in front of its first transposed read — a full
// drain of the K-tile + 2 prefetch on every K-tile. Untracked, these pieces are retired only by
// the kernel's own counted waits (in-order vmcnt retirement: the compiler's waits for its own
// loads can only get stronger from extra outstanding pieces, never weaker). M0 is saved and
// restored. A kernel gains only if none of its operands uses the builtin.
__device__ __forceinline__ void glds_u(const void* src, char* lds) {
#ifdef TTD_GLDS_BUILTIN  // A/B builds only (tools/build_alt_lib.py --flags=-DTTD_GLDS_BUILTIN)
  glds(src, lds);
  return;
#endif
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<size_t>((lds_void_t*)(lds))));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l));
}

struct DenseP {
  const void* p;
  long long ld;   // elements
  int rows;
};

struct ConvP {  // implicit-GEMM geometry: source tensor [Nimg, Hs, Ws, Cs]; GEMM rows on the (P, Q) grid
  const void* x;
  int Hs, Ws, Cs;
  int P, Q;
  int R, S;
  int sh, sw, ph, pw, dh, dw;
  int rows;
};

// ---- dense K-major: half = HROWS rows x 128 B
template <int HROWS, int ESZ, int T = THR>
struct OpDenseK {
  using Params = DenseP;
  static constexpr int THREADS = T;
  static constexpr int G = HROWS * 8 / T;  // glds per wave per half
  const char* src[2][G];
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int q = i * T + tid;
        const int row = q >> 3, slot = q & 7;
        const int chunk = slot ^ ((row >> 1) & 7);
        const int r = min(row0 + h * HROWS + row, P.rows - 1);
        src[h][i] = static_cast<const char*>(P.p) + (static_cast<long long>(r) * P.ld) * ESZ + chunk * 16;
      }
  }
  template <int H>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < G; ++i) glds(src[H][i] + static_cast<long long>(kt) * 128, lds + (i * T + wave * 64) * 16);
  }
};

// K-major dense operand whose DMA is the untracked asm form (glds_u): for kernels whose other
// operand is MN-major, so no tracked LDS-DMA is left to force vmcnt(0) drains in front of the
// transposed fragment reads (the K-major x K-major kernels keep the builtin: there the compiler
// inserts no such waits, and the asm form's 64-bit address pairs spilled the persistent kernel)
template <int HROWS, int ESZ, int T = THR>
struct OpDenseKU : OpDenseK<HROWS, ESZ, T> {
  template <int H>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < OpDenseK<HROWS, ESZ, T>::G; ++i)
      glds_u(this->src[H][i] + static_cast<long long>(kt) * 128, lds + (i * T + wave * 64) * 16);
  }
};

// ---- dense MN-major (bf16): half = HROWS cols x 64 k
template <int HROWS, int T = THR>
struct OpDenseMN {
  using Params = DenseP;
  static constexpr int THREADS = T;
  static constexpr int G = HROWS * 8 / T;
  static constexpr int CPR = HROWS / 8;  // 16-B chunks per k-row
  const char* src[2][G];
  long long kstep;
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int q = i * T + tid;
        const int k = q / CPR, j = q % CPR;
        const int col = ((((j >> 1) ^ swz_mn<HROWS>(k))) << 4) + (j & 1) * 8;
        const int c = min(row0 + h * HROWS + col, P.rows - 8);
        src[h][i] = static_cast<const char*>(P.p) + (static_cast<long long>(k) * P.ld + c) * 2;
      }
    kstep = 64 * P.ld * 2;
  }
  template <int H>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < G; ++i) glds_u(src[H][i] + kt * kstep, lds + (i * T + wave * 64) * 16);
  }
};

// ---- implicit-GEMM conv rows (K-major): row = output pixel of the (P, Q) grid, k = (r, s, c);
// one K-tile (128 B) lies inside one tap (requires Cs*ESZ % 128 == 0).
template <int HROWS, int ESZ, bool DGRAD, bool UNIT_STRIDE = false, int T = THR>
struct OpConvK {
  using Params = ConvP;
  static constexpr int THREADS = T;
  static constexpr int G = HROWS * 8 / T;
  static constexpr int KT = 128 / ESZ;  // elements per K-tile
  const char* x;
  int Hs, Ws, Cs, S, sh, sw, dh, dw, tid;
  int img[2][G], hb[2][G], wb[2][G];  // img < 0: row beyond M (reads the zero page)
  __device__ __forceinline__ void init(const Params& P, int row0, int tid_) {
    x = static_cast<const char*>(P.x);
    Hs = P.Hs; Ws = P.Ws; Cs = P.Cs; S = P.S; sh = P.sh; sw = P.sw; dh = P.dh; dw = P.dw;
    tid = tid_;
    const int pq = P.P * P.Q;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int row = (i * T + tid) >> 3;
        const int m = row0 + h * HROWS + row;
        const bool ok = m < P.rows;
        const int mm = ok ? m : 0;
        const int n = mm / pq, rem = mm - n * pq;
        const int p = rem / P.Q, qq = rem - p * P.Q;
        img[h][i] = ok ? n * P.Hs : -1;
        if (DGRAD) {
          hb[h][i] = p + P.ph;
          wb[h][i] = qq + P.pw;
        } else {
          hb[h][i] = p * P.sh - P.ph;
          wb[h][i] = qq * P.sw - P.pw;
        }
      }
  }
  template <int H>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
    const int k0 = kt * KT;
    const int tap = k0 / Cs, c0 = k0 - tap * Cs;
    const int rr = tap / S, ss = tap - rr * S;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int row = (i * T + tid) >> 3;
      const int coff = (((tid & 7) ^ ((row >> 1) & 7))) * 16;
      int hh, ww;
      bool v = img[H][i] >= 0;
      if (DGRAD && UNIT_STRIDE) {
        hh = hb[H][i] - rr * dh;
        ww = wb[H][i] - ss * dw;
        v = v && hh >= 0 && ww >= 0;
      } else if (DGRAD) {
        const int hn = hb[H][i] - rr * dh, wn = wb[H][i] - ss * dw;
        hh = hn / sh;
        ww = wn / sw;
        v = v && hn >= 0 && wn >= 0 && hh * sh == hn && ww * sw == wn;
      } else {
        hh = hb[H][i] + rr * dh;
        ww = wb[H][i] + ss * dw;
        v = v && hh >= 0 && ww >= 0;
      }
      v = v && hh < Hs && ww < Ws;
      const char* s = v ? x + ((static_cast<long long>(img[H][i] + hh) * Ws + ww) * Cs + c0) * ESZ + coff
                        : reinterpret_cast<const char*>(g_zero) + coff;
      glds(s, lds + (i * T + wave * 64) * 16);
    }
  }
};

// ---- weight-gradient im2col columns (MN-major, bf16): k = output pixel, column = (r, s, c)
template <int HROWS, int T = THR>
struct OpWgradMN {
  using Params = ConvP;
  static constexpr int THREADS = T;
  static constexpr int G = HROWS * 8 / T;
  static constexpr int CPR = HROWS / 8;
  const char* x;
  int H, W, C, pq, Q, sh, sw;
  int krow[2][G], roff[2][G], soff[2][G], cc[2][G];
  bool cok[2][G];
  // (incremental pixel tracking as in MNConvGather was tried here: the extra state spilled this
  // register-bound 256-row kernel to scratch and doubled its time, so it keeps the divisions)
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    x = static_cast<const char*>(P.x);
    H = P.Hs; W = P.Ws; C = P.Cs; pq = P.P * P.Q; Q = P.Q; sh = P.sh; sw = P.sw;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int q = i * T + tid;
        const int k = q / CPR, j = q % CPR;
        const int col = row0 + h * HROWS + ((((j >> 1) ^ swz_mn<HROWS>(k))) << 4) + (j & 1) * 8;
        krow[h][i] = k;
        cok[h][i] = col < P.rows;
        const int cl = cok[h][i] ? col : 0;
        const int tap = cl / C, c = cl - tap * C;
        const int rr = tap / P.S, ss = tap - rr * P.S;
        roff[h][i] = rr * P.dh - P.ph;
        soff[h][i] = ss * P.dw - P.pw;
        cc[h][i] = c;
      }
  }
  template <int HH>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int k = kt * 64 + krow[HH][i];
      const int n = k / pq, rem = k - n * pq;
      const int p = rem / Q, qq = rem - p * Q;
      const int hh = p * sh + roff[HH][i], ww = qq * sw + soff[HH][i];
      const bool v = cok[HH][i] && hh >= 0 && ww >= 0 && hh < H && ww < W;
      const char* s = v ? x + ((static_cast<long long>(n * H + hh) * W + ww) * C + cc[HH][i]) * 2
                        : reinterpret_cast<const char*>(g_zero);
      glds_u(s, lds + (i * T + wave * 64) * 16);
    }
  }
};

// ---- fp8 MN-major operands (the fp8 weight gradient: k = pixel, column = output channel or
// im2col column (r, s, c); OCP e4m3 / e5m2 bytes). Half = 128 columns x 128 k (one byte each),
// the same 16 KB as a bf16 half: k-row r holds its 128 columns as 8 16-B slots, slot j stored
// at j ^ mn8_swz(r), so the 16 k-rows one ds_read_b64_tr_b8 of a 32-lane group touches land on
// 16 distinct 4-bank groups (rows alternate bank halves; within a half the 8 rows of one parity
// take slots m | 4g for m = (r >> 1) & 3 and the lane group g = bit 5 of r).
// HROWS = 64 (the B half of a 256 x 128 tile): k-rows of 64 B (4 slots); a 32-lane read covers
// 4 bank quarters (r & 3), and the 4 rows of one quarter take slots (bit 2 of r) | (g << 1).
template <int HROWS>
__device__ __forceinline__ int mn8_swz(int k) {
  if constexpr (HROWS == 128)
    return ((k >> 1) & 3) | ((k >> 3) & 4);
  else
    return ((k >> 2) & 1) | ((k >> 4) & 2);
}
template <int HROWS>
__device__ __forceinline__ int mn8_off(int k, int col) {
  return k * HROWS + (((col >> 4) ^ mn8_swz<HROWS>(k)) << 4) + (col & 15);
}

template <int HROWS, int T = THR>
struct OpDenseMN8 {  // element (k, row) at p[k * ld + row] (bytes); ld % 16 == 0, rows % 16 == 0
  static_assert(HROWS == 128 || HROWS == 64, "fp8 MN-major halves are 128 or 64 columns");
  static constexpr int SPR = HROWS / 16;  // 16-B slots per k-row
  using Params = DenseP;
  static constexpr int THREADS = T;
  static constexpr int G = HROWS * 8 / T;
  // 32-bit piece offsets from the uniform base (k < 128 rows of ld <= 2^24 bytes): 64-bit
  // pointers per piece were reloaded from scratch inside the fp8 main loop
  const char* base;
  int off[2][G];
  long long kstep;
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    base = static_cast<const char*>(P.p);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int q = i * T + tid;
        const int k = q / SPR, j = q % SPR;
        const int c = min(row0 + h * HROWS + ((j ^ mn8_swz<HROWS>(k)) << 4), P.rows - 16);
        off[h][i] = k * static_cast<int>(P.ld) + c;
      }
    kstep = 128 * P.ld;
  }
  template <int H>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
    const char* b = base + kt * kstep;
#pragma unroll
    for (int i = 0; i < G; ++i) glds_u(b + off[H][i], lds + (i * T + wave * 64) * 16);
  }
};

// fp8 im2col columns of the weight gradient (as OpWgradMN; C % 16 == 0 so a 16-column slot stays
// inside one filter tap)
template <int HROWS, int T = THR>
struct OpWgradMN8 {
  static_assert(HROWS == 128 || HROWS == 64, "fp8 MN-major halves are 128 or 64 columns");
  static constexpr int SPR = HROWS / 16;
  using Params = ConvP;
  static constexpr int THREADS = T;
  static constexpr int G = HROWS * 8 / T;
  const char* x;
  int H, W, C, pq, Q, sh, sw;
  // per piece, packed (the unpacked five arrays spilled inside the fp8 main loop, whose i32x8
  // fragments already hold the register file at 256): kc = k | c << 7 (k < 128 pixels of the
  // K-tile, c the channel), rs = (roff + 64) | (soff + 64) << 8 | valid-column << 16
  int kc[2][G], rs[2][G];
  __device__ __forceinline__ void init(const Params& P, int row0, int tid) {
    x = static_cast<const char*>(P.x);
    H = P.Hs; W = P.Ws; C = P.Cs; pq = P.P * P.Q; Q = P.Q; sh = P.sh; sw = P.sw;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int q = i * T + tid;
        const int k = q / SPR, j = q % SPR;
        const int col = row0 + h * HROWS + ((j ^ mn8_swz<HROWS>(k)) << 4);
        const bool ok = col < P.rows;
        const int cl = ok ? col : 0;
        const int tap = cl / C, c = cl - tap * C;
        const int rr = tap / P.S, ss = tap - rr * P.S;
        kc[h][i] = k | (c << 7);
        rs[h][i] = (rr * P.dh - P.ph + 64) | ((ss * P.dw - P.pw + 64) << 8) | (ok ? 1 << 16 : 0);
      }
  }
  template <int HH>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int k = kt * 128 + (kc[HH][i] & 127);
      const int n = k / pq, rem = k - n * pq;
      const int p = rem / Q, qq = rem - p * Q;
      const int hh = p * sh + (rs[HH][i] & 255) - 64, ww = qq * sw + ((rs[HH][i] >> 8) & 255) - 64;
      const bool v = (rs[HH][i] >> 16) && hh >= 0 && ww >= 0 && hh < H && ww < W;
      // one 32-bit byte offset (the host keeps x8 under 4 GiB): as a 64-bit x + c hoisted per
      // piece, the address pairs were spilled inside the main loop
      const uint32_t o = static_cast<uint32_t>((n * H + hh) * W + ww) * static_cast<uint32_t>(C) +
                         static_cast<uint32_t>(kc[HH][i] >> 7);
      const char* s = v ? x + o : reinterpret_cast<const char*>(g_zero);
      glds_u(s, lds + (i * T + wave * 64) * 16);
    }
  }
};

// dense K-major A operand whose tile gets a BN operand prologue (EpiParams::py/pcoef/pdz/pmask):
// MODE 1 BN backward apply, 2 BN forward apply + residual + ReLU, 3 the same with the residual's
// own BN (projection shortcut)
template <int HROWS, int ESZ, int T = THR, int MODE = 1>
struct OpDenseKBN : OpDenseK<HROWS, ESZ, T> {};

template <class OP>
struct Traits {
  static constexpr bool kmaj = true;
  static constexpr int bnpro = 0;
};
template <int HR, int E, int T, int MODE>
struct Traits<OpDenseKBN<HR, E, T, MODE>> {
  static constexpr bool kmaj = true;
  static constexpr int bnpro = MODE;
};
template <int HR, int T>
struct Traits<OpDenseMN<HR, T>> {
  static constexpr bool kmaj = false;
  static constexpr int bnpro = 0;
};
template <int HR, int T>
struct Traits<OpWgradMN<HR, T>> {
  static constexpr bool kmaj = false;
  static constexpr int bnpro = 0;
};
template <int HR, int T>
struct Traits<OpDenseMN8<HR, T>> {
  static constexpr bool kmaj = false;
  static constexpr int bnpro = 0;
};
template <int HR, int T>
struct Traits<OpWgradMN8<HR, T>> {
  static constexpr bool kmaj = false;
  static constexpr int bnpro = 0;
};

// fragment readers
__device__ __forceinline__ bf16x8_t frag_k(const char* lds, int base, int ks, int lane) {
  return lds_read_b128(lds + kmaj_off(base + (lane & 15), ks * 4 + (lane >> 4)));
}
__device__ __forceinline__ i32x8_t frag_k8(const char* lds, int base, int lane) {
  const int row = base + (lane & 15), g = lane >> 4;
  const uint4 lo = *reinterpret_cast<const uint4*>(lds + kmaj_off(row, 2 * g));
  const uint4 hi = *reinterpret_cast<const uint4*>(lds + kmaj_off(row, 2 * g + 1));
  i32x8_t v = {static_cast<int>(lo.x), static_cast<int>(lo.y), static_cast<int>(lo.z), static_cast<int>(lo.w),
               static_cast<int>(hi.x), static_cast<int>(hi.y), static_cast<int>(hi.z), static_cast<int>(hi.w)};
  return v;
}
template <int HROWS>
__device__ __forceinline__ bf16x8_t frag_mn(const char* lds, int colbase, int ks, int lane) {
  return mn_frag<HROWS>(lds, colbase, ks, lane);
}
// fp8 MN-major fragment of v_mfma_scale_f32_16x16x128_f8f6f4: lane (i = lane & 15, g = lane >> 4)
// gets column colbase + i, k = 32 g .. 32 g + 31, as four ds_read_b64_tr_b8 (measured on gfx950,
// tools/probe/tr8_probe.hip: within a 16-lane group, lane l receives byte l % 8 of the 8-byte
// pieces addressed by lanes 2j + (l >= 8), j = 0..7; so lane i addresses k-row k0 + i / 2 at
// column colbase + 8 (i & 1), and every lane ends up with 8 consecutive k of its own column).
template <int HROWS>
__device__ __forceinline__ i32x8_t frag_mn8(const char* lds, int colbase, int lane) {
  typedef __attribute__((ext_vector_type(2))) int i32x2_t;
  typedef __attribute__((address_space(3))) i32x2_t lds_i32x2_t;
  const int i = lane & 15, g = lane >> 4;
  const int col = colbase + 8 * (i & 1);
  i32x8_t v;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 32 * g + 8 * q + (i >> 1);
    const i32x2_t r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2_t*)(lds + mn8_off<HROWS>(k, col)));
    v[2 * q] = r[0];
    v[2 * q + 1] = r[1];
  }
  return v;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- prefetched "feeding BN" epilogue of the 256-row kernel (dgrad with beta accumulate and
// the next BN's backward statistics: by = that BN's conv output, bmask = its ReLU bits, no
// bias / residual / activation / remap / second BN: with the by2 variant instantiated too the
// 256-row kernels spilled). A short-K data gradient spends most of a
// tile in this epilogue, moving 3x the output tile through HBM; with one workgroup per CU the
// generic row loop paid a full load latency per 8-row batch, twice per tile, exposed (ResNet
// c1 dgrads ran at 2.3-3.3 TB/s: tools/dgrad_epi_ab.py). Here a thread's rows go in batches of
// FQ: the first batch is loaded before the accumulators are staged through LDS and every next
// batch before the current one is consumed, so the load latency hides under the staging and
// the stores (two small batches live at a time: no spills next to the live accumulators).
// Same arithmetic and rounding as epi_rows (out = bf16(bf16(acc) + old) * mask, sums of the
// stored values).
constexpr int FQ = 4;  // (8-row batches measured 5-10 % slower on these kernels, ResNet +0.3-0.8 ms)

template <bool BY2>
struct FeedRows {
  uint4 old[FQ], y[FQ], y2[FQ];
  uint32_t mb[FQ];
};

template <int RPP, bool BY2>
__device__ __forceinline__ void feed_load(FeedRows<BY2>& f, const EpiParams& E, int rb, int m0, int M, int n, int N) {
  const bf16_t* out = static_cast<const bf16_t*>(E.out);
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int m = m0 + rb + u * RPP;
    if (m < M && n < N) {
      const long long o = static_cast<long long>(m) * E.ldo + n;
      f.old[u] = (E.beta && beta_row(E, m)) ? *reinterpret_cast<const uint4*>(out + o) : make_uint4(0, 0, 0, 0);
      f.y[u] = *reinterpret_cast<const uint4*>(E.by + o);
      if (BY2 || E.by2) f.y2[u] = *reinterpret_cast<const uint4*>(E.by2 + o);
      f.mb[u] = E.bmask ? E.bmask[o >> 3] : 0xffu;
    }
  }
}

template <int RPP, int PITCH, bool BY2>
__device__ __forceinline__ void feed_rows(const FeedRows<BY2>& f, const EpiParams& E, const char* smem, int c, int rb,
                                          int m0, int M, int n, int N, float (&s8)[8], float (&q8)[8],
                                          float (&r8)[8]) {
  if (n >= N) return;
  bf16_t* out = static_cast<bf16_t*>(E.out);
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int r = rb + u * RPP, m = m0 + r;
    if (m >= M) break;
    float v[8], ov[8], yv[8];
    unpack8(*reinterpret_cast<const uint4*>(smem + r * PITCH + c * 16), v);
    unpack8(f.old[u], ov);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (f.mb[u] >> j) & 1u ? v[j] + ov[j] : 0.f;
    const uint4 packed = pack8(v);
    *reinterpret_cast<uint4*>(out + static_cast<long long>(m) * E.ldo + n) = packed;
    unpack8(packed, v);  // statistics of the gradient actually stored
    unpack8(f.y[u], yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s8[j] += v[j];
      q8[j] += v[j] * yv[j];
    }
    if (BY2 || E.by2) {
      unpack8(f.y2[u], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) r8[j] += v[j] * yv[j];
    }
  }
}

// The whole pipelined feeding epilogue: NR rows per thread in NR / FQ batches.
template <int NR, int RPP, int PITCH, bool BY2, class Stage>
__device__ __forceinline__ void feed_epilogue(const EpiParams& E, char* smem, Stage&& stage, int c, int r0, int m0,
                                              int M, int n, int N, float (&s8)[8], float (&q8)[8], float (&r8)[8]) {
  static_assert(NR % FQ == 0, "rows per thread in whole batches");
  constexpr int NBT = NR / FQ;
  FeedRows<BY2> A, B;
  stage(std::integral_constant<int, 0>{});
  stage(std::integral_constant<int, 1>{});
  feed_load<RPP>(A, E, r0, m0, M, n, N);  // the accumulators are dead: loads overlap the LDS barrier
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();
#pragma unroll
  for (int bt = 0; bt < NBT; bt += 2) {
    if (bt + 1 < NBT) feed_load<RPP>(B, E, r0 + (bt + 1) * FQ * RPP, m0, M, n, N);
    feed_rows<RPP, PITCH>(A, E, smem, c, r0 + bt * FQ * RPP, m0, M, n, N, s8, q8, r8);
    if (bt + 2 < NBT) feed_load<RPP>(A, E, r0 + (bt + 2) * FQ * RPP, m0, M, n, N);
    if (bt + 1 < NBT) feed_rows<RPP, PITCH>(B, E, smem, c, r0 + (bt + 1) * FQ * RPP, m0, M, n, N, s8, q8, r8);
  }
}

template <int BN>
struct Geo {
  static constexpr int BNH = BN / 2;          // B half rows
  static constexpr int AH = 128 * 128;        // A half bytes
  static constexpr int BH = BNH * 128;        // B half bytes
  static constexpr int STAGE = 2 * AH + 2 * BH;
  static constexpr int PITCH = BN * 2 + 16;
  static constexpr int EPI = BM * PITCH + 8 * 3 * BN * 4;  // staged tile + [8 waves][3][BN] statistics
  static constexpr int COEF = 2 * STAGE;  // BN prologue: [2 stages][64 lanes x 16 B] ([3][64] fp32 used)
  static constexpr int SMEM = (2 * STAGE + 2048 > EPI) ? 2 * STAGE + 2048 : EPI;
};

// F8: 0 = bf16, 1 = fp8 e4m3 x e4m3, 2 = e5m2 (A) x e4m3 (B)  (dgrad: gradients in e5m2)
// PP: ping-pong schedule — every quadrant phase is {fragment reads + DMA issue} barrier
// {MFMA cluster} barrier, with the wm = 1 wave half one barrier behind the wm = 0 half, so
// the two waves of a SIMD alternate MFMA clusters and load segments.
template <int BN, class OA, class OB, int F8, int PP = 0, int RS = 0>
__global__ __launch_bounds__(OA::THREADS, 1) void gemm256_kernel(typename OA::Params pa, typename OB::Params pb, EpiParams E,
                                                         int M, int N, int K, int tiles_m, int tiles_n,
                                                         int kt_per_split, int m_base) {
  using Gm = Geo<BN>;
  // T threads = NW waves in a 2 x WN grid: 8 waves (2 per SIMD, 128 x BN/4 each; the shipped
  // shape) or 4 waves (1 per SIMD, 128 x BN/2 each: half the LDS fragment reads per MFMA, but
  // at BN = 256 hipcc spills the 128 fragment + 256 accumulator registers: 5x slower, unused)
  constexpr int T = OA::THREADS, NW = T / 64, WN = NW / 2;
  static_assert(OB::THREADS == T && (NW == 8 || NW == 4), "operand policies must agree on the block size");
  constexpr int BNH = Gm::BNH, WC = BNH / WN, NB = WC / 16, GA = OA::G, GB = OB::G;
  constexpr bool AK = Traits<OA>::kmaj, BKM = Traits<OB>::kmaj;
  static_assert(F8 == 0 || AK == BKM, "fp8 operands: both K-major or both MN-major (OpDenseMN8 / OpWgradMN8)");
  __shared__ __attribute__((aligned(16))) char smem[Gm::SMEM];
  // RS: A-operand row sums (EpiParams::rsum). MN-major A only, PP schedule, fp32 slab / store
  // epilogues (the per-wave sum slots [NW][256] fp32 sit after the coefficient area, inside the
  // bf16 staging region that a mode-1/2 epilogue never uses).
  static_assert(!RS || (!AK && PP == 1 && F8 == 0 && Traits<OA>::bnpro == 0 && BN == 256),
                "row sums: MN-major bf16 A on the ping-pong schedule");
  constexpr int RS_OFF = 2 * Gm::STAGE + 2048;
  static_assert(!RS || RS_OFF + 8 * 256 * 4 <= Gm::SMEM, "row-sum slots fit the shared memory");
  const int nblk = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nblk);
  const int tile_n = t % tiles_n;
  // m_base: first GEMM row of this launch (0 for every launch today); the tile row index used
  // for the BN statistics rows is absolute
  const int tile_m = m_base / BM + t / tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  OA la;
  OB lb;
  la.init(pa, m0, tid);
  lb.init(pb, n0, tid);

  // acc[ha][hb][a][b]: rows ha*128 + wm*64 + a*16, cols hb*BNH + wn*WC + b*16
  f32x4_t acc[2][2][4][NB];
#pragma unroll
  for (int ha = 0; ha < 2; ++ha)
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[ha][hb][a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ktiles = K / (F8 ? 128 : 64);
  const int kt0 = blockIdx.y * kt_per_split;
  const int kt1 = min(kt0 + kt_per_split, ktiles);
  auto buf = [&](int kt) { return smem + ((kt - kt0) & 1) * Gm::STAGE; };
  constexpr int A0 = 0, A1 = Gm::AH, B0 = 2 * Gm::AH, B1 = 2 * Gm::AH + Gm::BH;

  // fragments: [slot][ks][block]; fp8 uses one "ks" of K = 128
  constexpr int KS = F8 ? 1 : 2;
  typedef typename std::conditional<F8 != 0, i32x8_t, bf16x8_t>::type frag_t;
  frag_t fa[2][KS][4], fb[2][KS][NB];
  auto read_a = [&](const char* sA, frag_t (&f)[KS][4]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        if constexpr (F8 != 0 && AK) f[ks][a] = frag_k8(sA, wm * 64 + a * 16, lane);
        else if constexpr (F8 != 0) f[ks][a] = frag_mn8<128>(sA, wm * 64 + a * 16, lane);
        else if constexpr (AK) f[ks][a] = frag_k(sA, wm * 64 + a * 16, ks, lane);
        else f[ks][a] = frag_mn<128>(sA, wm * 64 + a * 16, ks, lane);
      }
  };
  auto read_b = [&](const char* sB, frag_t (&f)[KS][NB]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if constexpr (F8 != 0 && BKM) f[ks][b] = frag_k8(sB, wn * WC + b * 16, lane);
        else if constexpr (F8 != 0) f[ks][b] = frag_mn8<BNH>(sB, wn * WC + b * 16, lane);
        else if constexpr (BKM) f[ks][b] = frag_k(sB, wn * WC + b * 16, ks, lane);
        else f[ks][b] = frag_mn<BNH>(sB, wn * WC + b * 16, ks, lane);
      }
  };
  auto mma = [&](const frag_t (&x)[KS][4], const frag_t (&y)[KS][NB], f32x4_t (&c)[4][NB]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          if constexpr (F8 == 1)
            c[a][b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(y[ks][b], x[ks][a], c[a][b], 0, 0, 0, 127, 0, 127);
          else if constexpr (F8 == 2)  // A (x operand, second arg) in e5m2: blgp = 1
            c[a][b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(y[ks][b], x[ks][a], c[a][b], 0, 1, 0, 127, 0, 127);
          else
            c[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y[ks][b], x[ks][a], c[a][b], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  // issue order per tile: A0, B1, A1, B0 (B0 last) => one counted wait retires a whole tile
  // (a deeper stream — every half issued 4-7 phases ahead with counted waits + barriers at
  // q0/q1/q3 — measured 10-40 % slower on every shape, so the shallow schedule stays)
  if constexpr (PP) {
    // ping-pong: the half with wm = 1 runs one barrier behind. Per K-tile kt (cb = its stage):
    //   P0 (A0,B0): issue (kt+1).A1      P1 (A0,B1): -
    //   P2 (A1,B1): issue (kt+2).A0, (kt+2).B0
    //   P3 (A1,B0): counted wait retiring tile kt+1 (the two kt+2 halves stay in flight),
    //               issue (kt+2).B1
    // RAW: tile kt+1 is read from P0 of kt+1 on, >= 2 barriers after every wave's wait (one
    // more than lockstep needs, for the lag). WAR: a half is re-staged >= 2 phases after the
    // phase that read it (its reads complete before that phase's MFMAs), which with the lag
    // still trails the slower half's reads. The last half of tile kt+1 is issued 3 phases
    // before its wait.
    const bool lag = __builtin_amdgcn_readfirstlane(wm) == 1;
    // RS: thread -> (column group cg of 8 A rows, k-set ks): chunks (ks, cg) and (ks + 32, cg) of
    // a half (the MN-major image's 32-B slot swizzle, OpDenseMN); the four lanes of a wave with
    // the same cg (l, l^16, l^32, l^48) are summed by permlane swaps, and lane cg < 16 adds its
    // wave's partial into the wave's own slots: no atomics, a fixed order -> deterministic.
    float* rs_slot = reinterpret_cast<float*>(smem + RS_OFF) + wave * 256;
    const int rs_cg = lane & 15, rs_ks = tid >> 4;
    const int rs_tn = tile_n, rs_nt = tiles_n;
    auto rs_half = [&](const char* sA, int rbase) {
      if constexpr (RS) {
        float f[8], g2[8];
        const int j0 = ((rs_cg >> 1) ^ swz_mn<128>(rs_ks)) * 2 + (rs_cg & 1);
        unpack8(*reinterpret_cast<const uint4*>(sA + (rs_ks * 16 + j0) * 16), f);
        const int j1 = ((rs_cg >> 1) ^ swz_mn<128>(rs_ks + 32)) * 2 + (rs_cg & 1);
        unpack8(*reinterpret_cast<const uint4*>(sA + ((rs_ks + 32) * 16 + j1) * 16), g2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = f[j] + g2[j];
          const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
          v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
          const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
          f[j] = __uint_as_float(b[0]) + __uint_as_float(b[1]);
        }
        if (lane < 16) {
          float* d = rs_slot + rbase + rs_cg * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) d[j] += f[j];
        }
      }
    };
    if constexpr (RS) {
      if (lane < 64) {
        float* z = reinterpret_cast<float*>(smem + RS_OFF) + wave * 256 + lane * 4;
        *reinterpret_cast<f32x4_t*>(z) = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (kt0 < kt1) {
      char* b0 = buf(kt0);
      la.template issue<0>(b0 + A0, kt0, wave);
      lb.template issue<0>(b0 + B0, kt0, wave);
      lb.template issue<1>(b0 + B1, kt0, wave);
      la.template issue<1>(b0 + A1, kt0, wave);
      if (kt0 + 1 < kt1) {
        char* b1 = buf(kt0 + 1);
        la.template issue<0>(b1 + A0, kt0 + 1, wave);
        lb.template issue<0>(b1 + B0, kt0 + 1, wave);
        lb.template issue<1>(b1 + B1, kt0 + 1, wave);
        wait_vm<GA + 2 * GB>();
      } else {
        wait_vm<0>();
      }
      barrier();
      if (lag) barrier();
    }
    // RS turn counter: K-tile kt is this workgroup's when (kt - kt0) % tiles_n == tile_n, kept as
    // a wave-uniform cycling counter (a run-time modulo is VALU work: it made the condition
    // divergent and the row-sum code ran exec-masked on every K-tile)
    int rs_cnt = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool has1 = kt + 1 < kt1, has2 = kt + 2 < kt1;
      char* cb = buf(kt);
      // P0: (A0, B0)
      read_a(cb + A0, fa[0]);
      read_b(cb + B0, fb[0]);
      const bool rs_on = RS && __builtin_amdgcn_readfirstlane(rs_cnt == rs_tn ? 1 : 0) != 0;
      if constexpr (RS) rs_cnt = rs_cnt + 1 == rs_nt ? 0 : rs_cnt + 1;
      if (rs_on) rs_half(cb + A0, 0);
      if (has1) la.template issue<1>(buf(kt + 1) + A1, kt + 1, wave);
      barrier();
      mma(fa[0], fb[0], acc[0][0]);
      barrier();
      // P1: (A0, B1)
      read_b(cb + B1, fb[1]);
      barrier();
      mma(fa[0], fb[1], acc[0][1]);
      barrier();
      // P2: (A1, B1)
      read_a(cb + A1, fa[1]);
      if (rs_on) rs_half(cb + A1, 128);
      if (has2) {
        la.template issue<0>(cb + A0, kt + 2, wave);
        lb.template issue<0>(cb + B0, kt + 2, wave);
      }
      barrier();
      mma(fa[1], fb[1], acc[1][1]);
      barrier();
      // P3: (A1, B0)
      if (has1) {
        if (has2) wait_vm<GA + GB>(); else wait_vm<0>();
      }
      if (has2) lb.template issue<1>(cb + B1, kt + 2, wave);
      barrier();
      mma(fa[1], fb[0], acc[1][0]);
      barrier();
    }
    if (kt0 < kt1 && !lag) barrier();
  } else {
  // BN-backward operand prologue (OpDenseKBN): every thread's A pieces of a K-tile are the same
  // logical 16-B k-chunk (8 channels) of 4 rows; their y values are loaded into registers one
  // K-tile ahead (before that tile's remaining DMAs, so the counted waits retire them too), the
  // tile's 3 x 64 coefficients are DMA'd next to the operand stages, and once the tile has landed
  // each thread rewrites its own pieces in LDS (one extra barrier per K-tile).
  constexpr int BNP = Traits<OA>::bnpro;
  static_assert(!BNP || (PP == 0 && F8 == 0 && T == THR && GA == 2), "BN prologue: bf16 two-barrier 512-thread path");
  constexpr int NCOEF = BNP == 1 ? 3 : (BNP == 2 ? 2 : 4);  // fp32 [NCOEF][K] arrays in pcoef
  uint4 yv[2][GA];
  const int pchunk = (tid & 7) ^ ((tid >> 4) & 7);
  auto prow = [&](int h, int i) { return m0 + h * 128 + ((i * T + tid) >> 3); };
  auto load_y = [&](int kt) {
    if constexpr (BNP) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          const int r = min(prow(h, i), M - 1);
          yv[h][i] = *reinterpret_cast<const uint4*>(E.py + static_cast<long long>(r) * E.pld + kt * 64 + pchunk * 8);
        }
    }
  };
  auto issue_coef = [&](int kt) {
    if constexpr (BNP) {
      const float* src = lane < 16 * NCOEF ? E.pcoef + static_cast<long long>(lane >> 4) * K + kt * 64 + (lane & 15) * 4
                                           : reinterpret_cast<const float*>(g_zero);
      glds(src, smem + Gm::COEF + ((kt - kt0) & 1) * 1024);
    }
  };
  auto transform = [&](int kt, char* b) {
    if constexpr (BNP) {
      const float* cf = reinterpret_cast<const float*>(smem + Gm::COEF + ((kt - kt0) & 1) * 1024) + pchunk * 8;
      float c0[8], c1[8], c2[8], c3[8];
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        *reinterpret_cast<f32x4_t*>(c0 + j) = *reinterpret_cast<const f32x4_t*>(cf + j);
        *reinterpret_cast<f32x4_t*>(c1 + j) = *reinterpret_cast<const f32x4_t*>(cf + 64 + j);
        if constexpr (NCOEF >= 3) *reinterpret_cast<f32x4_t*>(c2 + j) = *reinterpret_cast<const f32x4_t*>(cf + 128 + j);
        if constexpr (NCOEF >= 4) *reinterpret_cast<f32x4_t*>(c3 + j) = *reinterpret_cast<const f32x4_t*>(cf + 192 + j);
      }
      const bool store = tile_n == 0;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          uint4* q = reinterpret_cast<uint4*>(b + (h ? A1 : A0) + (i * T + tid) * 16);
          float gv[8], yf[8];
          unpack8(*q, gv);
          unpack8(yv[h][i], yf);
          if constexpr (BNP == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] = c0[j] * gv[j] + c1[j] * yf[j] + c2[j];  // = bwd_apply_kernel
          } else {  // = apply_kernel: y*scale + shift, + residual (or its BN), ReLU
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] = gv[j] * c0[j] + c1[j];
            if constexpr (BNP == 3) {
#pragma unroll
              for (int j = 0; j < 8; ++j) gv[j] += yf[j] * c2[j] + c3[j];
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j) gv[j] += yf[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] = relu(gv[j]);
          }
          const uint4 o = pack8(gv);
          *q = o;
          const int r = prow(h, i);
          if (store && r < M) {
            const long long off = static_cast<long long>(r) * E.pld + kt * 64 + pchunk * 8;
            *reinterpret_cast<uint4*>(E.pdz + off) = o;
            if constexpr (BNP != 1) {  // ReLU bit per element of the stored value
              const uint32_t wv[4] = {o.x, o.y, o.z, o.w};
              uint32_t mb = 0;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const uint32_t hh = (wv[j >> 1] >> (16 * (j & 1))) & 0xffffu;
                mb |= ((hh & 0x7fffu) != 0 && !(hh & 0x8000u) ? 1u : 0u) << j;
              }
              E.pmask[off >> 3] = static_cast<uint8_t>(mb);
            }
          }
        }
    }
  };
  if (kt0 < kt1) {
    char* b0 = buf(kt0);
    load_y(kt0);
    issue_coef(kt0);
    la.template issue<0>(b0 + A0, kt0, wave);
    lb.template issue<1>(b0 + B1, kt0, wave);
    la.template issue<1>(b0 + A1, kt0, wave);
    lb.template issue<0>(b0 + B0, kt0, wave);
    if (kt0 + 1 < kt1) {
      char* b1 = buf(kt0 + 1);
      issue_coef(kt0 + 1);
      la.template issue<0>(b1 + A0, kt0 + 1, wave);
      lb.template issue<1>(b1 + B1, kt0 + 1, wave);
      wait_vm<GA + GB>();
    } else {
      wait_vm<0>();
    }
    barrier();
    if constexpr (BNP) {
      transform(kt0, b0);
      barrier();
    }
    read_a(b0 + A0, fa[0]);
    read_b(b0 + B0, fb[0]);
  }
  for (int kt = kt0; kt < kt1; ++kt) {
    const bool has1 = kt + 1 < kt1, has2 = kt + 2 < kt1;
    char* cb = buf(kt);
    // q0: (A0, B0)
    if (has1) {
      load_y(kt + 1);
      la.template issue<1>(buf(kt + 1) + A1, kt + 1, wave);
    }
    mma(fa[0], fb[0], acc[0][0]);
    read_b(cb + B1, fb[1]);
    // q1: (A0, B1)
    if (has1) lb.template issue<0>(buf(kt + 1) + B0, kt + 1, wave);
    mma(fa[0], fb[1], acc[0][1]);
    read_a(cb + A1, fa[1]);
    // q2: (A1, B1)
    barrier();
    if (has2) {
      issue_coef(kt + 2);
      la.template issue<0>(cb + A0, kt + 2, wave);
    }
    mma(fa[1], fb[1], acc[1][1]);
    // q3: (A1, B0); retire tile kt+1 ((kt+2).A0 may stay in flight), prefetch its A0/B0
    if (has1) {
      if (has2) wait_vm<GA>(); else wait_vm<0>();
    }
    barrier();
    if (has2) lb.template issue<1>(cb + B1, kt + 2, wave);
    mma(fa[1], fb[0], acc[1][0]);
    if constexpr (BNP) {
      // after the last MFMA of the tile: the fragment registers are dead here (no spills at
      // BN = 256), and the VALU work still overlaps the MFMAs in flight
      if (has1) {
        transform(kt + 1, buf(kt + 1));
        barrier();
      }
    }
    if (has1) {
      char* nb = buf(kt + 1);
      read_a(nb + A0, fa[0]);
      read_b(nb + B0, fb[0]);
    }
  }
  }
  wait_vm<0>();
  __syncthreads();
  if constexpr (RS) {
    // per-row sum of the eight waves' slots, fixed order
    if (tid < 256 && m0 + tid < M) {
      const float* sl = reinterpret_cast<const float*>(smem + RS_OFF);
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += sl[w * 256 + tid];
      E.rsum[(static_cast<long long>(blockIdx.y) * tiles_n + tile_n) * M + m0 + tid] = v;
    }
  }

  // ---------------------------------------------------------------- epilogue
  const int g = lane >> 4, i16 = lane & 15;
  const float alpha_e = epi_alpha(E);
  if (E.mode != 0) {
    float* out = static_cast<float*>(E.out) + (E.mode == 1 || E.mode == 3 ? blockIdx.y * E.slab_stride : 0);
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int m = m0 + ha * 128 + wm * 64 + a * 16 + i16;
        if (m >= M) continue;
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const int n = n0 + hb * BNH + wn * WC + b * 16 + 4 * g;
            f32x4_t v = acc[ha][hb][a][b] * alpha_e;
            float* o = out + out_row(E, m) * E.ldo + n;
            if (n + 3 < N && (E.ldo & 3) == 0) {
              if (E.beta && E.mode == 2) v += *reinterpret_cast<const f32x4_t*>(o);
              *reinterpret_cast<f32x4_t*>(o) = v;
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (n + j < N) o[j] = v[j] + (E.beta && E.mode == 2 ? o[j] : 0.f);
            }
          }
      }
    if (E.mode == 3) {
      // release this split's slab (device scope: other XCDs' L2s must see it), count arrivals
      __threadfence();
      __syncthreads();
      __shared__ int last_split;
      if (tid == 0) last_split = atomicAdd(E.kctr + t, 1) == static_cast<int>(gridDim.y) - 1;
      __syncthreads();
      if (last_split) {
        __threadfence();  // acquire: the other splits' slabs
        const float* ws = static_cast<const float*>(E.out);
        const int S = gridDim.y;
        float* ko = E.kout;
        for (int q = tid; q < BM * (BN / 4); q += T) {
          const int r = q / (BN / 4), c4 = q - r * (BN / 4);
          const int m = m0 + r, n = n0 + c4 * 4;
          if (m >= M || n >= N) continue;
          const long long o = static_cast<long long>(m) * E.ldo + n;
          if (n + 3 < N && (E.ldo & 3) == 0) {
            f32x4_t v = *reinterpret_cast<const f32x4_t*>(ws + o);
            for (int sp = 1; sp < S; ++sp) v += *reinterpret_cast<const f32x4_t*>(ws + sp * E.slab_stride + o);
            if (E.beta) v += *reinterpret_cast<const f32x4_t*>(ko + o);
            *reinterpret_cast<f32x4_t*>(ko + o) = v;
          } else {
            for (int jj = 0; jj < 4 && n + jj < N; ++jj) {
              float v = ws[o + jj];
              for (int sp = 1; sp < S; ++sp) v += ws[sp * E.slab_stride + o + jj];
              ko[o + jj] = v + (E.beta ? ko[o + jj] : 0.f);
            }
          }
        }
        if (tid == 0) E.kctr[t] = 0;  // ready for the next launch on this counter block
      }
    }
    return;
  }
  constexpr int PITCH = Gm::PITCH;
  constexpr int CPR = BN / 8;     // 16-B chunks per row
  constexpr int RPP = T / CPR;    // rows per pass
  const int c = tid % CPR, r0 = tid / CPR;
  const int n = n0 + c * 8;
  auto stage = [&](auto HA) {  // accumulator half HA -> LDS as bf16 (compile-time index)
    constexpr int ha = decltype(HA)::value;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const int r = ha * 128 + wm * 64 + a * 16 + i16, cc = hb * BNH + wn * WC + b * 16 + 4 * g;
            const f32x4_t v = acc[ha][hb][a][b] * alpha_e;
            *reinterpret_cast<uint2*>(smem + r * PITCH + cc * 2) =
                make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
          }
  };
  float s8[8], q8[8], r8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s8[j] = q8[j] = r8[j] = 0.f;
  // host guarantees for E.by: N % 8 == 0 and ldo % 8 == 0 (whole 16-B chunks)
  const bool feed = E.feed_pf && E.by && !E.residual && !E.bias && E.act == kActNone && !E.remap &&
                    !E.aux && E.stat;
  if (feed) {
    feed_epilogue<BM / RPP, RPP, PITCH, false>(E, smem, stage, c, r0, m0, M, n, N, s8, q8, r8);
  } else {
    stage(std::integral_constant<int, 0>{});
    stage(std::integral_constant<int, 1>{});
    __syncthreads();
    const bool nfull = n + 8 <= N;
    const bool vst = nfull && (E.ldo & 7) == 0;
    const bool vres = nfull && (E.ldr & 7) == 0;
    float bias8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bias8[j] = (E.bias && n + j < N) ? E.bias[n + j] : 0.f;
    if (E.beta || E.residual || E.by)  // batched loads only where there are loads (no cost to plain stores)
      epi_rows<BM, RPP, PITCH, true>(E, smem, c, r0, n, m0, M, N, vst, vres, bias8, s8, q8, r8);
    else
      epi_rows<BM, RPP, PITCH, false>(E, smem, c, r0, n, m0, M, N, vst, vres, bias8, s8, q8, r8);
  }
  if (E.stat) {
    // threads sharing a chunk column c: tid % CPR equal -> within a wave lanes c, c+CPR, ...
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        s8[j] += __shfl_xor(s8[j], o, 64);
        q8[j] += __shfl_xor(q8[j], o, 64);
        if (E.stat2) r8[j] += __shfl_xor(r8[j], o, 64);
      }
    }
    float* red = reinterpret_cast<float*>(smem + BM * PITCH);  // [NW waves][3][BN]
    if (lane < CPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wave * 3 + 0) * BN + c * 8 + j] = s8[j];
        red[(wave * 3 + 1) * BN + c * 8 + j] = q8[j];
        red[(wave * 3 + 2) * BN + c * 8 + j] = r8[j];
      }
    }
    __syncthreads();
    for (int t2 = tid; t2 < BN; t2 += T) {
      if (n0 + t2 < N) {
        float ss = 0.f, qq = 0.f, rr = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
          ss += red[(k * 3 + 0) * BN + t2];
          qq += red[(k * 3 + 1) * BN + t2];
          rr += red[(k * 3 + 2) * BN + t2];
        }
        E.stat[(static_cast<long long>(tile_m) * 2 + 0) * N + n0 + t2] = ss;
        E.stat[(static_cast<long long>(tile_m) * 2 + 1) * N + n0 + t2] = qq;
        if (E.stat2) {
          E.stat2[(static_cast<long long>(tile_m) * 2 + 0) * N + n0 + t2] = ss;
          E.stat2[(static_cast<long long>(tile_m) * 2 + 1) * N + n0 + t2] = rr;
        }
      }
    }
  }
}


// Epilogue kinds of the persistent kernel (compile-time: the run-time flags of EpiParams made
// every element a branch; BERT needs these five)
constexpr int kEkBias = 1, kEkDGelu = 2, kEkBeta = 4, kEkAux = 8, kEkGelu = 16;

// Register epilogue of gemm256p_kernel: acc[ha][hb][a][b][v] = C[m0 + ha*128 + wm*64 + a*16 +
// (lane & 15)][n0 + hb*BNH + wn*WC + b*16 + 4*(lane >> 4) + v]. Lane pairs (g even, g + 1)
// swap halves so each lane stores 16 B (8 columns): 16 rows x 64 contiguous bytes per store.
// CHECK: the tile overhangs M or N (row / column guards per lane).
template <int EK, bool CHECK, int BNH, int WC>
__device__ __forceinline__ void pers_epi(const f32x4_t (&acc)[2][2][4][2], const EpiParams& E, int m0, int n0, int M,
                                         int N, float alpha, int lane, int wm, int wn) {
  const int g = lane >> 4, i16 = lane & 15;
  const bool odd = g & 1;
  bf16_t* const out = static_cast<bf16_t*>(E.out);
  // residual (dGELU) / old-output (beta) loads are software-pipelined one row block ahead: the
  // loads of block it + 1 are in flight while block it is computed and stored (a load-use per
  // block left every block's latency exposed)
  constexpr bool LD = (EK & (kEkDGelu | kEkBeta)) != 0;
  uint2 rvb[2][2][2], ovb[2][2][2];  // [slot][hb][b]
  auto load_blk = [&](int it, uint2 (&rv)[2][2], uint2 (&ov)[2][2]) {
    const int ha = it >> 2, a = it & 3;
    const int m = m0 + ha * 128 + wm * 64 + a * 16 + i16;
    if (CHECK && m >= M) return;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const int nb = n0 + hb * BNH + wn * WC + 4 * g;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if constexpr ((EK & kEkDGelu) != 0)
          if (!CHECK || nb + 16 * b < N)
            rv[hb][b] = *reinterpret_cast<const uint2*>(E.residual + static_cast<long long>(m) * E.ldr + nb + 16 * b);
        if constexpr ((EK & kEkBeta) != 0)
          if (!CHECK || nb + 16 * b < N)
            ov[hb][b] = *reinterpret_cast<const uint2*>(out + static_cast<long long>(m) * E.ldo + nb + 16 * b);
      }
    }
  };
  if constexpr (LD) load_blk(0, rvb[0], ovb[0]);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int ha = it >> 2, a = it & 3;
    if constexpr (LD)
      if (it + 1 < 8) load_blk(it + 1, rvb[(it + 1) & 1], ovb[(it + 1) & 1]);
    {
      const int m = m0 + ha * 128 + wm * 64 + a * 16 + i16;
      if (CHECK && m >= M) continue;
      const long long row = static_cast<long long>(m) * E.ldo;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        const int nb = n0 + hb * BNH + wn * WC + 4 * g;  // block b: nb + 16 b
        const uint2(&rv)[2] = rvb[it & 1][hb];
        const uint2(&ov)[2] = ovb[it & 1][hb];
        uint2 po[2], pa[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          f32x4_t v = acc[ha][hb][a][b] * alpha;
          if constexpr ((EK & kEkBias) != 0)
            if (!CHECK || nb + 16 * b < N) v += *reinterpret_cast<const f32x4_t*>(E.bias + nb + 16 * b);
          if constexpr ((EK & kEkDGelu) != 0) {
            v[0] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv[b].x & 0xffff)));
            v[1] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv[b].x >> 16)));
            v[2] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv[b].y & 0xffff)));
            v[3] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv[b].y >> 16)));
          }
          if constexpr ((EK & kEkBeta) != 0) {
            v[0] += bf2f(static_cast<bf16_t>(ov[b].x & 0xffff));
            v[1] += bf2f(static_cast<bf16_t>(ov[b].x >> 16));
            v[2] += bf2f(static_cast<bf16_t>(ov[b].y & 0xffff));
            v[3] += bf2f(static_cast<bf16_t>(ov[b].y >> 16));
          }
          if constexpr ((EK & kEkAux) != 0) pa[b] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
          if constexpr ((EK & kEkGelu) != 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(v[j]);
          }
          po[b] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
        const int nst = odd ? nb + 12 : nb;  // odd lane: columns 4(g-1).. of block 1
        {
          const uint2 snd = odd ? po[0] : po[1];
          const uint2 rcv = make_uint2(__shfl_xor(snd.x, 16, 64), __shfl_xor(snd.y, 16, 64));
          const uint4 w = odd ? make_uint4(rcv.x, rcv.y, po[1].x, po[1].y) : make_uint4(po[0].x, po[0].y, rcv.x, rcv.y);
          if (!CHECK || nst < N) *reinterpret_cast<uint4*>(out + row + nst) = w;
        }
        if constexpr ((EK & kEkAux) != 0) {
          const uint2 snd = odd ? pa[0] : pa[1];
          const uint2 rcv = make_uint2(__shfl_xor(snd.x, 16, 64), __shfl_xor(snd.y, 16, 64));
          const uint4 w = odd ? make_uint4(rcv.x, rcv.y, pa[1].x, pa[1].y) : make_uint4(pa[0].x, pa[0].y, rcv.x, rcv.y);
          if (!CHECK || nst < N) *reinterpret_cast<uint4*>(E.aux + row + nst) = w;
        }
      }
    }
  }
}

// Persistent 256 x BN GEMM for elementwise epilogues (bias, residual / dGELU, beta, aux copy,
// ReLU / GELU / tanh; no BN statistics, no row remap, no split-K): one workgroup per CU walks
// tiles vt = blockIdx.x, + gridDim.x, ... (the same XCD-aware order as the one-tile kernel).
// When a tile's last K-tile has been consumed, the DMA of the next tile's first two K-tiles is
// issued into the now idle stage buffers and only then does the epilogue run, straight from
// the accumulator registers (8-B stores of 4 consecutive columns per lane; no LDS staging, so
// the stage buffers stay free): the next tile's operand latency hides under this tile's
// epilogue instead of both sitting exposed between two one-tile workgroups (the per-tile
// prologue + epilogue were ~15 % of a K = 1024 BERT GEMM on one workgroup per CU).
// Main loop: the ping-pong schedule of gemm256_kernel (PP = 1), bf16 operands.
template <int BN, class OA, class OB, int EK>
__global__ __launch_bounds__(OA::THREADS, 1) void gemm256p_kernel(typename OA::Params pa, typename OB::Params pb,
                                                                EpiParams E, int M, int N, int K, int tiles_m,
                                                                int tiles_n, int ovl, int fullwait, int* tq) {
  using Gm = Geo<BN>;
  constexpr int T = OA::THREADS, NW = T / 64, WN = NW / 2;
  static_assert(OB::THREADS == T && NW == 8, "8-wave operand policies");
  constexpr int BNH = Gm::BNH, WC = BNH / WN, NB = WC / 16, GA = OA::G, GB = OB::G;
  constexpr bool AK = Traits<OA>::kmaj, BKM = Traits<OB>::kmaj;
  static_assert(NB == 2, "the 16-B store exchange pairs the two 16-column blocks of a wave");
  __shared__ __attribute__((aligned(16))) char smem[2 * Gm::STAGE];
  const int nblk = tiles_m * tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const bool lag = __builtin_amdgcn_readfirstlane(wm) == 1;
  const int ktiles = K / 64;
  constexpr int A0 = 0, A1 = Gm::AH, B0 = 2 * Gm::AH, B1 = 2 * Gm::AH + Gm::BH;
  auto buf = [&](int kt) { return smem + (kt & 1) * Gm::STAGE; };

  OA la;
  OB lb;
  bf16x8_t fa[2][2][4], fb[2][2][NB];
  auto read_a = [&](const char* sA, bf16x8_t (&f)[2][4]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        if constexpr (AK) f[ks][a] = frag_k(sA, wm * 64 + a * 16, ks, lane);
        else f[ks][a] = frag_mn<128>(sA, wm * 64 + a * 16, ks, lane);
      }
  };
  auto read_b = [&](const char* sB, bf16x8_t (&f)[2][NB]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if constexpr (BKM) f[ks][b] = frag_k(sB, wn * WC + b * 16, ks, lane);
        else f[ks][b] = frag_mn<BNH>(sB, wn * WC + b * 16, ks, lane);
      }
  };
  auto mma = [&](const bf16x8_t (&x)[2][4], const bf16x8_t (&y)[2][NB], f32x4_t (&c)[4][NB]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) c[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y[ks][b], x[ks][a], c[a][b], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // first two K-tiles of a tile: all four halves of K-tile 0, then A0 / B0 / B1 of K-tile 1
  // (its A1 is issued in the first phase of the main loop, as in gemm256_kernel)
  auto prologue = [&](int m0, int n0) {
    la.init(pa, m0, tid);
    lb.init(pb, n0, tid);
    char* b0 = buf(0);
    la.template issue<0>(b0 + A0, 0, wave);
    lb.template issue<0>(b0 + B0, 0, wave);
    lb.template issue<1>(b0 + B1, 0, wave);
    la.template issue<1>(b0 + A1, 0, wave);
    if (ktiles > 1) {
      char* b1 = buf(1);
      la.template issue<0>(b1 + A0, 1, wave);
      lb.template issue<0>(b1 + B0, 1, wave);
      lb.template issue<1>(b1 + B1, 1, wave);
    }
  };

  // Tiles: XCD x = blockIdx.x & 7 owns the contiguous tile range of xcd_remap; its G8 = gridDim.x / 8
  // workgroups take tiles idx = blockIdx.x >> 3 first, then idx + G8, ... (static), or — with the
  // tile queue tq (9 ints: one counter per XCD + a finished-workgroup count) — the next unclaimed idx
  // of their XCD's range: a workgroup that only gets a CU late (the BERT weight-gradient side stream
  // holds up to 192 of them for hundreds of us) then takes fewer tiles instead of finishing its
  // static share late and holding the whole launch.
  const int xcd = blockIdx.x & 7, G8 = gridDim.x >> 3;
  const int xq = nblk >> 3, xr = nblk & 7;
  const int xbase = xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq;
  const int xcnt = xq + (xcd < xr ? 1 : 0);
  __shared__ int s_next;
  int idx = blockIdx.x >> 3;
  if (idx >= xcnt) return;  // (never with a tile queue: the host launches it only for tiles > 8 G8)
  int t = xbase + idx;
  prologue((t / tiles_n) * BM, (t % tiles_n) * BN);
  const float alpha_e = epi_alpha(E);
  // store instructions per thread of a whole-tile (unchecked) epilogue: 8 row blocks x 2 column
  // halves, twice with the aux copy
  constexpr int EPI_ST = 16 * (((EK & kEkAux) != 0) ? 2 : 1);
  // how the previous tile ended: 0 = nothing issued after this tile's prologue DMA (first tile,
  // or no overlap), 1 = a whole-tile epilogue's EPI_ST stores issued after it, 2 = a checked
  // (edge) epilogue, whose store count is data-dependent
  int prev = 0;

  for (;;) {
    const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
    // claim the next tile now: the atomic's round trip hides under this tile's main loop
    int claim = 0;
    if (tq && tid == 0) claim = atomicAdd(tq + xcd, 1);
    f32x4_t acc[2][2][4][NB];
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < NB; ++b) acc[ha][hb][a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // K-tile 0 landed. vmcnt retires in issue order: prologue (K-tile 0: 2 GA + 2 GB
    // instructions, K-tile 1: GA + 2 GB), then the previous tile's epilogue stores; the count
    // leaves K-tile 1 and those stores in flight (a wait for every store of the previous
    // epilogue left 128 KB of stores per CU exposed between two tiles: ~6 us per tile at a
    // K = 1024 BERT GEMM's ~14 us of MFMA work). Edge epilogues issue a data-dependent number
    // of stores: wait for all.
    if (prev == 2) wait_vm<0>();
    else if (ktiles > 1) {
      if (prev == 1) wait_vm<GA + 2 * GB + EPI_ST>();
      else wait_vm<GA + 2 * GB>();
    } else {
      if (prev == 1) wait_vm<EPI_ST>();
      else wait_vm<0>();
    }
    barrier();
    if (lag) barrier();
    for (int kt = 0; kt < ktiles; ++kt) {
      const bool has1 = kt + 1 < ktiles, has2 = kt + 2 < ktiles;
      char* cb = buf(kt);
      read_a(cb + A0, fa[0]);
      read_b(cb + B0, fb[0]);
      if (has1) la.template issue<1>(buf(kt + 1) + A1, kt + 1, wave);
      barrier();
      mma(fa[0], fb[0], acc[0][0]);
      barrier();
      read_b(cb + B1, fb[1]);
      barrier();
      mma(fa[0], fb[1], acc[0][1]);
      barrier();
      read_a(cb + A1, fa[1]);
      if (has2) {
        la.template issue<0>(cb + A0, kt + 2, wave);
        lb.template issue<0>(cb + B0, kt + 2, wave);
      }
      barrier();
      mma(fa[1], fb[1], acc[1][1]);
      barrier();
      if (has1) {
        if (has2) wait_vm<GA + GB>(); else wait_vm<0>();
      }
      if (has2) lb.template issue<1>(cb + B1, kt + 2, wave);
      barrier();
      mma(fa[1], fb[0], acc[1][0]);
      barrier();
    }
    if (tq) {
      if (tid == 0) s_next = claim;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (!lag) barrier();  // both wave halves past their last LDS read: the stage buffers are free
    const int nidx = tq ? G8 + __builtin_amdgcn_readfirstlane(s_next) : idx + G8;
    const bool more = nidx < xcnt;
    if (ovl && more) {
      t = xbase + nidx;
      prologue((t / tiles_n) * BM, (t % tiles_n) * BN);
    }
    // ------------------------------------------------------------ register epilogue
    const bool whole = m0 + BM <= M && n0 + BN <= N;
    if (whole) pers_epi<EK, false, BNH, WC>(acc, E, m0, n0, M, N, alpha_e, lane, wm, wn);
    else pers_epi<EK, true, BNH, WC>(acc, E, m0, n0, M, N, alpha_e, lane, wm, wn);
    if (!more) break;
    prev = !ovl ? 0 : (whole && !fullwait ? 1 : 2);
    if (!ovl) {
      t = xbase + nidx;
      prologue((t / tiles_n) * BM, (t % tiles_n) * BN);
    }
    idx = nidx;
  }
  if (tq && tid == 0) {
    // every workgroup's last claim (the one past its XCD's range) precedes its arrival here, so
    // the last to arrive can reset the queue for the next launch (graph replays included)
    if (atomicAdd(tq + 8, 1) == static_cast<int>(gridDim.x) - 1) {
#pragma unroll
      for (int i = 0; i < 9; ++i) tq[i] = 0;
    }
  }
}

// Per-stream arrival counters of the in-kernel split-K fold (EpiParams mode 3): zeroed once at
// allocation, every launch leaves them zero again (the last workgroup of a tile resets its
// counter). Allocated on first use (an eager warm-up step precedes any hipGraph capture).
// Returns nullptr when more than kMaxCtr tiles are asked for (the caller keeps the fold kernel).
constexpr int kMaxCtr = 1 << 16;
inline int* tile_counters(hipStream_t st, int tiles) {
  if (tiles > kMaxCtr - 16) return nullptr;  // (the last 16 ints: the persistent GEMM's tile queue)
  struct Buf {
    hipStream_t st;
    int* p;
  };
  static Buf bufs[16] = {};
  for (auto& b : bufs)
    if (b.p && b.st == st) return b.p;
  for (auto& b : bufs) {
    if (!b.p) {
      if (hipMalloc(&b.p, kMaxCtr * sizeof(int)) != hipSuccess) return b.p = nullptr, nullptr;
      if (hipMemsetAsync(b.p, 0, kMaxCtr * sizeof(int), st) != hipSuccess) return nullptr;
      b.st = st;
      return b.p;
    }
  }
  return nullptr;
}

// In-kernel split-K fold (TTD_SPLITK_FOLD_INKERNEL=1; off by default). Measured slower in both
// steps (ResNet-50 b1024 73.0 -> 82.7 ms, BERT-Large b128 187.1 -> 195.8 ms): the device-scope
// release of every split writes back its XCD's whole L2 (cross-XCD visibility of the slab),
// which the concurrent main-chain kernels pay for, and a tile's last split sums up to
// hundreds of slabs alone (ResNet's few-tile weight gradients) where the fold pass spreads
// that work over the chip.
inline bool inkernel_fold() { return ::ttdk_rt::fold_flag() != 0; }

inline int device_cus_total() {
  static int cus = [] {
    int dev = 0, n = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}

// CUs a persistent one-workgroup-per-CU grid may assume it owns: all of them, minus the CTA
// budget of the collective engine while this process runs data-parallel (ttdk_set_reserved_cus,
// set by parallel/rccl.py to RCCL's maxCTAs). A persistent grid statically partitions its work,
// so a workgroup that waits for a CU an all-reduce CTA holds delays the whole launch by a full
// share; sized to the free CUs it never waits (the reserved CUs idle, or take side-stream work,
// when no bucket is in flight).
inline int device_cus() {
  const int total = device_cus_total();
  const int r = ::ttdk_rt::reserved_cus();
  return (r > 0 && total - r >= total / 2) ? total - r : total;
}

template <int BN, class OA, class OB, int F8 = 0, int PP = 0>
hipError_t launch(const typename OA::Params& pa, const typename OB::Params& pb, const EpiParams& pe, int M, int N,
                  int K, int splits, hipStream_t st) {
  const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
  const int ktiles = K / (F8 ? 128 : 64);
  // (Wave quantisation — a launch of R full rounds plus a thin last round on one workgroup per
  // CU — is left to the side stream's weight gradients, which fill the idle CUs of the thin
  // round. A split-K tail for these launches was tried in rounds 1-2: 5-7 % faster standalone,
  // slower inside the two-stream step, and its b1024 data gradients disagreed with the plain
  // kernel far beyond rounding (profiles/r3_tail_split_check.json: gradient cosine 0.81), so it is gone.)
  const int cus = device_cus();
  const int tiles = tm * tn;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  if constexpr (F8 == 0 && PP == 1 && OA::THREADS == THR && BN == 256) {
    // elementwise-only epilogue on more than one round of tiles: persistent kernel, the next
    // tile's operand DMA in flight under this tile's register epilogue
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    int ek = -1;
    if (pe.act == kActNone && !pe.residual) ek = 0;
    else if (pe.act == kActGelu && !pe.residual) ek = kEkGelu;
    else if (pe.act == kActDGelu && pe.residual) ek = kEkDGelu;
    if (ek >= 0) {
      if (pe.bias) ek |= kEkBias;
      if (pe.beta) ek |= kEkBeta;
      if (pe.aux) ek |= kEkAux;
    }
    if (::ttdk_rt::pers_flag() && splits == 1 && pe.mode == 0 && !pe.remap && !pe.stat && !pe.by && !pe.bH && tiles > cus &&
        N % 8 == 0 && pe.ldo % 8 == 0 && (!pe.residual || pe.ldr % 4 == 0) && (!pe.bias || al16(pe.bias)) &&
        al16(pe.out) && (!pe.aux || al16(pe.aux)) && (!pe.residual || (reinterpret_cast<uintptr_t>(pe.residual) & 7) == 0)) {
      const int ovl = ::ttdk_rt::pers_flag() == 1;
      // TTD_PERS_STORE_WAIT=1: wait for every store of the previous epilogue (A/B)
      static const int fullwait = getenv_int("TTD_PERS_STORE_WAIT", 0);
      // per-XCD tile queue (TTD_PERS_QUEUE, default 1): the stream's counter buffer, last 16 ints
      static const int queue = getenv_int("TTD_PERS_QUEUE", 1);
      int* tq = nullptr;
      if (queue && cus % 8 == 0) {
        int* c = tile_counters(st, 0);
        if (c) tq = c + kMaxCtr - 16;
      }
#define TTDK_PERS(EKV)                                                                                                \
  case EKV:                                                                                                           \
    hipLaunchKernelGGL((gemm256p_kernel<BN, OA, OB, EKV>), dim3(cus), dim3(THR), 0, st, pa, pb, pe, M, N, K, tm, tn, ovl, \
                       fullwait, tq);                                                                                 \
    return hipGetLastError();
      switch (ek) {
        TTDK_PERS(0)
        TTDK_PERS(kEkBias)
        TTDK_PERS(kEkBias | kEkAux | kEkGelu)
        TTDK_PERS(kEkDGelu)
        TTDK_PERS(kEkBeta)
        default: break;
      }
#undef TTDK_PERS
    }
  }
  hipLaunchKernelGGL((gemm256_kernel<BN, OA, OB, F8, PP>), dim3(tm * tn, splits), dim3(OA::THREADS), 0, st, pa, pb, pe, M, N,
                     K, tm, tn, per, 0);
  return hipGetLastError();
}

// dense GEMM entry: A (M rows) and B (N rows), each K-major or MN-major, bf16. Long-K 256-wide
// tiles take the ping-pong schedule (BERT-Large shapes +2-5 % standalone, +1.3 % per step);
// short K keeps the two-barrier schedule (ping-pong everywhere cost ResNet-50 2 %).
template <int BN, int PP>
hipError_t dense_pp(const bf16_t* A, long long lda, bool ak, const bf16_t* B, long long ldb, bool bk,
                    const EpiParams& pe, int M, int N, int K, int splits, hipStream_t st) {
  DenseP pa{A, lda, M}, pb{B, ldb, N};
  constexpr int BH = BN / 2;
  if (ak && bk) return launch<BN, OpDenseK<128, 2>, OpDenseK<BH, 2>, 0, PP>(pa, pb, pe, M, N, K, splits, st);
  if (ak) return launch<BN, OpDenseKU<128, 2>, OpDenseMN<BH>, 0, PP>(pa, pb, pe, M, N, K, splits, st);
  if (bk) return launch<BN, OpDenseMN<128>, OpDenseKU<BH, 2>, 0, PP>(pa, pb, pe, M, N, K, splits, st);
  return launch<BN, OpDenseMN<128>, OpDenseMN<BH>, 0, PP>(pa, pb, pe, M, N, K, splits, st);
}

// Weight gradient with the A operand's row sums (EpiParams::rsum: a bias gradient): MN-major A
// and B, 256-wide tiles, ping-pong schedule, fp32 slab (split-K) or store epilogue.
inline hipError_t dense_rowsum(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, const EpiParams& pe,
                               int M, int N, int K, int splits, hipStream_t st) {
  DenseP pa{A, lda, M}, pb{B, ldb, N};
  const int tm = ceil_div(M, BM), tn = ceil_div(N, 256);
  const int ktiles = K / 64;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  hipLaunchKernelGGL((gemm256_kernel<256, OpDenseMN<128>, OpDenseMN<128>, 0, 1, 1>), dim3(tm * tn, splits), dim3(THR), 0,
                     st, pa, pb, pe, M, N, K, tm, tn, per, 0);
  return hipGetLastError();
}

template <int BN>
hipError_t dense(const bf16_t* A, long long lda, bool ak, const bf16_t* B, long long ldb, bool bk,
                 const EpiParams& pe, int M, int N, int K, int splits, hipStream_t st) {
  if constexpr (BN == 256) {
    static const int pp_on = getenv_int("TTD_BIG_PP", 1);
    const int kts = K / 64 / (splits > 1 ? splits : 1);  // K-tiles per workgroup
    if (kts >= 16 && pp_on)
      return dense_pp<BN, 1>(A, lda, ak, B, ldb, bk, pe, M, N, K, splits, st);
  }
  return dense_pp<BN, 0>(A, lda, ak, B, ldb, bk, pe, M, N, K, splits, st);
}

}  // namespace big

// ------------------------------------------------------------------ host-side dispatch
template <int BM, int BN, class LA, class LB>
hipError_t launch(const typename LA::Params& pa, const typename LB::Params& pb, const EpiParams& pe, int M, int N,
                  int K, int splits, hipStream_t st) {
  const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
  const int ktiles = ceil_div(K, BK);
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = ceil_div(ktiles, splits);
  splits = ceil_div(ktiles, per);
  dim3 grid(tm * tn, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB>), grid, dim3(NTHR), 0, st, pa, pb, pe, M, N, K, tm, tn, per);
  return hipGetLastError();
}

template <int BM, int BN, class LA, class LB>
hipError_t launch_batched(const typename LA::Params& pa, const typename LB::Params& pb, const EpiParams& pe, int M,
                          int N, int K, int batch, long long sa, long long sb, long long so, hipStream_t st) {
  const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
  const int ktiles = ceil_div(K, BK);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB>), dim3(tm * tn, 1, batch), dim3(NTHR), 0, st, pa, pb, pe, M, N, K, tm,
                     tn, ktiles, sa, sb, so);
  return hipGetLastError();
}

// Tile choice: prefer 128x128; shrink a dimension when it is small.
// Tile width of the 256-row LDS-DMA kernel for an M x N x K GEMM, or 0 when the 4-wave
// kernel is the better fit (small tiles / small GEMMs). Mirrored by ops/gemm.py big_bn().
inline int big_bn(int M, int N, int K) {
  if (M < 256 || N < 128 || K % 64 || N % 8 || static_cast<long long>(M) * N < (1LL << 20)) return 0;
  return N >= 256 ? 256 : 128;
}
inline bool big_fits(int M, int N, int K) { return big_bn(M, N, K) != 0; }
// Weight gradients have a long K (pixels) and split-K fills the machine, so only the tile
// shape (not M*N) decides.
inline int big_bn_wgrad(int M, int N, int K) {
  if (M < 256 || N < 128 || K % 64 || N % 8) return 0;
  return N >= 256 ? 256 : 128;
}

inline void pick_tile(int M, int N, int* bm, int* bn) {
  *bm = (M <= 64) ? 64 : 128;
  *bn = (N <= 64) ? 64 : 128;
}

template <template <int> class LA_T, template <int> class LB_T>
hipError_t dispatch(const void* pa_raw, const void* pb_raw, const EpiParams& pe, int M, int N, int K, int splits,
                    int bm, int bn, hipStream_t st) {
#define TTDK_CASE(BM_, BN_)                                                                                        \
  if (bm == BM_ && bn == BN_)                                                                                      \
    return launch<BM_, BN_, LA_T<BM_>, LB_T<BN_>>(*static_cast<const typename LA_T<BM_>::Params*>(pa_raw),         \
                                                  *static_cast<const typename LB_T<BN_>::Params*>(pb_raw), pe, M, N, \
                                                  K, splits, st);
  TTDK_CASE(128, 128)
  TTDK_CASE(128, 64)
  TTDK_CASE(64, 128)
  TTDK_CASE(64, 64)
#undef TTDK_CASE
  return hipErrorInvalidValue;
}

template <int R>
using KDenseS = KDense<R, false>;
template <int R>
using MNDenseS = MNDense<R, false>;
template <int R>
using KConvFwd = KConvGather<R, false>;
template <int R>
using KConvDgrad = KConvGather<R, true>;

}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Epilogue descriptor passed from Python (ctypes Structure with identical layout).
struct TtdkEpilogue {
  int mode;
  void* out;
  long long ldo;
  long long slab_stride;
  const float* bias;
  const bf16_t* residual;
  long long ldr;
  int act;
  int beta;
  int remap;
  int rP, rQ, rOH, rOW, rs;
  float* stat;
  float alpha;
  bf16_t* aux;  // optional second bf16 output: the pre-activation value (same layout as out)
  const float* ascale0;  // optional device scalars multiplied into alpha (fp8 dequant scales)
  const float* ascale1;
  const bf16_t* by;      // optional BN-backward statistics source (see EpiParams::by)
  const uint8_t* bmask;
  const bf16_t* by2;     // optional second statistics source (EpiParams::by2 / stat2)
  float* stat2;
  int bH, bW;            // EpiParams::bH/bW (stride-2-sampled beta)
};

inline EpiParams to_epi(const TtdkEpilogue* e) {
  EpiParams p;
  static const int feed_pf = [] { const char* v = getenv("TTD_FEED_PREFETCH"); return v ? atoi(v) : 1; }();
  p.feed_pf = feed_pf;
  p.mode = e->mode;
  p.out = e->out;
  p.ldo = e->ldo;
  p.slab_stride = e->slab_stride;
  p.bias = e->bias;
  p.residual = e->residual;
  p.ldr = e->ldr;
  p.act = e->act;
  p.beta = e->beta;
  p.remap = e->remap;
  p.rP = e->rP;
  p.rQ = e->rQ;
  p.rOH = e->rOH;
  p.rOW = e->rOW;
  p.rs = e->rs;
  p.stat = e->stat;
  p.alpha = e->alpha == 0.f ? 1.f : e->alpha;
  p.aux = e->aux;
  p.ascale0 = e->ascale0;
  p.ascale1 = e->ascale1;
  p.by = e->by;
  p.bmask = e->bmask;
  p.by2 = e->by2;
  p.stat2 = e->stat2;
  p.bH = e->bH;
  p.bW = e->bW;
  p.py = nullptr;
  p.pcoef = nullptr;
  p.pdz = nullptr;
  p.pmask = nullptr;
  p.pld = 0;
  p.kout = nullptr;
  p.kctr = nullptr;
  p.rsum = nullptr;
  return p;
}

struct TtdkConv {
  int N, H, W, C;   // input NHWC
  int K, R, S;      // filters [K][R][S][C]
  int P, Q;         // output spatial
  int sh, sw, ph, pw, dh, dw;
};

inline bool is_pointwise(const TtdkConv* g) {
  return g->R == 1 && g->S == 1 && g->sh == 1 && g->sw == 1 && g->ph == 0 && g->pw == 0;
}

// y[N,P,Q,K] = conv(x[N,H,W,C], w[K,R,S,C]).
inline big::ConvP conv_params(const void* src, int Hs, int Ws, int Cs, int P, int Q, const TtdkConv* g, int rows) {
  return big::ConvP{src, Hs, Ws, Cs, P, Q, g->R, g->S, g->sh, g->sw, g->ph, g->pw, g->dh, g->dw, rows};
}

