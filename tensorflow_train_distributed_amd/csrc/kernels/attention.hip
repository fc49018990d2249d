// Fused multi-head attention (flash-style) forward and backward for head_dim 64 on gfx950
// MFMA (v_mfma_f32_16x16x32_bf16): BERT-Large self-attention (SURVEY.md §2.6 [NS] BERT
// kernels; BASELINE.json config 4). The S x S score matrix is never materialised.
//
// Layout: token-major activations straight out of / into the fused QKV projection GEMM:
//   element (b, s, h, d) of Q/K/V/O/dQ/dK/dV at base + (b*S + s)*ld + h*64 + d
// so no transposes surround the kernels. Per (batch, head) softmax statistics lse2 / delta
// are fp32 [B*H][S]. Scores live in the log2 domain: s2 = (q.k) * log2(e)/sqrt(64),
// P = exp2(s2 - lse2).
//
// Options: per-batch key lengths (keys >= len masked), and attention-probability dropout
// whose keep mask is a counter hash of (seed, step, site, (b*H+h, q, key)) — regenerated
// identically in both backward kernels, never stored.
//
// Kernels (4 waves / workgroup, XCD-aware block order so the Q-blocks of one head share an
// L2):
//   fwd     : 128 query rows per workgroup (32 per wave); K/V tiles of 64 keys double-buffered
//             in LDS (register-staged prefetch); online softmax in registers; the swapped QK^T
//             puts 4 keys x 1 query in each lane, so P feeds the PV MFMA without any shuffle.
//   bwd_kv  : 128 keys per workgroup; loops over 64-query tiles of Q/dO (one LDS image read
//             by rows for S, dP and by columns (ds_read_b64_tr_b16) for dV^T, dK^T); dK, dV
//             accumulate in registers — no cross-workgroup sums.
//   bwd_q   : 128 queries per workgroup; first delta = rowsum(dO * O) of its query rows (the
//             dO fragments are already in registers; O is read once, here) — stored for
//             bwd_kv, which runs after it; then recomputes S, dP per key tile; dQ in registers
//             (deterministic, no float atomics). (A separate delta pass re-read O and dO:
//             227 us per BERT-Large b128 layer, 5.5 ms per step.)
//   bwd_fused (opt-in): all of dQ, dK, dV of one (batch, head) in one workgroup — five MFMA
//             products instead of seven, one dropout hash per element instead of two; slower
//             at BERT-Large's S = 512 (occupancy: see ttdk_attn_set_fused_bwd).
#include "tile_common.h"

#include <type_traits>

namespace ttdk {
namespace {

using tile::mfma;
using tile::off64;
using tile::pack_frag;
using tile::rd_col;
using tile::rd_row;

constexpr int D = 64;
constexpr int KT = 64;    // keys (fwd/bwd_q) or queries (bwd_kv) per streamed tile
constexpr int QBLK = 128; // rows per workgroup
constexpr int TILE_BYTES = KT * D * 2;

struct AttnParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  const bf16_t* o;
  const bf16_t* dout;
  long long ldq, ldk, ldv, ldo, lddo;
  bf16_t* out;   // fwd: O ; bwd_q: dQ ; bwd_kv: dK
  bf16_t* out2;  // bwd_kv: dV ; fused bwd: dK
  bf16_t* out3;  // fused bwd: dV
  long long ld_out, ld_out2, ld_out3;
  float* lse;          // [B*H][S] log2 domain
  float* delta;        // [B*H][S]: written by bwd_q, read by bwd_kv
  const int* seqlen;   // [B] or null
  int B, H, S;
  float scale_log2;    // log2(e) / sqrt(D)
  float scale;         // 1 / sqrt(D)
  uint32_t drop_thr;
  float drop_scale;    // 1 / (1 - p)
  const long long* rng;
  uint32_t site;
};

__device__ __forceinline__ uint4 ldg16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ bf16x8_t ldg_frag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}

// 64 rows x 64 cols tile loader: thread t moves rows (t >> 3) and (t >> 3) + 32, chunk t & 7.
// The lane's row / chunk offset is folded into its pointer once; per tile only the block-uniform
// row0 * ld is formed (scalar), not a 64-bit vector multiply per row (v_mul_lo_u32 is a
// quarter-rate instruction in these VALU-bound loops).
struct TileLoader {
  const bf16_t* lanep;
  long long ld;
  int r, c;
  uint4 v[2];
  __device__ __forceinline__ void init(const bf16_t* b, long long l, int tid) {
    ld = l;
    r = tid >> 3;
    c = tid & 7;
    lanep = b + static_cast<long long>(r) * l + c * 8;
  }
  __device__ __forceinline__ void load(int row0, int nrows) {
    const bf16_t* p = lanep + static_cast<long long>(row0) * ld;
    if (row0 + 64 <= nrows) {  // block-uniform: whole tile in range, no per-dword selects
#pragma unroll
      for (int j = 0; j < 2; ++j) v[j] = ldg16(p + 32 * j * ld);
      return;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = row0 + r + 32 * j;
      v[j] = row < nrows ? ldg16(p + 32 * j * ld) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
    for (int j = 0; j < 2; ++j) *reinterpret_cast<uint4*>(lds + off64(r + 32 * j, c * 8)) = v[j];
  }
};

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ------------------------------------------------------------------------------ forward
// (launch_bounds(256, 4) — 128 VGPRs, 4 waves / SIMD instead of 3, 10-12 spilled — measured
// 10-18 % slower at BERT-Large b128: the spills land in the loop)
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnParams P) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];
  const int qblocks = P.S / QBLK;
  const int t = tile::xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / qblocks, qblk = t - bh * qblocks;
  const int b = bh / P.H, h = bh - b * P.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int q0 = qblk * QBLK + wave * 32;
  const int len = P.seqlen ? min(P.seqlen[b], P.S) : P.S;
  const long long tok0 = static_cast<long long>(b) * P.S;

  bf16x8_t qf[2][2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qb][ks] = ldg_frag(P.q + (tok0 + q0 + qb * 16 + i16) * P.ldq + h * D + ks * 32 + g * 8);

  TileLoader lk, lv;
  lk.init(P.k + tok0 * P.ldk + h * D, P.ldk, tid);
  lv.init(P.v + tok0 * P.ldv + h * D, P.ldv, tid);

  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  f32x4_t o[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int db = 0; db < 4; ++db) o[qb][db] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const uint32_t key = DROP ? drop_key(P.rng, P.site) : 0u;
  const int ntiles = (len + KT - 1) / KT;
  if (ntiles > 0) {
    lk.load(0, len);
    lv.load(0, len);
    lk.store(smem);
    lv.store(smem + TILE_BYTES);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ntiles; ++kt) {
    const bool nxt = kt + 1 < ntiles;
    if (nxt) {
      lk.load((kt + 1) * KT, len);
      lv.load((kt + 1) * KT, len);
    }
    const char* sK = smem + cur * 2 * TILE_BYTES;
    const char* sV = sK + TILE_BYTES;
    // ---- S^T tile: lane holds keys kb*16 + 4g + i for query qb*16 + i16
    f32x4_t s[2][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const bf16x8_t k0 = rd_row(sK, kb * 16 + i16, g);
      const bf16x8_t k1 = rd_row(sK, kb * 16 + i16, 4 + g);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        s[qb][kb] = mfma(k0, qf[qb][0], f32x4_t{0.f, 0.f, 0.f, 0.f});
        s[qb][kb] = mfma(k1, qf[qb][1], s[qb][kb]);
      }
    }
    const int kbase = kt * KT;
    if (kbase + KT > len) {
      // (block-uniform: only the last key tile of a padded sequence; the full tiles run no
      // per-element compare / select — the kernel is VALU-bound, profiles/r3_bert_*_pmc_*)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (kbase + kb * 16 + 4 * g + i >= len) s[qb][kb][i] = -INFINITY;
    }
    bf16x8_t pf[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      // max over the raw scores (scale > 0 commutes with max); the scale rides in the exp2 FMA
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[qb][kb][i]);
      mx = tile::rows4_max(mx);
      // lazy rescale: the running max moves (and O, l are rescaled) only when some row of the
      // wave saw its max grow by more than 8 (log2 units) — otherwise P = exp2(s - m) stays
      // below 2^8 (exact in fp32, in range for the bf16 P operand) and the 16 O multiplies and
      // the alpha exp2 of the tile are skipped (wave-uniform branch; lse = m + log2 l either way)
      const float mxs = mx * P.scale_log2;
      float alpha = 1.f;
      const bool grow = mxs > m[qb] + 8.f;
      if (__builtin_amdgcn_ballot_w64(grow) != 0) {
        const float mnew = fmaxf(m[qb], mxs);
        alpha = fast_exp2(m[qb] - (mnew == -INFINITY ? 0.f : mnew));
        m[qb] = mnew;
#pragma unroll
        for (int db = 0; db < 4; ++db) o[qb][db] *= alpha;
      }
      const float msub = m[qb] == -INFINITY ? 0.f : m[qb];
      float rs = 0.f;
      const int qrow = q0 + qb * 16 + i16;
      // keys kbase + kb*16 + 4g + i: pair kbase/2 + (kb >> 1)*16 + 4g + i, half kb & 1 — the
      // hash input is a per-tile base plus constants
      uint32_t hp[2][4] = {};
      if constexpr (DROP) {
        const uint32_t hbase = attn_row_term(static_cast<uint32_t>(bh * P.S + qrow)) +
                               (static_cast<uint32_t>(kbase >> 1) + 4u * g) * kAttnPairMul;
#pragma unroll
        for (int kp = 0; kp < 2; ++kp)
#pragma unroll
          for (int i = 0; i < 4; ++i) hp[kp][i] = attn_hash_input(key, hbase + (16u * kp + i) * kAttnPairMul);
      }
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = fast_exp2(__builtin_fmaf(s[qb][kb][i], P.scale_log2, -msub));
          rs += p;
          float pd = p;
          if constexpr (DROP) pd = attn_keep_half(hp[kb >> 1][i], kb & 1, P.drop_thr) ? p : 0.f;
          s[qb][kb][i] = pd;
        }
      }
      rs = tile::rows4_sum(rs);
      l[qb] = l[qb] * alpha + rs;
      pf[qb][0] = pack_frag(s[qb][0], s[qb][1]);
      pf[qb][1] = pack_frag(s[qb][2], s[qb][3]);
    }
    // ---- O += P V
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8_t vf = rd_col(sV, ks * 32, ks * 32 + 16, db * 16, lane);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) o[qb][db] = mfma(vf, pf[qb][ks], o[qb][db]);
      }
    if (nxt) {
      lk.store(smem + (cur ^ 1) * 2 * TILE_BYTES);
      lv.store(smem + (cur ^ 1) * 2 * TILE_BYTES + TILE_BYTES);
    }
    __syncthreads();
    cur ^= 1;
  }
  // ---- normalise, store O (bf16) and lse2
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qrow = q0 + qb * 16 + i16;
    const float inv = l[qb] > 0.f ? (DROP ? P.drop_scale : 1.f) / l[qb] : 0.f;
    bf16_t* op = P.out + (tok0 + qrow) * P.ld_out + h * D + 4 * g;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4_t v = o[qb][db] * inv;
      uint2 w;
      w.x = pack_bf16x2(v[0], v[1]);
      w.y = pack_bf16x2(v[2], v[3]);
      *reinterpret_cast<uint2*>(op + db * 16) = w;
    }
    if (g == 0 && P.lse)
      P.lse[static_cast<long long>(bh) * P.S + qrow] = l[qb] > 0.f ? m[qb] + __log2f(l[qb]) : -INFINITY;
  }
}

// ------------------------------------------------------------------------------ bwd dK, dV
// Per 64-query tile, four phases that each put one wave's MFMA work beside independent VALU
// work of the same wave (sched_barrier-separated, so the scheduler interleaves within a phase):
// S/dP of query rows 0-31 | S/dP of rows 32-63 + P/dS of rows 0-31 | dV/dK over rows 0-31 + P/dS
// of rows 32-63 | dV/dK over rows 32-63. The previous loop ran all of S/dP, then all P/dS, then
// all dV/dK per wave: 20 % MFMA busy, 50 % of wave cycles waiting at BERT-Large b128
// (profiles/r5_attn_bwd_pmc_before.txt). Two LDS buffers with compile-time offsets (the loop
// handles two tiles per trip), register-staged global loads one tile ahead, one barrier per tile.
// MODE (diagnostics, TTD_ATTN_KV_DIAG; 0 in production): bit 0 skips the elementwise P / dS,
// bit 1 the per-tile Q / dO reloads, bit 2 the per-tile barrier (only with bit 1) — wrong
// results, for attributing the kernel's time; bit 3 writes per-workgroup clock stamps (entry,
// prologue done, loop done, exit as s_memtime; entry / exit as s_memrealtime) over dV as
// int64[grid][8] instead of dV (tools/attn_kv_stamps.py).
template <bool DROP, int MODE = 0>
__global__ __launch_bounds__(256, 2) void attn_bwd_kv_kernel(AttnParams P) {
  constexpr int BUF = 2 * TILE_BYTES + 2 * KT * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int kblocks = P.S / QBLK;
  const int t = tile::xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / kblocks, kblk = t - bh * kblocks;
  const int b = bh / P.H, h = bh - b * P.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int k0 = kblk * QBLK + wave * 32;
  const int len = P.seqlen ? min(P.seqlen[b], P.S) : P.S;
  const long long tok0 = static_cast<long long>(b) * P.S;
  long long stamp[6] = {};
  if constexpr ((MODE & 8) != 0) {
    stamp[0] = __builtin_amdgcn_s_memtime();
    stamp[4] = __builtin_amdgcn_s_memrealtime();
  }

  f32x4_t dk[2][4], dv[2][4];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int db = 0; db < 4; ++db) dk[kb][db] = dv[kb][db] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const bool any = kblk * QBLK < len;  // block-uniform: some key of this block is valid
  if (any) {
    bf16x8_t kf[2][2], vf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const long long row = tok0 + k0 + kb * 16 + i16;
        kf[kb][ks] = ldg_frag(P.k + row * P.ldk + h * D + ks * 32 + g * 8);
        vf[kb][ks] = ldg_frag(P.v + row * P.ldv + h * D + ks * 32 + g * 8);
      }
    TileLoader lq, ld;
    lq.init(P.q + tok0 * P.ldq + h * D, P.ldq, tid);
    ld.init(P.dout + tok0 * P.lddo + h * D, P.lddo, tid);
    // per-tile statistics, staged with the dropout scale folded in: lse2 - log2(1/(1-p)) (exp2
    // then gives P / (1-p), a kept probability's value) and delta * (1-p) (the product P * delta
    // unchanged). Thread t < 64 moves lse of query t, 64 <= t < 128 delta of query t - 64.
    const float* st_src = (tid < KT ? P.lse : P.delta) + static_cast<long long>(bh) * P.S + (tid & (KT - 1));
    const float st_add = tid < KT && DROP ? -__builtin_amdgcn_logf(P.drop_scale) : 0.f;
    const float st_mul = tid >= KT && DROP ? 1.f / P.drop_scale : 1.f;
    float stv = 0.f;
    const uint32_t key = DROP ? drop_key(P.rng, P.site) : 0u;
    const int ntiles = P.S / KT;  // even: S is a multiple of QBLK = 2 * KT

    auto load = [&](int qt) {
      lq.load(qt * KT, P.S);
      ld.load(qt * KT, P.S);
      if (tid < 2 * KT) stv = st_src[qt * KT];
    };
    auto store = [&](char* nb) {
      lq.store(nb);
      ld.store(nb + TILE_BYTES);
      if (tid < 2 * KT) reinterpret_cast<float*>(nb + 2 * TILE_BYTES)[tid] = (stv + st_add) * st_mul;
    };
    // S[q][key] and dP[q][key] for the query rows of half hq (qb = 2 hq, 2 hq + 1) of the tile
    // image sQ: lane holds q = qb*16 + 4g + i, key = kb*16 + i16
    auto sdp = [&](const char* sQ, int hq, f32x4_t (&sc)[4][2], f32x4_t (&dp)[4][2]) {
      const char* sD = sQ + TILE_BYTES;
#pragma unroll
      for (int qb = 2 * hq; qb < 2 * hq + 2; ++qb) {
        const bf16x8_t q0f = rd_row(sQ, qb * 16 + i16, g), q1f = rd_row(sQ, qb * 16 + i16, 4 + g);
        const bf16x8_t d0f = rd_row(sD, qb * 16 + i16, g), d1f = rd_row(sD, qb * 16 + i16, 4 + g);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          sc[qb][kb] = mfma(q0f, kf[kb][0], f32x4_t{0.f, 0.f, 0.f, 0.f});
          sc[qb][kb] = mfma(q1f, kf[kb][1], sc[qb][kb]);
          dp[qb][kb] = mfma(d0f, vf[kb][0], f32x4_t{0.f, 0.f, 0.f, 0.f});
          dp[qb][kb] = mfma(d1f, vf[kb][1], dp[qb][kb]);
        }
      }
    };
    // P_d and dS in place for half hq (sc <- P_d = P * keep / (1-p); dp <- dS = P * (keep * dP /
    // (1-p) - delta) = P_d * dP - (P / (1-p)) * (delta * (1-p))): exp2, and per element one keep
    // test, one select, one multiply and one FMA. Keys >= len are not masked here: a key's P and
    // dS feed only its own dK / dV rows (the key is the MFMA column), which are zeroed at the
    // store. Dropout: keys k0 + i16 and k0 + 16 + i16 (kb = 0, 1) are the halves of pair
    // k0/2 + i16 — one hash per query row, no lane exchange.
    auto hashes = [&](uint32_t hrow, int hq, uint32_t (&hh)[2][4]) {
      if constexpr (DROP)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            hh[u][i] = attn_hash_input(key, hrow + static_cast<uint32_t>((2 * hq + u) * 16 + i) * 0x9E3779B1u);
    };
    auto pds = [&](const float* sL, const uint32_t (&hq_hash)[2][4], int hq, f32x4_t (&sc)[4][2], f32x4_t (&dp)[4][2]) {
      const float* sDel = sL + KT;
#pragma unroll
      for (int qb = 2 * hq; qb < 2 * hq + 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ql = qb * 16 + 4 * g + i;
          const float lse2 = sL[ql], del = sDel[ql];
          const uint32_t hh = hq_hash[qb - 2 * hq][i];
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            const float p = fast_exp2(__builtin_fmaf(sc[qb][kb][i], P.scale_log2, -lse2));
            const float dpv = dp[qb][kb][i];
            if constexpr (DROP) {
              const float pd = attn_keep_half(hh, kb, P.drop_thr) ? p : 0.f;
              sc[qb][kb][i] = pd;
              dp[qb][kb][i] = __builtin_fmaf(pd, dpv, -(p * del));
            } else {
              sc[qb][kb][i] = p;
              dp[qb][kb][i] = p * (dpv - del);
            }
          }
        }
    };
    // dV^T += dO^T P_d ; dK^T += Q^T dS over the 32 queries of half ks
    auto pv = [&](const char* sQ, int ks, const f32x4_t (&sc)[4][2], const f32x4_t (&dp)[4][2]) {
      const char* sD = sQ + TILE_BYTES;
      bf16x8_t pfr[2], sfr[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        pfr[kb] = pack_frag(sc[2 * ks][kb], sc[2 * ks + 1][kb]);
        sfr[kb] = pack_frag(dp[2 * ks][kb], dp[2 * ks + 1][kb]);
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8_t dof = rd_col(sD, ks * 32, ks * 32 + 16, db * 16, lane);
        const bf16x8_t qcf = rd_col(sQ, ks * 32, ks * 32 + 16, db * 16, lane);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          dv[kb][db] = mfma(dof, pfr[kb], dv[kb][db]);
          dk[kb][db] = mfma(qcf, sfr[kb], dk[kb][db]);
        }
      }
    };
    // one tile from LDS buffer BUFI (compile-time: every LDS address is a lane base plus an
    // immediate); the next tile's global loads are in flight meanwhile and stored into the other
    // buffer at the end
    f32x4_t sc[4][2], dp[4][2];
    auto tile = [&](int qt, auto bufi_c) {
      constexpr int BUFI = decltype(bufi_c)::value;
      const bool nxt = qt + 1 < ntiles && !(MODE & 2);
      if (nxt) load(qt + 1);
      const char* sQ = smem + BUFI * BUF;
      const float* sL = reinterpret_cast<const float*>(sQ + 2 * TILE_BYTES);
      const uint32_t hrow = DROP ? attn_row_term(static_cast<uint32_t>(bh * P.S + qt * KT + 4 * g)) +
                                       (static_cast<uint32_t>(k0 >> 1) + i16) * kAttnPairMul
                                 : 0u;
      // four phases, MFMA work beside independent VALU work of the same wave, spread one MFMA per
      // few VALU instructions by sched_group_barrier:
      //   S/dP(rows 0-31) + hashes(rows 0-31) | S/dP(rows 32-63) + P/dS(rows 0-31) + hashes(rows
      //   32-63) | dV/dK(rows 0-31) + P/dS(rows 32-63) | dV/dK(rows 32-63)
      uint32_t h0[2][4] = {}, h1[2][4] = {};
      sdp(sQ, 0, sc, dp);
      hashes(hrow, 0, h0);
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, DROP ? 3 : 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      sdp(sQ, 1, sc, dp);
      if constexpr (!(MODE & 1)) pds(sL, h0, 0, sc, dp);
      hashes(hrow, 1, h1);
      __builtin_amdgcn_sched_group_barrier(0x100, 12, 1);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x002, DROP ? 10 : 6, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      pv(sQ, 0, sc, dp);
      if constexpr (!(MODE & 1)) pds(sL, h1, 1, sc, dp);
      __builtin_amdgcn_sched_group_barrier(0x100, 20, 2);
      __builtin_amdgcn_sched_group_barrier(0x002, 8, 2);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        __builtin_amdgcn_sched_group_barrier(0x002, DROP ? 8 : 5, 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      pv(sQ, 1, sc, dp);
      if (nxt) store(smem + (BUFI ^ 1) * BUF);
      if constexpr (!(MODE & 4)) __syncthreads();
    };
    load(0);
    store(smem);
    __syncthreads();
    if constexpr ((MODE & 8) != 0) stamp[1] = __builtin_amdgcn_s_memtime();
    for (int qt = 0; qt < ntiles; qt += 2) {  // ntiles is even
      tile(qt, std::integral_constant<int, 0>{});
      tile(qt + 1, std::integral_constant<int, 1>{});
    }
    if constexpr ((MODE & 8) != 0) stamp[2] = __builtin_amdgcn_s_memtime();
  }
  // store dK (scaled by 1/sqrt(D)) and dV: lane holds key kb*16 + i16, d = db*16 + 4g + i; keys
  // >= len get zeros (their accumulators saw unmasked probabilities)
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const long long row = tok0 + k0 + kb * 16 + i16;
    bf16_t* pk = P.out + row * P.ld_out + h * D + 4 * g;
    bf16_t* pv = P.out2 + row * P.ld_out2 + h * D + 4 * g;
    const bool valid = k0 + kb * 16 + i16 < len;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4_t zero = {0.f, 0.f, 0.f, 0.f};
      const f32x4_t a = valid ? dk[kb][db] * P.scale : zero, c = valid ? dv[kb][db] : zero;
      *reinterpret_cast<uint2*>(pk + db * 16) = make_uint2(pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]));
      if constexpr ((MODE & 8) == 0)
        *reinterpret_cast<uint2*>(pv + db * 16) = make_uint2(pack_bf16x2(c[0], c[1]), pack_bf16x2(c[2], c[3]));
    }
  }
  if constexpr ((MODE & 8) != 0) {
    __builtin_amdgcn_s_waitcnt(0);
    stamp[3] = __builtin_amdgcn_s_memtime();
    stamp[5] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      long long* o = reinterpret_cast<long long*>(P.out2) + static_cast<long long>(blockIdx.x) * 8;
#pragma unroll
      for (int j = 0; j < 6; ++j) o[j] = stamp[j];
      o[6] = t;
      o[7] = __smid();
    }
  }
}

// ------------------------------------------------------------------------------ bwd dQ
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn_bwd_q_kernel(AttnParams P) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];
  const int qblocks = P.S / QBLK;
  const int t = tile::xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / qblocks, qblk = t - bh * qblocks;
  const int b = bh / P.H, h = bh - b * P.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int q0 = qblk * QBLK + wave * 32;
  const int len = P.seqlen ? min(P.seqlen[b], P.S) : P.S;
  const long long tok0 = static_cast<long long>(b) * P.S;

  bf16x8_t qf[2][2], df[2][2];
  float lse2[2], del[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const long long row = tok0 + q0 + qb * 16 + i16;
    float acc = 0.f;  // this lane's 16 of the row's 64 dims of dO . O
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qb][ks] = ldg_frag(P.q + row * P.ldq + h * D + ks * 32 + g * 8);
      df[qb][ks] = ldg_frag(P.dout + row * P.lddo + h * D + ks * 32 + g * 8);
      float a[8], d[8];
      unpack8(ldg16(P.o + row * P.ldo + h * D + ks * 32 + g * 8), a);
      unpack8(__builtin_bit_cast(uint4, df[qb][ks]), d);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += a[j] * d[j];
    }
    // the 4 lane groups g hold the row's 4 slices
    acc = tile::rows4_sum(acc);
    del[qb] = acc;
    const long long srow = static_cast<long long>(bh) * P.S + q0 + qb * 16 + i16;
    lse2[qb] = P.lse[srow];
    if (g == 0) P.delta[srow] = acc;
    if constexpr (DROP) {
      // dS = P * (keep * dP / (1-p) - delta) = P_d' * dP - P' * (delta * (1-p)) with P' = P / (1-p)
      // = exp2(s - (lse2 - log2(1/(1-p)))) and P_d' = keep ? P' : 0
      lse2[qb] -= __builtin_amdgcn_logf(P.drop_scale);
      del[qb] *= 1.f / P.drop_scale;
    }
  }
  f32x4_t dq[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int db = 0; db < 4; ++db) dq[qb][db] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  TileLoader lk, lv;
  lk.init(P.k + tok0 * P.ldk + h * D, P.ldk, tid);
  lv.init(P.v + tok0 * P.ldv + h * D, P.ldv, tid);
  const uint32_t key = DROP ? drop_key(P.rng, P.site) : 0u;
  const int ntiles = (len + KT - 1) / KT;
  if (ntiles > 0) {
    lk.load(0, len);
    lv.load(0, len);
    lk.store(smem);
    lv.store(smem + TILE_BYTES);
  }
  __syncthreads();
  // S, dP for the keys of half hk (kb = 2 hk, 2 hk + 1) of the tile: lane holds keys
  // kb*16 + 4g + i of query qb*16 + i16
  auto sdp = [&](const char* sK, int hk, f32x4_t (&sc)[2][4], f32x4_t (&dp)[2][4]) {
    const char* sV = sK + TILE_BYTES;
#pragma unroll
    for (int kb = 2 * hk; kb < 2 * hk + 2; ++kb) {
      const bf16x8_t k0f = rd_row(sK, kb * 16 + i16, g), k1f = rd_row(sK, kb * 16 + i16, 4 + g);
      const bf16x8_t v0f = rd_row(sV, kb * 16 + i16, g), v1f = rd_row(sV, kb * 16 + i16, 4 + g);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        sc[qb][kb] = mfma(k0f, qf[qb][0], f32x4_t{0.f, 0.f, 0.f, 0.f});
        sc[qb][kb] = mfma(k1f, qf[qb][1], sc[qb][kb]);
        dp[qb][kb] = mfma(v0f, df[qb][0], f32x4_t{0.f, 0.f, 0.f, 0.f});
        dp[qb][kb] = mfma(v1f, df[qb][1], dp[qb][kb]);
      }
    }
  };
  // dropout pair hashes of the tile at kbase for key half hk (pairs as in the forward kernel:
  // kb = 2 hk, 2 hk + 1 at the same i share one)
  auto hashes = [&](int kbase, int hk, uint32_t (&hp)[2][4]) {
    if constexpr (DROP)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const uint32_t hbase = attn_row_term(static_cast<uint32_t>(bh * P.S + q0 + qb * 16 + i16)) +
                               (static_cast<uint32_t>(kbase >> 1) + 4u * g + 16u * hk) * kAttnPairMul;
#pragma unroll
        for (int i = 0; i < 4; ++i) hp[qb][i] = attn_hash_input(key, hbase + static_cast<uint32_t>(i) * kAttnPairMul);
      }
  };
  // dS in place for key half hk. (DROP: lse2 / del carry the dropout scale, p is P / (1-p) — see
  // the prologue.) Keys >= len need no mask: their K rows are zero-filled in LDS, so whatever dS
  // they get adds nothing to dQ = dS K (and their S = 0, dP = 0 keep dS finite).
  auto pds = [&](int hk, const uint32_t (&hp)[2][4], f32x4_t (&sc)[2][4], const f32x4_t (&dp)[2][4]) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int kb = 2 * hk; kb < 2 * hk + 2; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = fast_exp2(__builtin_fmaf(sc[qb][kb][i], P.scale_log2, -lse2[qb]));
          const float dpv = dp[qb][kb][i];
          if constexpr (DROP) {
            const float pd = attn_keep_half(hp[qb][i], kb & 1, P.drop_thr) ? p : 0.f;
            sc[qb][kb][i] = __builtin_fmaf(pd, dpv, -(p * del[qb]));
          } else {
            sc[qb][kb][i] = p * (dpv - del[qb]);
          }
        }
  };
  // dQ += dS K over the 32 keys of half ks
  auto dqh = [&](const char* sK, int ks, const f32x4_t (&sc)[2][4]) {
    bf16x8_t sfr[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) sfr[qb] = pack_frag(sc[qb][2 * ks], sc[qb][2 * ks + 1]);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const bf16x8_t kc = rd_col(sK, ks * 32, ks * 32 + 16, db * 16, lane);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) dq[qb][db] = mfma(kc, sfr[qb], dq[qb][db]);
    }
  };
  // one 64-key tile in four phases (as attn_bwd_kv_kernel): S/dP(keys 0-31) + hashes | S/dP(keys
  // 32-63) + dS(keys 0-31) | dQ(keys 0-31) + dS(keys 32-63) | dQ(keys 32-63)
  int cur = 0;
  f32x4_t sc[2][4], dp[2][4];
  auto tile = [&](int kt) {
    const bool nxt = kt + 1 < ntiles;
    if (nxt) {
      lk.load((kt + 1) * KT, len);
      lv.load((kt + 1) * KT, len);
    }
    const char* sK = smem + cur * 2 * TILE_BYTES;
    const int kbase = kt * KT;
    uint32_t h0[2][4] = {}, h1[2][4] = {};
    sdp(sK, 0, sc, dp);
    hashes(kbase, 0, h0);
    hashes(kbase, 1, h1);
    __builtin_amdgcn_sched_barrier(0);
    sdp(sK, 1, sc, dp);
    pds(0, h0, sc, dp);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x002, DROP ? 6 : 4, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    dqh(sK, 0, sc);
    pds(1, h1, sc, dp);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 2);
    __builtin_amdgcn_sched_group_barrier(0x002, 4, 2);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
      __builtin_amdgcn_sched_group_barrier(0x002, DROP ? 12 : 8, 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    dqh(sK, 1, sc);
    if (nxt) {
      lk.store(smem + (cur ^ 1) * 2 * TILE_BYTES);
      lv.store(smem + (cur ^ 1) * 2 * TILE_BYTES + TILE_BYTES);
    }
    __syncthreads();
    cur ^= 1;
  };
  for (int kt = 0; kt < ntiles; ++kt) tile(kt);
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    bf16_t* op = P.out + (tok0 + q0 + qb * 16 + i16) * P.ld_out + h * D + 4 * g;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4_t v = dq[qb][db] * P.scale;
      *reinterpret_cast<uint2*>(op + db * 16) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
}

// ------------------------------------------------------------------------------ fused bwd
// dQ, dK and dV of one (batch, head) in ONE workgroup (S = 64 * NKB <= 512 keys): five MFMA
// products per (query slice, key tile) instead of the split kernels' seven (both recompute S and
// dP), every dropout hash computed once instead of twice, delta = rowsum(dO . O) formed while the
// query slice is staged, and no cross-workgroup sum for dQ (deterministic, no atomics).
//   * 4 waves, one per SIMD (launch_bounds(256, 1): 512 registers per lane); wave w owns keys
//     [w*16*NKB, (w+1)*16*NKB): its dK^T and dV^T live in accumulators for the whole sweep (key
//     on the MFMA lane, so the S / dP accumulators are already the B operands of dV^T += dO^T P
//     and dK^T += Q^T dS), its V fragments in registers;
//   * LDS: K of all S keys (S rows for the Q.K^T B operand, K^T column reads for dQ), dS^T of
//     the slice for all keys (two 32-column halves, alternating per slice), and the 32-query
//     slice of Q / dO / lse / delta double-buffered (register-staged one slice ahead);
//   * per slice: S, dP -> P, dS for each pair of 16-key tiles; dV^T, dK^T accumulate; dS^T to
//     LDS; one barrier; dQ[32 x 64] = dS . K split over the 4 waves (16 columns each), stored.
template <int NKB, int NW, bool DROP>
__global__ __launch_bounds__(NW * 64, 1) void attn_bwd_fused_kernel(AttnParams P) {
  constexpr int NT = NW * 64;
  constexpr int SK = 16 * NKB * NW;      // keys = queries of one (b, h)
  constexpr int QS = 32;                 // queries per slice
  constexpr int IMG = SK * 128;          // [SK][64] bf16 image
  constexpr int QT = QS * 128;           // [32][64] bf16 slice image
  constexpr int STAGE = 2 * QT + 2 * QS * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + 2 * STAGE];
  char* const sK = smem;
  char* const sDS = smem + IMG;
  char* const sStage = smem + 2 * IMG;
  const int bh = tile::xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / P.H, h = bh - b * P.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int key0 = wave * 16 * NKB;
  const int len = P.seqlen ? min(P.seqlen[b], SK) : SK;
  const long long tok0 = static_cast<long long>(b) * SK;
  const uint32_t key = DROP ? drop_key(P.rng, P.site) : 0u;

  // K image of all keys (keys >= len zeroed: their dS is 0, keep 0 * K finite)
  for (int c = tid; c < SK * 8; c += NT) {
    const int row = c >> 3, ch = c & 7;
    const uint4 v = row < len ? ldg16(P.k + (tok0 + row) * P.ldk + h * D + ch * 8) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(sK + tile::off64(row, ch * 8)) = v;
  }
  bf16x8_t vf[NKB][2];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      vf[kb][ks] = ldg_frag(P.v + (tok0 + key0 + kb * 16 + i16) * P.ldv + h * D + ks * 32 + g * 8);
  f32x4_t dk[NKB][4], dv[NKB][4];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int db = 0; db < 4; ++db) dk[kb][db] = dv[kb][db] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // slice staging: thread t moves row (t & 255) >> 3, 16-B chunk t & 7 of Q, dO and O (delta
  // partial); with 512 threads the first 256 take Q, the others dO and O
  constexpr bool SPLIT_STAGE = NT >= 512;
  const int srow = (tid & 255) >> 3, sch = tid & 7;
  const bool do_q = !SPLIT_STAGE || tid < 256, do_d = !SPLIT_STAGE || (tid >= 256 && tid < 512);
  uint4 rq = make_uint4(0, 0, 0, 0), rd = rq, ro = rq;
  float rl = 0.f;
  auto stage_load = [&](int s) {
    const long long row = tok0 + s * QS + srow;
    if (do_q) rq = ldg16(P.q + row * P.ldq + h * D + sch * 8);
    if (do_d) {
      rd = ldg16(P.dout + row * P.lddo + h * D + sch * 8);
      ro = ldg16(P.o + row * P.ldo + h * D + sch * 8);
    }
    if (tid < QS) rl = P.lse[static_cast<long long>(bh) * SK + s * QS + tid];
  };
  auto stage_store = [&](int buf) {
    char* st = sStage + buf * STAGE;
    if (do_q) *reinterpret_cast<uint4*>(st + tile::off64(srow, sch * 8)) = rq;
    float* stats = reinterpret_cast<float*>(st + 2 * QT);
    if (tid < QS) stats[tid] = rl;
    if (!do_d) return;
    *reinterpret_cast<uint4*>(st + QT + tile::off64(srow, sch * 8)) = rd;
    float a[8], d[8];
    unpack8(ro, a);
    unpack8(rd, d);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * d[j];
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (sch == 0) stats[QS + srow] = acc;
  };
  constexpr int NSL = SK / QS;
  stage_load(0);
  stage_store(0);
  __syncthreads();

  for (int s = 0; s < NSL; ++s) {
    const int cur = s & 1;
    if (s + 1 < NSL) stage_load(s + 1);
    const char* sQ = sStage + cur * STAGE;
    const char* sD = sQ + QT;
    const float* sL = reinterpret_cast<const float*>(sQ + 2 * QT);
    const int dcol = cur * 32;  // dS^T columns of this slice
#pragma unroll
    for (int pp = 0; pp < NKB / 2; ++pp) {
      const int k0 = key0 + pp * 32;
      // Q / dO row fragments (re-read from LDS per key pair: registers go to dK^T, dV^T, V)
      bf16x8_t qf[2][2], df[2][2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          qf[qb][ks] = rd_row(sQ, qb * 16 + i16, ks * 4 + g);
          df[qb][ks] = rd_row(sD, qb * 16 + i16, ks * 4 + g);
        }
      // S[q][key], dP[q][key]: lane holds q = qb*16 + 4g + i, key = k0 + j*16 + i16
      f32x4_t sc[2][2], dp[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8_t k0f = rd_row(sK, k0 + j * 16 + i16, g), k1f = rd_row(sK, k0 + j * 16 + i16, 4 + g);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          sc[qb][j] = mfma(qf[qb][0], k0f, f32x4_t{0.f, 0.f, 0.f, 0.f});
          sc[qb][j] = mfma(qf[qb][1], k1f, sc[qb][j]);
          dp[qb][j] = mfma(df[qb][0], vf[2 * pp + j][0], f32x4_t{0.f, 0.f, 0.f, 0.f});
          dp[qb][j] = mfma(df[qb][1], vf[2 * pp + j][1], dp[qb][j]);
        }
      }
      // P, dS in place (sc <- P * keep * scale, dp <- dS). Dropout: keys k0 + i16 and k0 + 16 + i16
      // (j = 0, 1) are the two halves of pair k0/2 + i16: one hash per lane per query row
      const uint32_t pair = static_cast<uint32_t>(k0 >> 1) + i16;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        // this lane's query rows qb*16 + 4g + i: lse2 and delta
        const f32x4_t ls = *reinterpret_cast<const f32x4_t*>(sL + qb * 16 + 4 * g);
        const f32x4_t dl = *reinterpret_cast<const f32x4_t*>(sL + QS + qb * 16 + 4 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t hh = 0u;
          if constexpr (DROP) {
            const int qg = s * QS + qb * 16 + 4 * g + i;
            hh = attn_pair_hash(key, attn_row_term(static_cast<uint32_t>(bh * SK + qg)), pair);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int kcol = k0 + j * 16 + i16;
            const float p = kcol < len ? fast_exp2(sc[qb][j][i] * P.scale_log2 - ls[i]) : 0.f;
            float dpv = dp[qb][j][i];
            float pd = p;
            if constexpr (DROP) {
              const bool kp = attn_keep_half(hh, j, P.drop_thr);
              pd = kp ? p * P.drop_scale : 0.f;
              dpv = kp ? dpv * P.drop_scale : 0.f;
            }
            sc[qb][j][i] = pd;
            dp[qb][j][i] = p * (dpv - dl[i]);
          }
        }
      }
      bf16x8_t pfr[2], sfr[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        pfr[j] = pack_frag(sc[0][j], sc[1][j]);
        sfr[j] = pack_frag(dp[0][j], dp[1][j]);
        // dS^T rows (keys) x this slice's 32 query columns, for dQ
        const uint4 w = __builtin_bit_cast(uint4, sfr[j]);
        *reinterpret_cast<uint2*>(sDS + tile::off64(k0 + j * 16 + i16, dcol + 4 * g)) = make_uint2(w.x, w.y);
        *reinterpret_cast<uint2*>(sDS + tile::off64(k0 + j * 16 + i16, dcol + 16 + 4 * g)) = make_uint2(w.z, w.w);
      }
      // dV^T += dO^T P ; dK^T += Q^T dS (contraction over the slice's 32 queries)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8_t dof = rd_col(sD, 0, 16, db * 16, lane);
        const bf16x8_t qcf = rd_col(sQ, 0, 16, db * 16, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          dv[2 * pp + j][db] = mfma(dof, pfr[j], dv[2 * pp + j][db]);
          dk[2 * pp + j][db] = mfma(qcf, sfr[j], dk[2 * pp + j][db]);
        }
      }
    }
    if (s + 1 < NSL) stage_store(cur ^ 1);
    __syncthreads();
    // dQ^T[d][q] of the slice: 8 tiles of 16 d x 16 q, tile t = (qb = t >> 2, db = t & 3);
    // wave w takes tiles w, w + NW, ...
    constexpr int TPW = 8 / NW;
    f32x4_t dq[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) dq[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int ks = 0; ks < SK / 32; ++ks) {
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int t = wave + u * NW, qb = t >> 2, db = t & 3;
        dq[u] = mfma(rd_col(sK, ks * 32, ks * 32 + 16, db * 16, lane),
                     rd_col(sDS, ks * 32, ks * 32 + 16, dcol + qb * 16, lane), dq[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      const int t = wave + u * NW, qb = t >> 2, db = t & 3;
      const f32x4_t v = dq[u] * P.scale;
      bf16_t* op = P.out + (tok0 + s * QS + qb * 16 + i16) * P.ld_out + h * D + db * 16 + 4 * g;
      *reinterpret_cast<uint2*>(op) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
  // dK (scaled by 1/sqrt(D)) and dV: lane holds key key0 + kb*16 + i16, d = db*16 + 4g + i
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    const long long row = tok0 + key0 + kb * 16 + i16;
    bf16_t* pk = P.out2 + row * P.ld_out2 + h * D + 4 * g;
    bf16_t* pv = P.out3 + row * P.ld_out3 + h * D + 4 * g;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4_t a = dk[kb][db] * P.scale, c = dv[kb][db];
      *reinterpret_cast<uint2*>(pk + db * 16) = make_uint2(pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]));
      *reinterpret_cast<uint2*>(pv + db * 16) = make_uint2(pack_bf16x2(c[0], c[1]), pack_bf16x2(c[2], c[3]));
    }
  }
}

AttnParams make_params(int B, int H, int S, const int* seqlen, float p_drop, const long long* rng, uint32_t site) {
  AttnParams P{};
  P.B = B;
  P.H = H;
  P.S = S;
  P.seqlen = seqlen;
  P.scale = 0.125f;  // 1/sqrt(64)
  P.scale_log2 = 0.125f * 1.4426950408889634f;
  P.drop_thr = drop_threshold16(p_drop);
  // unbiased for the keep probability the 16-bit threshold actually realises
  P.drop_scale = p_drop > 0.f ? static_cast<float>(65536.0 / (65536.0 - static_cast<double>(P.drop_thr))) : 1.f;
  P.rng = rng;
  P.site = site;
  return P;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace ttdk

using namespace ttdk;

// Shapes: S % 128 == 0, head_dim 64, every ld % 8 == 0 and bases 16-B aligned (checked).
// Returns hipErrorInvalidValue on violation (the Python wrapper raises).
TTDK_EXPORT int ttdk_attn_fwd(const bf16_t* q, long long ldq, const bf16_t* k, long long ldk, const bf16_t* v,
                              long long ldv, bf16_t* o, long long ldo, float* lse, const int* seqlen, int B, int H,
                              int S, float p_drop, const long long* rng, unsigned site, hipStream_t st) {
  if (S % QBLK || (ldq | ldk | ldv | ldo) & 7 || !aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o) ||
      (p_drop > 0.f && !rng))
    return hipErrorInvalidValue;
  AttnParams P = make_params(B, H, S, seqlen, p_drop, rng, site);
  P.q = q; P.k = k; P.v = v; P.ldq = ldq; P.ldk = ldk; P.ldv = ldv;
  P.out = o; P.ld_out = ldo; P.lse = lse;
  dim3 grid(B * H * (S / QBLK)), block(256);
  if (p_drop > 0.f) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, block, 0, st, P);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, block, 0, st, P);
  return hipGetLastError();
}

// Single-kernel backward (attn_bwd_fused_kernel) for S in {128, 256, 512}: opt-in
// (TTD_ATTN_FUSED_BWD=1 or ttdk_attn_set_fused_bwd(1)). Measured at BERT-Large b128 (S = 512,
// p = 0.1): 1190 us standalone vs 980 us for the split dQ / dK-dV kernels, BERT step 185.2 vs
// 177.2 ms — one workgroup per (b, h) holds 4 waves (the S = 512 dK^T / dV^T accumulators need
// 256 AGPRs per lane: one wave per SIMD, LDS 145 KB: one workgroup per CU), too little
// occupancy to hide the MFMA -> softmax dependencies; the 8-wave form spills 65 VGPRs.
static int g_attn_fused = -1;
static bool attn_fused_bwd() {
  if (g_attn_fused < 0) {
    const char* e = getenv("TTD_ATTN_FUSED_BWD");
    g_attn_fused = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return g_attn_fused != 0;
}
TTDK_EXPORT int ttdk_attn_set_fused_bwd(int on) {
  g_attn_fused = on ? 1 : 0;
  return 0;
}

// dq/dk/dv may alias one fused [tokens, 3*H*64] buffer (different column offsets).
TTDK_EXPORT int ttdk_attn_bwd(const bf16_t* q, long long ldq, const bf16_t* k, long long ldk, const bf16_t* v,
                              long long ldv, const bf16_t* o, long long ldo, const bf16_t* dout, long long lddo,
                              const float* lse, float* delta, bf16_t* dq, long long lddq, bf16_t* dk, long long lddk,
                              bf16_t* dv, long long lddv, const int* seqlen, int B, int H, int S, float p_drop,
                              const long long* rng, unsigned site, hipStream_t st) {
  if (S % QBLK || (ldq | ldk | ldv | ldo | lddo | lddq | lddk | lddv) & 7 || !aligned16(q) || !aligned16(k) ||
      !aligned16(v) || !aligned16(o) || !aligned16(dout) || (p_drop > 0.f && !rng))
    return hipErrorInvalidValue;
  AttnParams P = make_params(B, H, S, seqlen, p_drop, rng, site);
  P.q = q; P.k = k; P.v = v; P.o = o; P.dout = dout;
  P.ldq = ldq; P.ldk = ldk; P.ldv = ldv; P.ldo = ldo; P.lddo = lddo;
  P.lse = const_cast<float*>(lse);
  P.delta = delta;
  if (attn_fused_bwd() && (S == 128 || S == 256 || S == 512)) {
    // one workgroup per (batch, head): dQ, dK, dV in one pass (attn_bwd_fused_kernel)
    P.out = dq; P.ld_out = lddq; P.out2 = dk; P.ld_out2 = lddk; P.out3 = dv; P.ld_out3 = lddv;
    const dim3 g1(B * H);
    const bool d = p_drop > 0.f;
    // S = 512: 8 waves x 64 keys (two waves per SIMD); S = 256 / 128: 4 waves x 64 / 32 keys
    if (S == 512) {
      if (d) hipLaunchKernelGGL((attn_bwd_fused_kernel<4, 8, true>), g1, dim3(512), 0, st, P);
      else hipLaunchKernelGGL((attn_bwd_fused_kernel<4, 8, false>), g1, dim3(512), 0, st, P);
    } else if (S == 256) {
      if (d) hipLaunchKernelGGL((attn_bwd_fused_kernel<4, 4, true>), g1, dim3(256), 0, st, P);
      else hipLaunchKernelGGL((attn_bwd_fused_kernel<4, 4, false>), g1, dim3(256), 0, st, P);
    } else {
      if (d) hipLaunchKernelGGL((attn_bwd_fused_kernel<2, 4, true>), g1, dim3(256), 0, st, P);
      else hipLaunchKernelGGL((attn_bwd_fused_kernel<2, 4, false>), g1, dim3(256), 0, st, P);
    }
    return hipGetLastError();
  }
  dim3 grid(B * H * (S / QBLK)), block(256);
  // dQ first: it computes delta (rowsum dO . O) on the way and stores it for dK / dV
  P.out = dq; P.ld_out = lddq; P.out2 = nullptr;
  if (p_drop > 0.f) hipLaunchKernelGGL(attn_bwd_q_kernel<true>, grid, block, 0, st, P);
  else hipLaunchKernelGGL(attn_bwd_q_kernel<false>, grid, block, 0, st, P);
  P.out = dk; P.ld_out = lddk; P.out2 = dv; P.ld_out2 = lddv;
  static const int kv_diag = [] {
    const char* e = getenv("TTD_ATTN_KV_DIAG");
    return e ? atoi(e) : 0;
  }();
  if (p_drop > 0.f) {
    switch (kv_diag) {
      case 1: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 1>), grid, block, 0, st, P); break;
      case 2: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 2>), grid, block, 0, st, P); break;
      case 6: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 6>), grid, block, 0, st, P); break;
      case 7: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 7>), grid, block, 0, st, P); break;
      case 8: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 8>), grid, block, 0, st, P); break;
      case 15: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 15>), grid, block, 0, st, P); break;
      default: hipLaunchKernelGGL((attn_bwd_kv_kernel<true, 0>), grid, block, 0, st, P);
    }
  } else {
    hipLaunchKernelGGL(attn_bwd_kv_kernel<false>, grid, block, 0, st, P);
  }
  return hipGetLastError();
}
