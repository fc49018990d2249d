// MFMA tile helpers shared by the attention kernels (gfx950, v_mfma_f32_16x16x32_bf16).
//
// Operand convention used throughout: mfma(X, Y, acc) with X/Y bf16x8 fragments where lane l
// supplies X[row = l & 15][k = 8 * (l >> 4) .. +8] and Y[col = l & 15][k = ...]; the result
// lane l holds acc[i] = sum_k X[4 * (l >> 4) + i][k] * Y[l & 15][k], i = 0..3 — i.e. the
// X index runs over 4 consecutive values per lane, the Y index lies on lane & 15.
//
// LDS images are 64-element (128-B) rows with the 16-B chunk index XOR-swizzled by row & 7:
// b128 row reads (K-major fragments, 16 rows per lane group), ds_read_b64_tr_b16 column reads
// (8 consecutive rows x 2 chunks per 32-lane half) and the fused backward's b64 dS stores
// (16 rows, one chunk) are all conflict-free, so one copy of a tile serves both orientations.
// (The previous XOR, (row >> 1) & 7, put rows r and r + 2 of a column read on the same two
// slots: a 2-way conflict on every transposed read — 28M conflict cycles per BERT-Large
// attn_bwd_kv launch, profiles/r5_attn_bwd_pmc_before.txt.)
#pragma once
#include "common.h"

namespace ttdk {
namespace tile {

__device__ __forceinline__ int off64(int row, int col) {  // byte offset of element (row, col), col % 4 == 0 ok
  return row * 128 + ((((col >> 3) ^ (row & 7))) << 4) + ((col & 7) << 1);
}

__device__ __forceinline__ bf16x8_t rd_row(const char* lds, int row, int kchunk) {
  return *reinterpret_cast<const bf16x8_t*>(lds + off64(row, kchunk * 8));
}

__device__ __forceinline__ s16x4_t rd_tr(const char* p) {
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p));
}

// Column fragment of a [rows][64] image: lane gets column (colbase + (lane & 15)) and the
// 8 k-rows {r0 + 4g .. r0 + 4g + 3} U {r1 + 4g .. r1 + 4g + 3}, g = lane >> 4.
__device__ __forceinline__ bf16x8_t rd_col(const char* lds, int r0, int r1, int colbase, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const s16x4_t lo = rd_tr(lds + off64(r0 + 4 * g + q, colbase + 4 * p));
  const s16x4_t hi = rd_tr(lds + off64(r1 + 4 * g + q, colbase + 4 * p));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ f32x4_t mfma(const bf16x8_t& x, const bf16x8_t& y, const f32x4_t& acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t pack_frag(const f32x4_t& a, const f32x4_t& b) {
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
  u32x4_t w = {pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(b[0], b[1]), pack_bf16x2(b[2], b[3])};
  return __builtin_bit_cast(bf16x8_t, w);
}

// Max / sum over the four lanes {l, l^16, l^32, l^48} (one MFMA result row spread over the 4 lane
// groups) on the VALU with the gfx950 permlane swaps instead of two ds_bpermute round trips
// through LDS (each followed by an lgkmcnt(0) wait in the softmax's serial chain).
__device__ __forceinline__ float rows4_max(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __builtin_elementwise_maximum(__uint_as_float(a[0]), __uint_as_float(a[1]));  // no canonicalising max
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __builtin_elementwise_maximum(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows4_sum(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Bijective blockIdx -> work-item map that keeps consecutive work items on one XCD
// (hardware dispatches blockIdx round-robin over the 8 XCDs).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace tile

// ---------------------------------------------------------------- dropout hash
// Counter-based 32-bit hash (murmur3 finalizer) for dropout masks that must be regenerated
// bit-identically in backward. The per-call key folds (seed, step, site) read from DEVICE
// memory, so a hipGraph-captured step draws a fresh mask each replay when the step counter
// advances on the device.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t drop_key(const long long* rng, uint32_t site) {
  const unsigned long long seed = static_cast<unsigned long long>(rng[0]);
  const unsigned long long step = static_cast<unsigned long long>(rng[1]);
  uint32_t k = fmix32(static_cast<uint32_t>(seed) ^ 0x243F6A88u);
  k = fmix32(k ^ static_cast<uint32_t>(seed >> 32) ^ (site * 0x9E3779B9u));
  k = fmix32(k ^ static_cast<uint32_t>(step) * 0x85EBCA77u ^ static_cast<uint32_t>(step >> 32));
  return k;
}

// keep iff hash >= threshold, threshold = p * 2^32 (saturated)
__device__ __forceinline__ bool drop_keep(uint32_t key, unsigned long long idx, uint32_t thr) {
  const uint32_t h = fmix32(key ^ (static_cast<uint32_t>(idx) * 0x9E3779B1u + static_cast<uint32_t>(idx >> 32) * 0x7FEB352Du));
  return h >= thr;
}

// Attention-probability dropout: one hash per PAIR of keys of a query row, each key taking one
// 16-bit half (keep iff half >= thr16 = floor(p * 2^16)). Key k belongs to pair
// ((k >> 5) << 4) | (k & 15) and takes half (k >> 4) & 1: keys k and k + 16 of an aligned 32-key
// block share a hash, and every kernel's lane layout holds both in ONE lane (fwd / bwd_q: key
// tiles kb and kb + 1 at the same i; bwd_kv / fused: the two 16-key tiles of a 32-key block at
// the same lane), so no lane exchange is needed. (Adjacent-key pairs sat in lanes l and l ^ 1 of
// the backward layouts: a DPP move and two byte permutes per hash.) The hash input is
// rowid * C1 + pair * C2 with rowid = (b*H + h)*S + q, so a lane derives its row term once and
// pays one mix per two probabilities. ops/transformer.attention_keep_mask mirrors it.
constexpr uint32_t kAttnPairMul = 0x7FEB352Du;
__device__ __forceinline__ uint32_t attn_row_term(uint32_t rowid) { return rowid * 0x9E3779B1u; }
__device__ __forceinline__ uint32_t attn_pair_of(uint32_t k) { return ((k >> 5) << 4) | (k & 15u); }
// One xorshift - 24-bit multiply - xorshift round: the hash is regenerated for every probability
// pair in the forward and both backward kernels, whose VALU issue bounds them; v_mul_u32_u24 is a
// full-rate instruction where the 32-bit v_mul_lo_u32 is quarter rate (16 of ~300 VALU
// instructions per tile, ~15 % of the tile's VALU cycles). Bits 24-31 of the input reach the
// product through the first xorshift (into bits 8-15). The input is already an odd-multiplier
// progression over (row, pair) xor a murmur-mixed key; statistics (keep rate, pair-half /
// neighbour-pair / neighbour-row / neighbour-head independence, same as the 32-bit multiply within
// sampling noise) are pinned by tests/test_kernels_transformer.py on the mirror.
__device__ __forceinline__ uint32_t attn_mix(uint32_t h) {
  h ^= h >> 16;
  // 24 x 24-bit multiply-add (one full-rate v_mad_u32_u24): the high byte, which the 24-bit
  // multiply cannot see, is added in, so all 32 input bits reach the output (the multiply alone
  // had at most 2^24 distinct outputs: x and x ^ 0x01000100 collided)
  h = __umul24(h, 0x9E3779u) + (h >> 24);
  h ^= h >> 16;
  return h;
}
// hash of a precomputed input row_term + pair * kAttnPairMul (kernels walking consecutive pairs
// form it incrementally instead of multiplying per pair)
__device__ __forceinline__ uint32_t attn_hash_input(uint32_t key, uint32_t input) { return attn_mix(key ^ input); }
__device__ __forceinline__ uint32_t attn_pair_hash(uint32_t key, uint32_t row_term, uint32_t pair) {
  return attn_hash_input(key, row_term + pair * kAttnPairMul);
}
// keep test of half `hi` ((key >> 4) & 1) of a pair hash
__device__ __forceinline__ bool attn_keep_half(uint32_t h, bool hi, uint32_t thr16) {
  return (hi ? (h >> 16) : (h & 0xffffu)) >= thr16;
}

inline uint32_t drop_threshold16(float p) {
  if (p <= 0.f) return 0u;
  if (p >= 1.f) return 0x10000u;
  return static_cast<uint32_t>(static_cast<double>(p) * 65536.0);
}

inline uint32_t drop_threshold(float p) {
  if (p <= 0.f) return 0u;
  if (p >= 1.f) return 0xffffffffu;
  return static_cast<uint32_t>(static_cast<double>(p) * 4294967296.0);
}

}  // namespace ttdk
