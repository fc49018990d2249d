// 4-wave 256 x 256 bf16 GEMM: one wave per SIMD, 128 x 128 outputs per wave, the 64 fp32
// accumulator tiles (256 registers) in the AGPR half of the register file.
//
// Why a second 256-row main loop (gemm_conv.h big::gemm256*_kernel is the 8-wave ping-pong
// form): at the BERT-Large FFN1 shape the 8-wave loop keeps the MFMA pipes 50 % busy and its
// waves wait 34 % of their cycles (two waves per SIMD taking turns at barriers; 24
// ds_read_b128 per 64 MFMAs), where a 4-wave tile of 128 x 128 per wave reads half the LDS
// bytes per MFMA (32 ds_read_b128 per 128 MFMAs) and needs no turn-taking
// (profiles/r3_gemm_pmc_ours_vs_hipblaslt.txt). Reference op: tf.layers.dense MatMul,
// /root/reference/distribute_training.py:54,61 and its gradients (:152).
//
// Structure (K-major A and B; C = A . B^T, A [M][K], B [N][K]):
//  * operand tiles reach LDS by buffer_load ... lds (LDS-DMA, 16 B per lane) from a buffer
//    resource per operand: one VGPR of per-lane offset per operand, the piece / K-tile offsets
//    are scalar (soffset), and rows past M / N read zeros (out-of-range buffer loads);
//  * LDS: two stages of one 64-deep K-tile each (A 256 x 128 B + B 256 x 128 B = 64 KB);
//    rows of 128 B with the 16-B chunk index XOR (row >> 1) & 7 (conflict-free b128 reads);
//  * per K-tile and wave: 32 ds_read_b128 (16 per 32-deep K-step, double-buffered fragment
//    registers) and 128 v_mfma_f32_16x16x32_bf16; the schedule is
//      phase 0: MFMAs of K-step 0 | fragment reads of K-step 1
//      lgkmcnt(0), barrier (the stage is free)
//      phase 1a: first 32 MFMAs of K-step 1 | LDS-DMA of K-tile kt + 2 into the freed stage
//      vmcnt(DMA of kt + 2 in flight), barrier (K-tile kt + 1 has landed for every wave)
//      phase 1b: last 32 MFMAs of K-step 1 | fragment reads of K-tile kt + 1, K-step 0
//    so every DMA has a whole K-tile of MFMA work (2048 MFMA cycles) to land;
//  * MFMA operands swapped (D = B . A^T) so a lane holds 4 consecutive output columns of one
//    row; the register epilogue pairs lanes (g, g ^ 1) for 16-B stores.
#include "gemm_conv.h"

#include <type_traits>

typedef __attribute__((ext_vector_type(4))) int ttd_i32x4_t;
extern "C" __device__ void ttd_raw_buffer_load_lds(ttd_i32x4_t rsrc, __attribute__((address_space(3))) void* lds,
                                                   int size, int voffset, int soffset, int offset,
                                                   int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

namespace ttdk {
namespace {
namespace g4 {

constexpr int BM = 256, BN = 256, T = 256;
constexpr int OPB = 256 * 128;  // bytes of one operand's K-tile image
constexpr int STAGE = 2 * OPB;  // A then B
constexpr int SMEM = 2 * STAGE; // 128 KB

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ ttd_i32x4_t make_srd(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  ttd_i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane(static_cast<int>((a >> 32) & 0xffffu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r[3] = 0x00020000;
  return r;
}

// K-major operand loader: 256 rows x 128 B per K-tile in 8 LDS-DMA pieces per thread. Piece i
// of thread tid: LDS bytes (i * 256 + tid) * 16 = image row i * 32 + tid / 8, slot tid % 8, which
// holds chunk slot ^ ((row >> 1) & 7) = (tid & 7) ^ ((tid >> 4) & 7) for every i (32-row steps
// leave the swizzle term unchanged). Rows past the operand's end are clamped to its last row
// (their outputs are never stored), so every access is in range whatever the buffer unit does
// with soffset in its range check; the K-tile offset is scalar (soffset).
struct LoadK {
  ttd_i32x4_t srd;
  uint32_t voff[8];
  __device__ __forceinline__ void init(const bf16_t* p, long long ld, int rows, int row0, int tid) {
    const uint32_t bytes = static_cast<uint32_t>(static_cast<long long>(rows) * ld * 2);
    srd = make_srd(p, bytes);
    const int chunk = (tid & 7) ^ ((tid >> 4) & 7);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = min(row0 + i * 32 + (tid >> 3), rows - 1);
      voff[i] = static_cast<uint32_t>((static_cast<long long>(r) * ld + chunk * 8) * 2);
    }
  }
  // pieces [I0, I1) of K-tile kt into the operand image at lds (wave-uniform)
  template <int I0, int I1>
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = I0; i < I1; ++i)
      ttd_raw_buffer_load_lds(srd, (lds_void_t*)(lds + i * 4096 + wave * 1024), 16, static_cast<int>(voff[i]),
                              kt * 128, 0, 0);
  }
};

__device__ __forceinline__ bf16x8_t rd(const char* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

using big::kEkBias;
using big::kEkDGelu;
using big::kEkBeta;
using big::kEkAux;
using big::kEkGelu;

// Register epilogue: acc[a][b] = C[m0 + wm*128 + a*16 + (lane & 15)][n0 + wn*128 + b*16 + 4*(lane >> 4) + v].
// Lanes g and g ^ 1 (g = lane >> 4) swap halves of the column-block pair (2p, 2p + 1) so each lane
// stores 8 consecutive columns (16 B).
template <int EK, bool CHECK>
__device__ __forceinline__ void epilogue(const f32x4_t (&acc)[8][8], const EpiParams& E, int m0, int n0, int M, int N,
                                         float alpha, int lane, int wm, int wn) {
  const int g = lane >> 4, i16 = lane & 15;
  const bool odd = g & 1;
  bf16_t* const out = static_cast<bf16_t*>(E.out);
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int m = m0 + wm * 128 + a * 16 + i16;
    if (CHECK && m >= M) continue;
    const long long row = static_cast<long long>(m) * E.ldo;
    const long long rrow = static_cast<long long>(m) * E.ldr;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int nb = n0 + wn * 128 + p * 32 + 4 * g;  // block b = 2p + j: columns nb + 16 j
      uint2 po[2], pa[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = nb + 16 * j;
        f32x4_t v = acc[a][2 * p + j] * alpha;
        if constexpr ((EK & kEkBias) != 0)
          if (!CHECK || n < N) v += *reinterpret_cast<const f32x4_t*>(E.bias + n);
        if constexpr ((EK & kEkDGelu) != 0) {
          uint2 rv = make_uint2(0, 0);
          if (!CHECK || n < N) rv = *reinterpret_cast<const uint2*>(E.residual + rrow + n);
          v[0] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv.x & 0xffff)));
          v[1] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv.x >> 16)));
          v[2] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv.y & 0xffff)));
          v[3] *= gelu_tanh_grad(bf2f(static_cast<bf16_t>(rv.y >> 16)));
        }
        if constexpr ((EK & kEkBeta) != 0) {
          uint2 ov = make_uint2(0, 0);
          if (!CHECK || n < N) ov = *reinterpret_cast<const uint2*>(out + row + n);
          v[0] += bf2f(static_cast<bf16_t>(ov.x & 0xffff));
          v[1] += bf2f(static_cast<bf16_t>(ov.x >> 16));
          v[2] += bf2f(static_cast<bf16_t>(ov.y & 0xffff));
          v[3] += bf2f(static_cast<bf16_t>(ov.y >> 16));
        }
        if constexpr ((EK & kEkAux) != 0) pa[j] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        if constexpr ((EK & kEkGelu) != 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = gelu_tanh(v[q]);
        }
        po[j] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
      const int nst = odd ? nb + 12 : nb;
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

template <int EK>
__global__ __launch_bounds__(T, 1) void gemm4w_kernel(const bf16_t* __restrict__ A, long long lda,
                                                     const bf16_t* __restrict__ B, long long ldb, EpiParams E, int M,
                                                     int N, int K, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int nblk = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nblk);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ktiles = K / 64;

  LoadK la, lb;
  la.init(A, lda, M, m0, tid);
  lb.init(B, ldb, N, n0, tid);

  // per-lane fragment offsets for K-step ks: row i16, chunk 4 ks + g, XOR (i16 >> 1) & 7
  const int i16 = lane & 15, g = lane >> 4;
  const int lk0 = i16 * 128 + (((g) ^ ((i16 >> 1) & 7)) << 4);
  const int lk1 = i16 * 128 + (((4 | g) ^ ((i16 >> 1) & 7)) << 4);
  const int aoff = wm * 16384, boff = OPB + wn * 16384;

  f32x4_t acc[8][8];
  bf16x8_t fa[2][8], fb[2][8];

  auto stage = [&](int kt) { return smem + (kt & 1) * STAGE; };
  auto read = [&](const char* st, int lk, bf16x8_t (&xa)[8], bf16x8_t (&xb)[8]) {
    // order of first use in the a-major MFMA sweep: a0, b0..b7, a1..a7
    xa[0] = rd(st + aoff + lk);
#pragma unroll
    for (int b = 0; b < 8; ++b) xb[b] = rd(st + boff + b * 2048 + lk);
#pragma unroll
    for (int a = 1; a < 8; ++a) xa[a] = rd(st + aoff + a * 2048 + lk);
  };
  // MFMAs as inline asm with the accumulator an "a" operand: hipcc allocates the 64 tiles in
  // AGPRs and leaves them there (with the builtin it re-homed accumulators between the VGPR and
  // AGPR halves every K-tile: 368 v_accvgpr_* per 128 MFMAs). FIRST: C = 0 (no zero-fill writes
  // into AGPRs, whose VALU-write -> MFMA-read wait states hipcc would not pad inside asm).
  auto mma = [&](const bf16x8_t (&xa)[8], const bf16x8_t (&xb)[8], int a0, int a1, auto first) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = a0; a < a1; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if constexpr (decltype(first)::value)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[a][b]) : "v"(xb[b]), "v"(xa[a]));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[a][b]) : "v"(xb[b]), "v"(xa[a]));
      }
    __builtin_amdgcn_s_setprio(0);
  };
  using F = std::false_type;
  using Tr = std::true_type;

  // prologue: K-tiles 0 and 1, wait for 0, read its K-step 0
  if (ktiles > 0) {
    la.issue<0, 8>(stage(0), 0, wave);
    lb.issue<0, 8>(stage(0) + OPB, 0, wave);
    if (ktiles > 1) {
      la.issue<0, 8>(stage(1), 1, wave);
      lb.issue<0, 8>(stage(1) + OPB, 1, wave);
      wait_vm<16>();
    } else {
      wait_vm<0>();
    }
    bar();
    read(stage(0), lk0, fa[0], fb[0]);
  }
  auto ktile = [&](int kt, auto first) {
    const bool has1 = kt + 1 < ktiles, has2 = kt + 2 < ktiles;
    char* cs = stage(kt);
    // phase 0: K-step 0 MFMAs, K-step 1 fragments
    read(cs, lk1, fa[1], fb[1]);
    mma(fa[0], fb[0], 0, 8, first);
    wait_lgkm0();
    bar();
    // phase 1a: DMA of K-tile kt + 2 into this stage
    if (has2) {
      la.issue<0, 8>(cs, kt + 2, wave);
      lb.issue<0, 8>(cs + OPB, kt + 2, wave);
    }
    mma(fa[1], fb[1], 0, 4, F{});
    if (has1) {
      if (has2) wait_vm<16>(); else wait_vm<0>();
    }
    bar();
    // phase 1b: K-tile kt + 1's K-step 0 fragments
    if (has1) read(stage(kt + 1), lk0, fa[0], fb[0]);
    mma(fa[1], fb[1], 4, 8, F{});
  };
  ktile(0, Tr{});
  for (int kt = 1; kt < ktiles; ++kt) ktile(kt, F{});
  // the last MFMAs' results -> the epilogue's v_accvgpr_read: XDL write -> read wait states
  // (hipcc pads nothing after asm); the empty "+a" statements order every read after the pad
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) asm volatile("" : "+a"(acc[a][b]));

  const float alpha = epi_alpha(E);
  if (m0 + BM <= M && n0 + BN <= N) epilogue<EK, false>(acc, E, m0, n0, M, N, alpha, lane, wm, wn);
  else epilogue<EK, true>(acc, E, m0, n0, M, N, alpha, lane, wm, wn);
}

}  // namespace g4
}  // namespace
}  // namespace ttdk

// C[M,N] = epilogue(alpha * A . B^T), A [M][K] (lda), B [N][K] (ldb) bf16 K-major; K % 64 == 0,
// N % 8 == 0, ldo % 8 == 0, 16-B aligned operands and outputs. Returns hipErrorInvalidValue for
// shapes this kernel does not take (the caller keeps another path).
TTDK_EXPORT int ttdk_gemm4w_bf16(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                                 const TtdkEpilogue* epi, hipStream_t st) {
  using namespace ttdk;
  EpiParams pe = to_epi(epi);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const long long lim = 1LL << 32;
  if (K < 64 || K % 64 || N % 8 || lda % 8 || ldb % 8 || pe.ldo % 8 || !al16(A) || !al16(B) || !al16(pe.out) ||
      (static_cast<long long>(M) + 256) * lda * 2 >= lim || (static_cast<long long>(N) + 256) * ldb * 2 >= lim ||
      pe.mode != 0 || pe.remap || pe.stat || pe.by || pe.bH)
    return hipErrorInvalidValue;
  int ek = -1;
  if (pe.act == kActNone && !pe.residual) ek = 0;
  else if (pe.act == kActGelu && !pe.residual) ek = g4::kEkGelu;
  else if (pe.act == kActDGelu && pe.residual) ek = g4::kEkDGelu;
  if (ek < 0) return hipErrorInvalidValue;
  if (pe.bias) ek |= g4::kEkBias;
  if (pe.beta) ek |= g4::kEkBeta;
  if (pe.aux) ek |= g4::kEkAux;
  const int tm = ceil_div(M, g4::BM), tn = ceil_div(N, g4::BN);
#define TTDK_G4(EKV)                                                                                             \
  case EKV:                                                                                                      \
    hipLaunchKernelGGL((g4::gemm4w_kernel<EKV>), dim3(tm * tn), dim3(g4::T), 0, st, A, lda, B, ldb, pe, M, N, K, \
                       tm, tn);                                                                                  \
    return hipGetLastError();
  switch (ek) {
    TTDK_G4(0)
    TTDK_G4(g4::kEkBias)
    TTDK_G4(g4::kEkBias | g4::kEkAux | g4::kEkGelu)
    TTDK_G4(g4::kEkDGelu)
    TTDK_G4(g4::kEkBeta)
    default: break;
  }
#undef TTDK_G4
  return hipErrorInvalidValue;
}
