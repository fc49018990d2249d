#pragma once
// Host/device plan of the direct xGMI all-reduce for small gradient buckets (ipc_allreduce.hip):
// which path a bucket takes and how its elements are split over ranks (two-shot chunks) and
// over workgroups (parts), as plain arithmetic. libttd_rt.so exports the same functions
// (runtime/ipc_plan.cc) so the choice logic and the partition's exact-cover property are
// unit-tested on the CPU (tests/test_ipc_plan.py) without a multi-GPU node.
//
// Why a second all-reduce next to RCCL: a ring all-reduce of a 1 MB bucket over 8 xGMI peers
// is 14 latency-bound steps; the first bucket of the backward (its communication should start
// as early as possible) and the last one (its all-reduce is fully exposed: nothing of the
// backward is left to hide it) are exactly the latency-bound ones. With every peer's staging
// buffer mapped into every process (hipIpcOpenMemHandle), a rank reads its peers' data over
// the point-to-point links directly:
//   one-shot (<= kOneShotMax):  every rank sums the whole bucket from all peers — 1 barrier,
//                               world x bytes read per rank, no ring steps;
//   two-shot (<= kTwoShotMax):  reduce-scatter (rank r sums chunk r from all peers) + all-gather
//                               (rank r copies chunk q from peer q) — 2 barriers, 2 x bytes
//                               per rank over the links;
//   RCCL (larger):              bandwidth-bound, the ring / tree stays better.

// (constexpr: host and device code share these, hipcc treats constexpr functions as both)
namespace ttd_ipc {

enum Path : int { kRccl = 0, kOneShot = 1, kTwoShot = 2 };

constexpr long long kOneShotMax = 1LL << 20;
constexpr long long kTwoShotMax = 8LL << 20;
constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;

// Path of a bucket of `bytes` on a group of `world` ranks. same_node: every rank of the group is
// on this node (the peers' memory is mappable); cap: bytes of the staging buffers (0 = none).
constexpr int choose(long long bytes, int world, int same_node, long long cap) {
  if (!same_node || world < 2 || world > kMaxRanks || bytes <= 0 || bytes > cap) return kRccl;
  if (bytes <= kOneShotMax) return kOneShot;
  if (bytes <= kTwoShotMax) return kTwoShot;
  return kRccl;
}

constexpr long long ceil_div_ll(long long a, long long b) { return (a + b - 1) / b; }

// Two-shot chunk r of `count` elements over `world` ranks, in whole vectors of `vec` elements
// (16 B): [*lo, *hi). Chunks are contiguous, in rank order, and cover [0, count) exactly once
// (trailing chunks may be empty).
constexpr void chunk(long long count, int vec, int world, int r, long long* lo, long long* hi) {
  const long long per = ceil_div_ll(ceil_div_ll(count, vec), world) * vec;
  long long a = per * r, b = per * (r + 1);
  if (a > count) a = count;
  if (b > count) b = count;
  *lo = a;
  *hi = b;
}

// Part b of nb of the element range [lo, hi), in whole vectors: contiguous, in block order,
// covering the range exactly once.
constexpr void part(long long lo, long long hi, int vec, int nb, int b, long long* plo, long long* phi) {
  const long long per = ceil_div_ll(ceil_div_ll(hi - lo, vec), nb) * vec;
  long long a = lo + per * b, e = lo + per * (b + 1);
  if (a > hi) a = hi;
  if (e > hi) e = hi;
  *plo = a;
  *phi = e;
}

// Workgroups of one launch: ~16 KB of the bucket per workgroup, 8 .. kMaxBlocks, and never more
// than `budget` (> 0): the CTA budget the RCCL engine was given for the collectives that run
// next to the backward (rccl.choose_cta_budget), so the direct path spins on no more CUs than
// RCCL would hold.
constexpr int blocks_for(long long bytes, int budget = 0) {
  long long b = ceil_div_ll(bytes, 16 << 10);
  if (b < 8) b = 8;
  if (b > kMaxBlocks) b = kMaxBlocks;
  if (budget > 0 && b > budget) b = budget;
  return static_cast<int>(b);
}

}  // namespace ttd_ipc
