#pragma once
// Host-side plan of one bucket reduction: the sequence of RCCL calls each rank issues for a
// tf.distribute cross-device algorithm (parallel/strategy.py), as plain data. The native
// engine (collective.hip) executes exactly this list; libttd_rt.so exports the same function
// (runtime/collective_plan.cc) so the arithmetic of the N-rank branches — chunk offsets, the
// count % nranks tail, matching call sequences on every rank — is unit-tested on the CPU
// (tests/test_rccl_engine.py) without a multi-GPU node.
//
// Algorithms:
//   0 allreduce      one all-reduce of the whole bucket (RcclAllReduce / NcclAllReduce)
//   1 hierarchical   reduce-scatter into this rank's chunk + all-gather of the chunks
//                    (HierarchicalCopyAllReduce); the count % nranks elements past the last
//                    whole chunk ride in one small all-reduce
//   2 reduce_to_one  reduce to rank 0 + broadcast from rank 0 (ReductionToOneDevice)
// A one-rank group always plans a single all-reduce (identity for SUM / AVG), so a one-GPU run
// still goes through RCCL.

namespace ttd_coll {

enum Kind : int { kAllReduce = 0, kReduceScatter = 1, kAllGather = 2, kReduce = 3, kBroadcast = 4 };

// One RCCL call on the bucket buffer (offsets / counts in elements):
//   kAllReduce      in place on [send, send + count)
//   kReduceScatter  send = start of nranks * count elements, recv = this rank's chunk
//   kAllGather      send = this rank's chunk (count elements), recv = start of nranks * count
//   kReduce         in place on [send, send + count), result on rank `root`
//   kBroadcast      in place on [send, send + count) from rank `root`
struct Step {
  int kind;
  int root;
  long long send;
  long long recv;
  long long count;
};

constexpr int kMaxSteps = 3;

// Fills out[0..n) and returns n (0 for an empty bucket, -1 for a bad argument).
inline int plan(int algo, long long count, int nranks, int rank, Step* out) {
  if (count < 0 || nranks < 1 || rank < 0 || rank >= nranks || algo < 0 || algo > 2) return -1;
  if (count == 0) return 0;
  int n = 0;
  if (nranks == 1 || algo == 0) {
    out[n++] = Step{kAllReduce, 0, 0, 0, count};
    return n;
  }
  if (algo == 1) {
    const long long per = count / nranks, main = per * nranks;
    if (per > 0) {
      out[n++] = Step{kReduceScatter, 0, 0, rank * per, per};
      out[n++] = Step{kAllGather, 0, rank * per, 0, per};
    }
    if (main < count) out[n++] = Step{kAllReduce, 0, main, main, count - main};
    return n;
  }
  out[n++] = Step{kReduce, 0, 0, 0, count};
  out[n++] = Step{kBroadcast, 0, 0, 0, count};
  return n;
}

}  // namespace ttd_coll
