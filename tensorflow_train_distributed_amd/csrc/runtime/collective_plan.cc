// CPU export of the native collective engine's per-rank call plan (kernels/collective_plan.h),
// for unit tests of the N-rank reduction arithmetic without a multi-GPU node.
#include "../kernels/collective_plan.h"

#include "common.h"

// out: kMaxSteps rows of 5 int64 (kind, root, send, recv, count). Returns the number of steps.
TTD_EXPORT int ttd_collective_plan(int algo, long long count, int nranks, int rank, long long* out) {
  ttd_coll::Step s[ttd_coll::kMaxSteps];
  const int n = ttd_coll::plan(algo, count, nranks, rank, s);
  for (int i = 0; i < n; ++i) {
    out[5 * i + 0] = s[i].kind;
    out[5 * i + 1] = s[i].root;
    out[5 * i + 2] = s[i].send;
    out[5 * i + 3] = s[i].recv;
    out[5 * i + 4] = s[i].count;
  }
  return n;
}

TTD_EXPORT int ttd_collective_plan_max_steps() { return ttd_coll::kMaxSteps; }
