// CPU export of the direct xGMI all-reduce plan (kernels/ipc_plan.h): path choice and the
// rank-chunk / workgroup-part partition, for unit tests without a multi-GPU node.
#include "../kernels/ipc_plan.h"

#include "common.h"

TTD_EXPORT int ttd_ipc_choose(long long bytes, int world, int same_node, long long cap) {
  return ttd_ipc::choose(bytes, world, same_node, cap);
}

TTD_EXPORT void ttd_ipc_chunk(long long count, int vec, int world, int r, long long* lo, long long* hi) {
  ttd_ipc::chunk(count, vec, world, r, lo, hi);
}

TTD_EXPORT void ttd_ipc_part(long long lo, long long hi, int vec, int nb, int b, long long* plo, long long* phi) {
  ttd_ipc::part(lo, hi, vec, nb, b, plo, phi);
}

TTD_EXPORT int ttd_ipc_blocks(long long bytes, int budget) { return ttd_ipc::blocks_for(bytes, budget); }
