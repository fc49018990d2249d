// Native collective engine: one RCCL communicator per replica group, driven from C++ on its own
// HIP stream (the MirroredStrategy / MultiWorkerMirroredStrategy gradient aggregation of
// BASELINE.json's north star; the reference aggregates through PS accumulators instead,
// /root/reference/distribute_training.py:142-148).
//
// Why native instead of torch.distributed's process group:
//  * the gradient buckets are slices of ONE flat fp32 buffer (train/flat.py): a bucket launch is
//    an event fork from the producing stream (the side stream that finished the bucket's weight
//    gradients) onto the communicator stream, then the RCCL call(s) — no tensor wrappers, no
//    record_stream bookkeeping, no per-call Python work objects;
//  * the communicator stream's priority is ours to choose (below the main chain's high-priority
//    stream, so BN / reduce kernels of the backward keep dispatching ahead of RCCL's workgroups)
//    and so is RCCL's CTA budget (minCTAs / maxCTAs: how many CUs a collective may occupy while
//    it overlaps the backward GEMMs);
//  * every call is stream-ordered and host-sync free, so the whole step — collectives
//    included — can be captured in one hipGraph (RCCL supports stream capture);
//  * bf16 gradient compression casts on the communicator stream (no extra pass on the compute
//    streams).
// Host waits (ttdc_synchronize) poll the stream and the communicator's asynchronous error
// against a deadline, so a peer that died becomes an error the recoverable session can act on
// (parallel/fault.py), not a hung process. Optionally (nonblocking = 1: ncclConfig.blocking = 0)
// creation is polled against the same deadline too; the default blocking communicator issues
// every collective from the calling thread, which hipGraph stream capture needs.
//
// Reduction algorithms (tf.distribute cross-device ops, parallel/strategy.py):
//   0 allreduce      one ring/tree all-reduce (RcclAllReduce / NcclAllReduce)
//   1 hierarchical   in-place reduce-scatter + all-gather (HierarchicalCopyAllReduce); the
//                    count % nranks tail rides in a small all-reduce
//   2 reduce_to_one  reduce to rank 0 + broadcast (ReductionToOneDevice)
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace ttdk {
namespace {

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  const long long n8 = n / 8;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i], b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
  for (long long i = n8 * 8 + static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    y[i] = f2bf(x[i]);
}

__global__ void bf16_to_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long long n) {
  const long long n8 = n / 8;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], f);
    reinterpret_cast<float4*>(y)[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(y)[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  for (long long i = n8 * 8 + static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    y[i] = bf2f(x[i]);
}

int cast_grid(long long n) {
  long long b = (n / 8 + 255) / 256;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;  // grid-stride; 2048 x 256 threads keep HBM busy without a long tail
  return static_cast<int>(b);
}

ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat64;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    default: return ncclFloat32;
  }
}

size_t dt_size(int dt) {
  switch (dt) {
    case 1: return 2;
    case 2: case 4: return 8;
    case 5: return 1;
    default: return 4;
  }
}

ncclRedOp_t to_op(int op) {
  switch (op) {
    case 1: return ncclAvg;
    case 2: return ncclMin;
    case 3: return ncclMax;
    default: return ncclSum;
  }
}

thread_local std::string g_err;

struct Engine {
  ncclComm_t comm = nullptr;
  hipStream_t cs = nullptr;  // communicator stream
  int rank = 0, nranks = 1, device = 0;
  double timeout = 300.0;
  hipEvent_t fork[64];      // producer -> communicator stream (ring of events)
  int fork_next = 0;
  hipEvent_t join = nullptr;
  void* stage = nullptr;    // bf16 staging for compressed buckets
  size_t stage_bytes = 0;
  bool failed = false;
  std::string err;
  // per-bucket timing (ttdc_set_timing): events around each bucket's reduction on the
  // communicator stream, recorded after its fork wait is satisfied
  bool timing = false;
  std::vector<hipEvent_t> t_begin, t_end;
  int n_timed = 0;
};

bool set_err(Engine* e, const std::string& m) {
  if (e) {
    e->err = m;
    e->failed = true;
  }
  g_err = m;
  return false;
}

// Wait for a non-blocking communicator to leave ncclInProgress (after init or an enqueue).
bool settle(Engine* e, ncclResult_t r, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    ncclResult_t a = ncclSuccess;
    const ncclResult_t q = ncclCommGetAsyncError(e->comm, &a);
    if (q != ncclSuccess) { r = q; break; }
    r = a;
    if (r != ncclInProgress) break;
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > e->timeout) {
      char b[256];
      snprintf(b, sizeof b, "%s: no progress after %.0f s (a peer did not join)", what, dt);
      return set_err(e, b);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(dt < 0.01 ? 5 : 500));
  }
  if (r != ncclSuccess) {
    const char* last = e->comm ? ncclGetLastError(e->comm) : "";
    return set_err(e, std::string(what) + ": " + ncclGetErrorString(r) + (last && *last ? std::string(" (") + last + ")" : ""));
  }
  return true;
}

bool hip_ok(Engine* e, hipError_t h, const char* what) {
  if (h == hipSuccess) return true;
  return set_err(e, std::string(what) + ": " + hipGetErrorString(h));
}

// Order the communicator stream after everything already queued on `producer`.
bool fork_from(Engine* e, hipStream_t producer) {
  hipEvent_t ev = e->fork[e->fork_next];
  e->fork_next = (e->fork_next + 1) % 64;
  return hip_ok(e, hipEventRecord(ev, producer), "hipEventRecord") &&
         hip_ok(e, hipStreamWaitEvent(e->cs, ev, 0), "hipStreamWaitEvent");
}

bool reduce_on(Engine* e, void* buf, size_t count, ncclDataType_t dt, size_t esz, ncclRedOp_t op, int algo,
               hipStream_t s) {
  if (count == 0) return true;
  if (e->nranks == 1) {
    // a one-rank group still goes through RCCL (the same code path as N ranks: it validates the
    // buffers and lets a one-GPU run exercise the engine); SUM / AVG of one replica = identity
    return settle(e, ncclAllReduce(buf, buf, count, dt, op, e->comm, s), "ncclAllReduce");
  }
  char* p = static_cast<char*>(buf);
  if (algo == 1) {
    const size_t per = count / e->nranks, main = per * e->nranks;
    if (per > 0) {
      char* mine = p + e->rank * per * esz;
      if (!settle(e, ncclReduceScatter(p, mine, per, dt, op, e->comm, s), "ncclReduceScatter")) return false;
      if (!settle(e, ncclAllGather(mine, p, per, dt, e->comm, s), "ncclAllGather")) return false;
    }
    if (main < count)
      return settle(e, ncclAllReduce(p + main * esz, p + main * esz, count - main, dt, op, e->comm, s), "ncclAllReduce");
    return true;
  }
  if (algo == 2) {
    if (!settle(e, ncclReduce(p, p, count, dt, op, 0, e->comm, s), "ncclReduce")) return false;
    return settle(e, ncclBroadcast(p, p, count, dt, 0, e->comm, s), "ncclBroadcast");
  }
  return settle(e, ncclAllReduce(p, p, count, dt, op, e->comm, s), "ncclAllReduce");
}

}  // namespace
}  // namespace ttdk

using namespace ttdk;

TTDK_EXPORT const char* ttdc_error(void* h) {
  Engine* e = static_cast<Engine*>(h);
  return e ? e->err.c_str() : g_err.c_str();
}

TTDK_EXPORT int ttdc_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

TTDK_EXPORT int ttdc_unique_id(char* out) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    g_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return -1;
  }
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return NCCL_UNIQUE_ID_BYTES;
}

// Create the communicator for (rank, nranks) from rank 0's unique id on `device`, plus its
// stream (priority `prio`: 0 = normal, < 0 = higher). min/max_ctas <= 0 keep RCCL's defaults.
// Returns nullptr on failure (ttdc_error(nullptr) says why).
TTDK_EXPORT void* ttdc_create(const char* id_bytes, int nranks, int rank, int device, int prio, int min_ctas,
                              int max_ctas, double timeout_s, int nonblocking) {
  Engine* e = new Engine();
  e->rank = rank;
  e->nranks = nranks;
  e->device = device;
  e->timeout = timeout_s > 0 ? timeout_s : 300.0;
  if (!hip_ok(e, hipSetDevice(device), "hipSetDevice") ||
      !hip_ok(e, hipStreamCreateWithPriority(&e->cs, hipStreamNonBlocking, prio), "hipStreamCreateWithPriority")) {
    g_err = e->err;
    delete e;
    return nullptr;
  }
  for (int i = 0; i < 64; ++i) hipEventCreateWithFlags(&e->fork[i], hipEventDisableTiming);
  hipEventCreateWithFlags(&e->join, hipEventDisableTiming);
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = nonblocking ? 0 : 1;
  if (min_ctas > 0) cfg.minCTAs = min_ctas;
  if (max_ctas > 0) cfg.maxCTAs = max_ctas;
  cfg.commName = "ttd_grad";
  const ncclResult_t r = ncclCommInitRankConfig(&e->comm, nranks, id, rank, &cfg);
  if (!settle(e, r, "ncclCommInitRankConfig")) {
    g_err = e->err;
    if (e->comm) ncclCommAbort(e->comm);
    for (int i = 0; i < 64; ++i) hipEventDestroy(e->fork[i]);
    hipEventDestroy(e->join);
    hipStreamDestroy(e->cs);
    delete e;
    return nullptr;
  }
  return e;
}

TTDK_EXPORT void* ttdc_stream(void* h) { return static_cast<Engine*>(h)->cs; }

namespace ttdk {
namespace {
// The reduction part of a bucket launch (after the fork).
int bucket_body(Engine* e, void* buf, long long count, int dtype, int op, int algo, int compress) {
  if (compress && dtype == 0) {
    const size_t need = static_cast<size_t>(count) * 2;
    if (need > e->stage_bytes) {
      // grow once (first step); the old staging buffer may still be read by queued work
      if (!hip_ok(e, hipStreamSynchronize(e->cs), "hipStreamSynchronize")) return -1;
      if (e->stage) hipFree(e->stage);
      e->stage = nullptr;
      if (!hip_ok(e, hipMalloc(&e->stage, need), "hipMalloc")) return -1;
      e->stage_bytes = need;
    }
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(cast_grid(count)), dim3(256), 0, e->cs, static_cast<const float*>(buf),
                       static_cast<bf16_t*>(e->stage), count);
    if (!reduce_on(e, e->stage, count, ncclBfloat16, 2, to_op(op), algo, e->cs)) return -1;
    hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(cast_grid(count)), dim3(256), 0, e->cs,
                       static_cast<const bf16_t*>(e->stage), static_cast<float*>(buf), count);
    return hip_ok(e, hipGetLastError(), "cast kernel") ? 0 : -1;
  }
  return reduce_on(e, buf, count, to_nccl(dtype), dt_size(dtype), to_op(op), algo, e->cs) ? 0 : -1;
}
}  // namespace
}  // namespace ttdk

// Bucket launch: the communicator stream waits for the work already queued on `producer`,
// then reduces buf[0:count) in place. compress (fp32 buffers only): cast to bf16 on the
// communicator stream, reduce in bf16, cast back.
TTDK_EXPORT int ttdc_bucket(void* h, void* buf, long long count, int dtype, int op, int algo, int compress,
                            hipStream_t producer) {
  Engine* e = static_cast<Engine*>(h);
  if (e->failed) return -1;
  if (count < 0 || algo < 0 || algo > 2) return set_err(e, "ttdc_bucket: bad argument"), -1;
  if (!fork_from(e, producer)) return -1;
  if (e->timing) {
    if (e->n_timed == static_cast<int>(e->t_begin.size())) {
      hipEvent_t a, b;
      if (!hip_ok(e, hipEventCreate(&a), "hipEventCreate") || !hip_ok(e, hipEventCreate(&b), "hipEventCreate")) return -1;
      e->t_begin.push_back(a);
      e->t_end.push_back(b);
    }
    hipEventRecord(e->t_begin[e->n_timed], e->cs);
  }
  const int rc = bucket_body(e, buf, count, dtype, op, algo, compress);
  if (e->timing && rc == 0) hipEventRecord(e->t_end[e->n_timed++], e->cs);
  return rc;
}

// Timing mode on (resets the bucket count) or off.
TTDK_EXPORT void ttdc_set_timing(void* h, int on) {
  Engine* e = static_cast<Engine*>(h);
  e->timing = on != 0;
  e->n_timed = 0;
}

// After ttdc_synchronize: *busy_ms = sum over the timed buckets of their reduction time,
// *span_ms = first bucket start -> last bucket end; returns the number of timed buckets.
TTDK_EXPORT int ttdc_timing(void* h, float* busy_ms, float* span_ms) {
  Engine* e = static_cast<Engine*>(h);
  *busy_ms = *span_ms = 0.f;
  for (int i = 0; i < e->n_timed; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->t_begin[i], e->t_end[i]) != hipSuccess) return -1;
    *busy_ms += ms;
  }
  if (e->n_timed > 0 && hipEventElapsedTime(span_ms, e->t_begin[0], e->t_end[e->n_timed - 1]) != hipSuccess) return -1;
  return e->n_timed;
}


// `consumer` waits for every collective queued so far (no host synchronisation). Also reports
// an asynchronous communicator failure (a peer died / aborted) as an error.
TTDK_EXPORT int ttdc_join(void* h, hipStream_t consumer) {
  Engine* e = static_cast<Engine*>(h);
  if (e->failed) return -1;
  ncclResult_t a = ncclSuccess;
  if (ncclCommGetAsyncError(e->comm, &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress)
    return set_err(e, std::string("communicator failed: ") + ncclGetErrorString(a)), -1;
  if (!hip_ok(e, hipEventRecord(e->join, e->cs), "hipEventRecord") ||
      !hip_ok(e, hipStreamWaitEvent(consumer, e->join, 0), "hipStreamWaitEvent"))
    return -1;
  return 0;
}

// Collective directly on stream `s` (metrics, SyncOnRead means, broadcasts of initial state).
// kind 0: reduce (op, algo 0); 1: broadcast from `root`.
TTDK_EXPORT int ttdc_collective(void* h, int kind, void* buf, long long count, int dtype, int op, int root,
                                hipStream_t s) {
  Engine* e = static_cast<Engine*>(h);
  if (e->failed) return -1;
  if (count <= 0) return 0;
  if (kind == 1)
    return settle(e, ncclBroadcast(buf, buf, count, to_nccl(dtype), root, e->comm, s), "ncclBroadcast") ? 0 : -1;
  return reduce_on(e, buf, count, to_nccl(dtype), dt_size(dtype), to_op(op), 0, s) ? 0 : -1;
}

// Block the host until the communicator stream drained, polling for communicator errors
// against the engine's deadline (a hung peer becomes an error instead of a hang).
TTDK_EXPORT int ttdc_synchronize(void* h) {
  Engine* e = static_cast<Engine*>(h);
  if (e->failed) return -1;
  if (!hip_ok(e, hipEventRecord(e->join, e->cs), "hipEventRecord")) return -1;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(e->join);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return hip_ok(e, q, "hipEventQuery"), -1;
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(e->comm, &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress)
      return set_err(e, std::string("communicator failed: ") + ncclGetErrorString(a)), -1;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > e->timeout)
      return set_err(e, "collectives did not complete before the deadline"), -1;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Bus bandwidth probe: `iters` all-reduces of buf[0:count) (fp32) on the communicator stream,
// timed with HIP events. *ms = mean time per all-reduce.
TTDK_EXPORT int ttdc_probe(void* h, void* buf, long long count, int iters, float* ms) {
  Engine* e = static_cast<Engine*>(h);
  if (e->failed || iters <= 0) return -1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int rc = 0;
  if (!settle(e, ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, e->comm, e->cs), "ncclAllReduce")) rc = -1;
  hipEventRecord(a, e->cs);
  for (int i = 0; rc == 0 && i < iters; ++i)
    if (!settle(e, ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, e->comm, e->cs), "ncclAllReduce")) rc = -1;
  hipEventRecord(b, e->cs);
  if (rc == 0 && ttdc_synchronize(e) == 0) {
    hipEventElapsedTime(ms, a, b);
    *ms /= iters;
  } else {
    rc = -1;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return rc;
}

// Abort (a failed peer: frees the communicator without waiting for the others) or destroy.
TTDK_EXPORT void ttdc_destroy(void* h, int abort) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return;
  if (e->comm) {
    if (abort || e->failed) {
      ncclCommAbort(e->comm);
    } else {
      ncclResult_t r = ncclCommFinalize(e->comm);
      if (settle(e, r, "ncclCommFinalize")) ncclCommDestroy(e->comm);
      else ncclCommAbort(e->comm);
    }
  }
  if (!abort) hipStreamSynchronize(e->cs);
  for (int i = 0; i < 64; ++i) hipEventDestroy(e->fork[i]);
  hipEventDestroy(e->join);
  for (hipEvent_t ev : e->t_begin) hipEventDestroy(ev);
  for (hipEvent_t ev : e->t_end) hipEventDestroy(ev);
  if (e->stage) hipFree(e->stage);
  hipStreamDestroy(e->cs);
  delete e;
}
