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

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "collective_plan.h"
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

long long now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Engine {
  // written only under `wmu` (abort swaps it to null before ncclCommAbort), read lock-free
  std::atomic<ncclComm_t> comm{nullptr};
  hipStream_t cs = nullptr;  // communicator stream
  int rank = 0, nranks = 1, device = 0;
  double timeout = 300.0;
  hipEvent_t fork[64];      // producer -> communicator stream (ring of events)
  int fork_next = 0;
  hipEvent_t join = nullptr;
  void* stage = nullptr;    // bf16 staging for compressed buckets
  size_t stage_bytes = 0;
  std::atomic<bool> failed{false};
  std::string err;
  // per-bucket timing (ttdc_set_timing): events around each bucket's reduction on the
  // communicator stream, recorded after its fork wait is satisfied
  bool timing = false;
  std::vector<hipEvent_t> t_begin, t_end;
  int n_timed = 0;
  // ---- watchdog: every join (outside stream capture) and every ttdc_arm (after a graph replay)
  // records a marker event on the communicator stream; a thread polls the oldest marker and
  // the communicator's asynchronous error. A marker older than `timeout` (a peer that died
  // mid-step leaves RCCL's kernels spinning and the compute stream waiting on the join), an
  // asynchronous error, or a host call blocked inside RCCL for longer than `timeout` (a dead
  // peer during RCCL's lazy connection setup) aborts the communicator: RCCL's kernels exit, the
  // streams drain, and the next bucket / join call returns an error the recoverable session
  // acts on (parallel/strategy.py recover()).
  // Locks: `mu` serialises the host threads' calls into RCCL and is held across them (a
  // blocking enqueue can block); the watchdog never waits for it. It takes `mu` only with
  // try_lock (nobody is between loading `comm` and calling RCCL: aborting is safe), and once a
  // call has held `mu` for longer than `timeout` it aborts without it (that caller is stuck
  // inside RCCL, which ncclCommAbort from another thread releases). `wmu` guards the watchdog's
  // own state (`pend`, `pool`, `stop`) and the comm swap.
  std::mutex mu;
  std::mutex wmu;
  std::atomic<long long> busy_ns{0};  // steady-clock start of the call holding `mu` (0 = none)
  std::condition_variable cv;
  bool stop = false;
  std::thread wd;
  struct Mark {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t;
  };
  std::deque<Mark> pend;
  std::vector<hipEvent_t> pool;
  std::vector<void*> retired;  // outgrown staging buffers, freed once the stream drained (under wmu)
  std::atomic<int> aborts{0};
};

// A host call into the engine: holds `mu` and publishes how long it has been inside.
struct Call {
  Engine* e;
  std::lock_guard<std::mutex> lk;
  explicit Call(Engine* en) : e(en), lk(en->mu) { e->busy_ns = now_ns(); }
  ~Call() { e->busy_ns = 0; }
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
    ncclResult_t a = ncclSuccess, q = ncclSuccess;
    {
      // under wmu: an abort (which swaps `comm` out under wmu before ncclCommAbort frees it)
      // cannot free the handle between this load and the query
      std::lock_guard<std::mutex> g(e->wmu);
      ncclComm_t c = e->comm.load();
      if (!c) return set_err(e, std::string(what) + ": communicator aborted");
      q = ncclCommGetAsyncError(c, &a);
    }
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
    std::string last;
    {
      std::lock_guard<std::mutex> g(e->wmu);
      ncclComm_t c = e->comm.load();
      const char* l = c ? ncclGetLastError(c) : "";
      if (l) last = l;
    }
    return set_err(e, std::string(what) + ": " + ncclGetErrorString(r) + (!last.empty() ? " (" + last + ")" : ""));
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
  ttd_coll::Step plan[ttd_coll::kMaxSteps];
  const int n = ttd_coll::plan(algo, static_cast<long long>(count), e->nranks, e->rank, plan);
  if (n < 0) return set_err(e, "collective plan: bad argument");
  char* p = static_cast<char*>(buf);
  for (int i = 0; i < n; ++i) {
    // reloaded per enqueue: a deadline abort between two steps leaves null, never a freed handle
    ncclComm_t comm = e->comm.load();
    if (!comm) return set_err(e, "communicator aborted");
    const ttd_coll::Step& st = plan[i];
    char* a = p + st.send * esz;
    char* b = p + st.recv * esz;
    const size_t c = static_cast<size_t>(st.count);
    bool ok = true;
    switch (st.kind) {
      case ttd_coll::kAllReduce: ok = settle(e, ncclAllReduce(a, a, c, dt, op, comm, s), "ncclAllReduce"); break;
      case ttd_coll::kReduceScatter:
        ok = settle(e, ncclReduceScatter(a, b, c, dt, op, comm, s), "ncclReduceScatter");
        break;
      case ttd_coll::kAllGather: ok = settle(e, ncclAllGather(a, b, c, dt, comm, s), "ncclAllGather"); break;
      case ttd_coll::kReduce: ok = settle(e, ncclReduce(a, a, c, dt, op, st.root, comm, s), "ncclReduce"); break;
      case ttd_coll::kBroadcast: ok = settle(e, ncclBroadcast(a, a, c, dt, st.root, comm, s), "ncclBroadcast"); break;
      default: ok = set_err(e, "collective plan: unknown step");
    }
    if (!ok) return false;
  }
  return true;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Abort the communicator: detach it (every later call sees the failure at once), then
// ncclCommAbort outside every lock (it can wait for queued work). Exactly one caller wins.
void abort_comm(Engine* e, const std::string& why) {
  ncclComm_t c;
  {
    std::lock_guard<std::mutex> g(e->wmu);
    c = e->comm.exchange(nullptr);
    if (!c) return;
    set_err(e, why);
    e->aborts.fetch_add(1);
  }
  ncclCommAbort(c);
}

// Why the communicator should be aborted now ("" = healthy). Caller holds wmu.
std::string health(Engine* e) {
  ncclComm_t c = e->comm.load();
  if (!c) return "";
  ncclResult_t a = ncclSuccess;
  if (ncclCommGetAsyncError(c, &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress)
    return std::string("communicator failed: ") + ncclGetErrorString(a);
  if (!e->pend.empty()) {
    const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() - e->pend.front().t).count();
    if (age > e->timeout) {
      char b[160];
      snprintf(b, sizeof b, "collectives made no progress for %.0f s (a peer died or hung): communicator aborted", age);
      return b;
    }
  }
  return "";
}

void watchdog(Engine* e) {
  hipSetDevice(e->device);
  std::unique_lock<std::mutex> wl(e->wmu);
  while (!e->stop) {
    e->cv.wait_for(wl, std::chrono::milliseconds(e->pend.empty() ? 50 : 2));
    if (e->stop) break;
    while (!e->pend.empty() && hipEventQuery(e->pend.front().ev) == hipSuccess) {
      e->pool.push_back(e->pend.front().ev);
      e->pend.pop_front();
    }
    if (!e->comm.load()) continue;
    std::string why = health(e);
    const long long b = e->busy_ns.load();
    const double busy = b ? (now_ns() - b) * 1e-9 : 0.0;
    if (why.empty() && busy > e->timeout) {
      char m[160];
      snprintf(m, sizeof m, "a collective call blocked for %.0f s (a peer died or hung): communicator aborted", busy);
      why = m;
    }
    if (why.empty()) continue;
    wl.unlock();
    if (busy > e->timeout) {
      abort_comm(e, why);  // the caller holding `mu` is stuck inside RCCL
    } else if (e->mu.try_lock()) {
      abort_comm(e, why);  // no call in flight
      e->mu.unlock();
    }  // else: a call is in flight; retry on the next tick (bounded by the busy deadline)
    wl.lock();
  }
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
// Starts the watchdog thread. Returns nullptr on failure (ttdc_error(nullptr) says why).
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
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRankConfig(&c, nranks, id, rank, &cfg);
  e->comm = c;
  if (!settle(e, r, "ncclCommInitRankConfig")) {
    g_err = e->err;
    if (c) ncclCommAbort(c);
    for (int i = 0; i < 64; ++i) hipEventDestroy(e->fork[i]);
    hipEventDestroy(e->join);
    hipStreamDestroy(e->cs);
    delete e;
    return nullptr;
  }
  e->wd = std::thread(watchdog, e);
  return e;
}

TTDK_EXPORT void* ttdc_stream(void* h) { return static_cast<Engine*>(h)->cs; }

namespace ttdk {
namespace {
bool grow_stage(Engine* e, size_t need) {
  if (need <= e->stage_bytes) return true;
  // the old staging buffer may still be read by queued work: retire it (freed once the stream
  // drained, ttdc_synchronize / ttdc_destroy) instead of synchronising under `mu`
  if (e->stage) {
    std::lock_guard<std::mutex> g(e->wmu);
    e->retired.push_back(e->stage);
  }
  e->stage = nullptr;
  e->stage_bytes = 0;
  if (!hip_ok(e, hipMalloc(&e->stage, need), "hipMalloc")) return false;
  e->stage_bytes = need;
  return true;
}

// The reduction part of a bucket launch (after the fork). Caller holds e->mu.
int bucket_body(Engine* e, void* buf, long long count, int dtype, int op, int algo, int compress) {
  if (compress && dtype == 0) {
    const size_t need = static_cast<size_t>(count) * 2;
    if (need > e->stage_bytes) {
      // growing needs a stream synchronize + hipMalloc, both illegal under hipGraph capture:
      // the reducer reserves its largest bucket up front (ttdc_reserve)
      if (capturing(e->cs)) return set_err(e, "bf16 staging buffer too small under stream capture"), -1;
      if (!grow_stage(e, need)) return -1;
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

// Fault injection for the watchdog test: holds the communicator stream until *flag != 0 or
// max_ms of wall clock passed (every wave exits by itself: no host action can leave it running).
__global__ void stall_kernel(const volatile int* flag, unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (*flag == 0 && wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(100);
}
// Stand-in for one RCCL bucket kernel (tools/comm_interference.py): `ctas` workgroups of 256
// threads with a 16 KB LDS footprint, each streaming read-modify-write over its share of `buf`
// (the copy / reduce traffic of a ring step) for `ticks` of wall clock from its own start.
__global__ __launch_bounds__(256) void comm_emulate_kernel(uint4* buf, long long n16, unsigned long long ticks) {
  __shared__ uint4 lds[1024];
  const unsigned long long t0 = wall_clock64();
  const long long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long long lo = per * blockIdx.x, hi = lo + per < n16 ? lo + per : n16;
  long long i = lo + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  while (wall_clock64() - t0 < ticks) {
    if (i >= hi) i = lo + threadIdx.x;
    if (i < hi) {
      uint4 v = buf[i];
      lds[threadIdx.x] = v;
      acc.x ^= v.x;
      buf[i] = v;
      i += blockDim.x;
    }
  }
  if (acc.x == 0x12345678u && threadIdx.x == 0) lds[1023] = acc;  // keep the loop's loads
}
}  // namespace
}  // namespace ttdk

// Interference harness: queue one emulated bucket all-reduce (comm_emulate_kernel) of `us`
// microseconds on `stream`.
TTDK_EXPORT int ttdc_emulate_bucket(hipStream_t stream, int ctas, double us, void* buf, long long nbytes) {
  int dev = 0, rate_khz = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
    rate_khz = 100000;
  const unsigned long long ticks = static_cast<unsigned long long>(us * rate_khz / 1000.0);
  hipLaunchKernelGGL(comm_emulate_kernel, dim3(ctas > 0 ? ctas : 1), dim3(256), 0, stream, static_cast<uint4*>(buf),
                     nbytes / 16, ticks);
  return hipGetLastError();
}

// Pre-size the bf16 staging buffer of compressed buckets for buckets of up to `count` fp32
// elements (call once before any step is captured).
TTDK_EXPORT int ttdc_reserve(void* h, long long count) {
  Engine* e = static_cast<Engine*>(h);
  Call call(e);
  if (e->failed) return -1;
  return grow_stage(e, static_cast<size_t>(count) * 2) ? 0 : -1;
}

// Bucket launch: the communicator stream waits for the work already queued on `producer`,
// then reduces buf[0:count) in place. compress (fp32 buffers only): cast to bf16 on the
// communicator stream, reduce in bf16, cast back.
namespace ttdk {
namespace {
int bucket_launch(Engine* e, void* buf, long long count, int dtype, int op, int algo, int compress, bool fork,
                  hipStream_t producer) {
  Call call(e);
  if (e->failed || !e->comm.load()) return -1;
  if (count < 0 || algo < 0 || algo > 2) return set_err(e, "ttdc_bucket: bad argument"), -1;
  if (fork && !fork_from(e, producer)) return -1;
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
}  // namespace
}  // namespace ttdk

TTDK_EXPORT int ttdc_bucket(void* h, void* buf, long long count, int dtype, int op, int algo, int compress,
                            hipStream_t producer) {
  return bucket_launch(static_cast<Engine*>(h), buf, count, dtype, op, algo, compress, true, producer);
}

// ttdc_bucket without the fork: the caller already ordered the communicator stream (an event
// node pair of a segmented hipGraph capture, utils/graphs.py).
TTDK_EXPORT int ttdc_bucket_nofork(void* h, void* buf, long long count, int dtype, int op, int algo, int compress) {
  return bucket_launch(static_cast<Engine*>(h), buf, count, dtype, op, algo, compress, false, nullptr);
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


// `consumer` waits for every collective queued so far (no host synchronisation). Reports a
// failure the watchdog detected (asynchronous communicator error, or no progress before the
// deadline) as an error, and arms the watchdog with a marker after the queued collectives
// (not under stream capture: a captured record never completes on its own).
namespace ttdk {
namespace {
// Arm the watchdog: a pooled marker event recorded on `s` after the work queued so far.
void arm(Engine* e, hipStream_t s) {
  std::lock_guard<std::mutex> g(e->wmu);
  hipEvent_t ev = nullptr;
  if (!e->pool.empty()) {
    ev = e->pool.back();
    e->pool.pop_back();
  } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    return;
  }
  if (hipEventRecord(ev, s) == hipSuccess) {
    e->pend.push_back(Engine::Mark{ev, std::chrono::steady_clock::now()});
    e->cv.notify_one();
  } else {
    e->pool.push_back(ev);
  }
}
}  // namespace
}  // namespace ttdk

TTDK_EXPORT int ttdc_join(void* h, hipStream_t consumer) {
  Engine* e = static_cast<Engine*>(h);
  Call call(e);
  ncclComm_t c = e->comm.load();
  if (e->failed || !c) return -1;
  ncclResult_t a = ncclSuccess;
  if (ncclCommGetAsyncError(c, &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress)
    return set_err(e, std::string("communicator failed: ") + ncclGetErrorString(a)), -1;
  if (!hip_ok(e, hipEventRecord(e->join, e->cs), "hipEventRecord") ||
      !hip_ok(e, hipStreamWaitEvent(consumer, e->join, 0), "hipStreamWaitEvent"))
    return -1;
  if (!capturing(e->cs) && !capturing(consumer)) arm(e, e->cs);
  return 0;
}

// Arm the watchdog after a hipGraph replay: a captured join records no marker (a captured
// record never completes on its own), so the replaying thread calls this with the replay stream
// once per replay and a step whose collectives never finish still trips the deadline.
TTDK_EXPORT int ttdc_arm(void* h, hipStream_t s) {
  Engine* e = static_cast<Engine*>(h);
  if (e->failed || !e->comm.load()) return -1;
  if (capturing(s)) return set_err(e, "ttdc_arm: stream is capturing"), -1;
  arm(e, s);
  return 0;
}

// Collective directly on stream `s` (metrics, SyncOnRead means, broadcasts of initial state).
// kind 0: reduce (op, algo 0); 1: broadcast from `root`.
TTDK_EXPORT int ttdc_collective(void* h, int kind, void* buf, long long count, int dtype, int op, int root,
                                hipStream_t s) {
  Engine* e = static_cast<Engine*>(h);
  Call call(e);
  ncclComm_t c = e->comm.load();
  if (e->failed || !c) return -1;
  if (count <= 0) return 0;
  if (kind == 1)
    return settle(e, ncclBroadcast(buf, buf, count, to_nccl(dtype), root, c, s), "ncclBroadcast") ? 0 : -1;
  return reduce_on(e, buf, count, to_nccl(dtype), dt_size(dtype), to_op(op), 0, s) ? 0 : -1;
}

// Block the host until the communicator stream drained, polling for communicator errors
// against the engine's deadline (a hung peer becomes an error instead of a hang).
TTDK_EXPORT int ttdc_synchronize(void* h) {
  Engine* e = static_cast<Engine*>(h);
  hipEvent_t done = nullptr;
  std::vector<void*> retired;
  {
    Call call(e);
    if (e->failed || !e->comm.load()) return -1;
    if (!hip_ok(e, hipEventRecord(e->join, e->cs), "hipEventRecord")) return -1;
    done = e->join;
    std::lock_guard<std::mutex> g(e->wmu);
    retired.swap(e->retired);  // queued before this record: free once it completed
  }
  // error returns hand the staging buffers back (ttdc_destroy frees them): recovery — abort,
  // then recreate — is exactly when this path runs, so dropping them leaked device memory
  auto keep_retired = [&] {
    std::lock_guard<std::mutex> g(e->wmu);
    e->retired.insert(e->retired.end(), retired.begin(), retired.end());
    retired.clear();
  };
  // abort from this thread only when no other host call is inside RCCL with the handle (the
  // watchdog aborts a call stuck past the busy deadline); otherwise mark the failure and leave
  // the abort to the watchdog
  auto fail_abort = [&](const std::string& why) {
    keep_retired();
    if (e->mu.try_lock()) {
      abort_comm(e, why);
      e->mu.unlock();
    } else {
      std::lock_guard<std::mutex> g(e->wmu);
      set_err(e, why);
    }
    return -1;
  };
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(done);
    if (q == hipSuccess) {
      for (void* p : retired) hipFree(p);
      return e->failed ? -1 : 0;
    }
    if (q != hipErrorNotReady) return keep_retired(), hip_ok(e, q, "hipEventQuery"), -1;
    // no `mu` here: the watchdog and other threads' calls proceed while this host waits
    if (e->failed) return keep_retired(), -1;  // the watchdog aborted the communicator
    ncclComm_t c = e->comm.load();
    ncclResult_t a = ncclSuccess;
    {
      std::lock_guard<std::mutex> g(e->wmu);  // the comm cannot be swapped out under wmu
      c = e->comm.load();
      if (c && ncclCommGetAsyncError(c, &a) != ncclSuccess) a = ncclSuccess;
    }
    if (c && a != ncclSuccess && a != ncclInProgress)
      return fail_abort(std::string("communicator failed: ") + ncclGetErrorString(a));
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > e->timeout)
      return fail_abort("collectives did not complete before the deadline: communicator aborted");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Number of times the watchdog / a deadline aborted this communicator (0 or 1).
TTDK_EXPORT int ttdc_aborts(void* h) { return static_cast<Engine*>(h)->aborts.load(); }

// Fault injection (tests): queue a kernel on the communicator stream that holds it until
// *flag (device-visible host memory) becomes non-zero or max_ms passed.
TTDK_EXPORT int ttdc_debug_stall(void* h, const int* flag, int max_ms) {
  Engine* e = static_cast<Engine*>(h);
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, e->device) != hipSuccess || rate_khz <= 0)
    rate_khz = 100000;
  const unsigned long long ticks = static_cast<unsigned long long>(rate_khz) * static_cast<unsigned long long>(max_ms);
  Call call(e);
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, e->cs, flag, ticks);
  return hip_ok(e, hipGetLastError(), "stall kernel") ? 0 : -1;
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
  {
    Call call(e);
    // the handle is reloaded per enqueue (a deadline abort leaves null, never a freed handle)
    auto once = [&] {
      ncclComm_t c = e->comm.load();
      if (!c) return set_err(e, "communicator aborted");
      return settle(e, ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c, e->cs), "ncclAllReduce");
    };
    if (!once()) rc = -1;
    hipEventRecord(a, e->cs);
    for (int i = 0; rc == 0 && i < iters; ++i)
      if (!once()) rc = -1;
    hipEventRecord(b, e->cs);
  }
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
  {
    std::lock_guard<std::mutex> g(e->wmu);
    e->stop = true;
  }
  e->cv.notify_all();
  if (e->wd.joinable()) e->wd.join();
  ncclComm_t c = e->comm.exchange(nullptr);
  if (c) {
    if (abort || e->failed) {
      ncclCommAbort(c);
    } else {
      e->comm = c;  // settle polls it while a non-blocking finalize completes
      ncclResult_t r = ncclCommFinalize(c);
      const bool fin = settle(e, r, "ncclCommFinalize");
      e->comm = nullptr;
      if (fin) ncclCommDestroy(c);
      else ncclCommAbort(c);
    }
  }
  if (!abort) hipStreamSynchronize(e->cs);
  for (void* p : e->retired) hipFree(p);
  for (int i = 0; i < 64; ++i) hipEventDestroy(e->fork[i]);
  hipEventDestroy(e->join);
  for (hipEvent_t ev : e->t_begin) hipEventDestroy(ev);
  for (hipEvent_t ev : e->t_end) hipEventDestroy(ev);
  for (auto& m : e->pend) hipEventDestroy(m.ev);
  for (hipEvent_t ev : e->pool) hipEventDestroy(ev);
  if (e->stage) hipFree(e->stage);
  hipStreamDestroy(e->cs);
  delete e;
}
