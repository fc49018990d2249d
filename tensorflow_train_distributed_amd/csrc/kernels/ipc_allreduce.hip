// Direct xGMI all-reduce for small gradient buckets: one-shot / two-shot reductions over staging
// buffers that every rank maps from every peer (hipIpcGetMemHandle / hipIpcOpenMemHandle), with
// a flag barrier per workgroup. Plan (path choice, chunk / part arithmetic): ipc_plan.h.
// Reference aggregation it serves: the gradient all-reduce of the Mirrored strategies
// (BASELINE.json north star; the reference's own PS accumulators are at
// /root/reference/distribute_training.py:142-148).
//
// Per rank: a data buffer [2 slots][2 regions (in, out)][cap bytes] and a flag array
// [2 slots][2 phases][kMaxBlocks][kMaxRanks] of u32, both mapped into every peer. A call:
//   epoch ep = device counter + 1 (the last workgroup of the previous call on this stream
//   advanced it: graph replays see fresh epochs), slot = ep & 1 (a slot is reused only two
//   calls later, after every peer has passed the next call's barrier, so no peer still reads it);
//   stage: workgroup b copies its part of the bucket into this rank's in-region;
//   barrier(phase 0, b): release, store ep into flags[slot][0][b][rank] of every peer, spin until
//   every peer's ep is in this rank's flags[slot][0][b][*], acquire;
//   one-shot: sum part b over the peers' in-regions into the bucket;
//   two-shot: sum part b of chunk `rank` over the peers' in-regions (into the bucket and this
//   rank's out-region), barrier(phase 1, b), copy part b of every other chunk q from peer q's
//   out-region.
// Spins are bounded (~1-2 s by default): a peer that never arrives sets the engine's error word
// and the kernel completes instead of a wave that never finishes. A workgroup whose barrier timed
// out (or that starts after an earlier call failed) does NOT sum: it overwrites its share of the
// bucket with NaN, so a late peer can never turn into a silently wrong gradient. The error word
// lives in host-mapped memory: the reducer reads it at its join points without a device sync
// (BucketedAllReducer.begin / finish raise UnavailableError into the session's recovery).
#include <cstring>

#include "common.h"
#include "ipc_plan.h"

namespace ttdk {
namespace {

using ttd_ipc::kMaxBlocks;
using ttd_ipc::kMaxRanks;

constexpr int kThreads = 512;
constexpr long long kSpinDefault = 1LL << 24;  // x s_sleep 2 (~128 cycles) + the poll: ~1-2 s (a
                                               // fresh process loads its code objects lazily)

struct Peers {
  char* data[kMaxRanks];
  unsigned* flags[kMaxRanks];
};

__device__ __forceinline__ int flag_idx(int slot, int phase, int b, int src) {
  return ((slot * 2 + phase) * kMaxBlocks + b) * kMaxRanks + src;
}
// after the barrier flags: the abort word. A rank whose barrier timed out sets it on EVERY rank,
// so the group fails together — a peer that was merely late (or skipped a call and would now
// pair its epochs with the wrong call) poisons its next launch instead of summing
constexpr int kAbortIdx = 2 * 2 * kMaxBlocks * kMaxRanks;

// Flag barrier of workgroup b; returns false (for the whole workgroup) when some peer did not
// arrive within spin_max polls or `*fail` was already set (an earlier call / phase failed).
__device__ __forceinline__ bool barrier(const Peers& P, int slot, int phase, int rank, int world, unsigned ep,
                                        int* err, long long spin_max, int* fail) {
  // every thread's stores of this workgroup are complete and visible system-wide before any
  // peer can see the flag
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  const int b = blockIdx.x, t = threadIdx.x;
  volatile int* vf = fail;
  // a failed workgroup does not publish its flag: what it staged (two-shot: its out-region part)
  // is not valid, so its peers must time out and poison this block too, not read it
  if (t < world && !*vf) {
    __hip_atomic_store(P.flags[t] + flag_idx(slot, phase, b, rank), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mine = P.flags[rank] + flag_idx(slot, phase, b, t);
    long long it = 0;
    while (!*vf && __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != ep) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > spin_max) {
        *vf = 1;  // LDS: the workgroup skips its sum
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int p = 0; p < world; ++p)
          __hip_atomic_store(P.flags[p] + kAbortIdx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the peers' data, not a stale cached copy
  return !*vf;
}

template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void add(float (&acc)[8], const uint4& v) {
    acc[0] += __uint_as_float(v.x);
    acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z);
    acc[3] += __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float (&acc)[8]) {
    return make_uint4(__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]),
                      __float_as_uint(acc[3]));
  }
};
template <>
struct Vec<bf16_t> {
  static constexpr int N = 8;
  __device__ static void add(float (&acc)[8], const uint4& v) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += f[i];
  }
  __device__ static uint4 pack(const float (&acc)[8]) { return pack8(acc); }
};

// dst[i] = sum over peers p of src_p[i] for the 16-B vectors of [lo, hi) (element offsets), peers
// summed in rank order (every rank gets the same bits); also into out2 when non-null
template <typename T>
__device__ void sum_range(const Peers& P, int world, long long region_off, long long lo, long long hi, T* dst,
                          T* out2) {
  constexpr int V = Vec<T>::N;
  for (long long v = lo / V + threadIdx.x; v < hi / V; v += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      const uint4* s = reinterpret_cast<const uint4*>(P.data[p] + region_off) + v;
      Vec<T>::add(acc, *s);
    }
    const uint4 r = Vec<T>::pack(acc);
    reinterpret_cast<uint4*>(dst)[v] = r;
    if (out2) reinterpret_cast<uint4*>(out2)[v] = r;
  }
}

template <typename T>
__device__ void copy_range(const uint4* src, uint4* dst, long long lo, long long hi) {
  constexpr int V = Vec<T>::N;
  for (long long v = lo / V + threadIdx.x; v < hi / V; v += kThreads) dst[v] = src[v];
}

// quiet NaN over the 16-B vectors of [lo, hi): the share of a workgroup that could not reduce
template <typename T>
__device__ void poison_range(T* dst, long long lo, long long hi) {
  constexpr int V = Vec<T>::N;
  const unsigned q = sizeof(T) == 4 ? 0x7FC00000u : 0x7FC07FC0u;
  const uint4 nan4 = make_uint4(q, q, q, q);
  for (long long v = lo / V + threadIdx.x; v < hi / V; v += kThreads) reinterpret_cast<uint4*>(dst)[v] = nan4;
}

// count: elements, a multiple of Vec<T>::N (the host rounds the staged range up and handles the
// tail through the padded staging buffer). ctr[0] = epoch, ctr[1] = finished workgroups.
template <typename T, int PATH>
__global__ __launch_bounds__(kThreads) void ipc_allreduce_kernel(Peers P, T* __restrict__ buf, long long count,
                                                                 int rank, int world, long long cap,
                                                                 unsigned* __restrict__ ctr, int* __restrict__ err,
                                                                 long long spin_max) {
  constexpr int V = Vec<T>::N;
  __shared__ int fail;
  if (threadIdx.x == 0) {
    // an earlier call failed here or on a peer: this engine is dead until the host recovers
    // (no barrier waits; the host sees the error word)
    const bool aborted =
        __hip_atomic_load(P.flags[rank] + kAbortIdx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    if (aborted) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    fail = aborted || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  }
  const unsigned ep = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const int slot = ep & 1, nb = gridDim.x, b = blockIdx.x;
  const long long in_off = static_cast<long long>(slot) * 2 * cap, out_off = in_off + cap;
  T* const my_in = reinterpret_cast<T*>(P.data[rank] + in_off);
  long long lo, hi;
  if constexpr (PATH == ttd_ipc::kOneShot) {
    // stage part b of the whole bucket; after barrier b every peer's part b is staged
    ttd_ipc::part(0, count, V, nb, b, &lo, &hi);
    copy_range<T>(reinterpret_cast<const uint4*>(buf), reinterpret_cast<uint4*>(my_in), lo, hi);
    if (barrier(P, slot, 0, rank, world, ep, err, spin_max, &fail))
      sum_range<T>(P, world, in_off, lo, hi, buf, static_cast<T*>(nullptr));
    else
      poison_range<T>(buf, lo, hi);
  } else {
    // stage part b of EVERY chunk: after barrier b, part b of the chunk this rank reduces is
    // staged on every peer
    for (int q = 0; q < world; ++q) {
      long long qlo, qhi;
      ttd_ipc::chunk(count, V, world, q, &qlo, &qhi);
      ttd_ipc::part(qlo, qhi, V, nb, b, &lo, &hi);
      copy_range<T>(reinterpret_cast<const uint4*>(buf), reinterpret_cast<uint4*>(my_in), lo, hi);
    }
    // reduce-scatter: part b of this rank's chunk, from every peer's in-region
    long long clo, chi, plo, phi;
    ttd_ipc::chunk(count, V, world, rank, &clo, &chi);
    ttd_ipc::part(clo, chi, V, nb, b, &plo, &phi);
    bool ok = barrier(P, slot, 0, rank, world, ep, err, spin_max, &fail);
    if (ok) sum_range<T>(P, world, in_off, plo, phi, buf, reinterpret_cast<T*>(P.data[rank] + out_off));
    // (a workgroup that failed phase 0 does not publish phase 1: its peers time out there and
    // poison block b as well, so nobody copies the out-region part it never wrote)
    ok = barrier(P, slot, 1, rank, world, ep, err, spin_max, &fail) && ok;
    // all-gather: part b of chunk q from peer q's out-region (or NaN: part b of every chunk)
    for (int q = 0; q < world; ++q) {
      ttd_ipc::chunk(count, V, world, q, &clo, &chi);
      ttd_ipc::part(clo, chi, V, nb, b, &plo, &phi);
      if (!ok) poison_range<T>(buf, plo, phi);
      else if (q != rank)
        copy_range<T>(reinterpret_cast<const uint4*>(P.data[q] + out_off), reinterpret_cast<uint4*>(buf), plo, phi);
    }
  }
  // the last workgroup advances the epoch for the next call on this stream
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == static_cast<unsigned>(nb - 1)) {
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct IpcEngine {
  int rank = 0, world = 1, device = 0;
  long long cap = 0;  // bytes per region
  char* data = nullptr;
  unsigned* flags = nullptr;
  unsigned* ctr = nullptr;  // [epoch, finished workgroups]
  int* err = nullptr;       // host-mapped (hipHostMalloc): the host reads it without a sync
  long long spin_max = kSpinDefault;
  Peers peers{};
  bool opened[kMaxRanks] = {};
};

constexpr size_t kFlagBytes = sizeof(unsigned) * (kAbortIdx + 64);  // flags + abort word (+ pad)
constexpr int kHandleBytes = 64;  // sizeof(hipIpcMemHandle_t)

}  // namespace
}  // namespace ttdk

using ttdk::IpcEngine;

// Staging buffers of `cap_bytes` per region on `device` (4 regions) + flags. spin_max: barrier
// polls before a peer counts as lost (<= 0: the default, ~1-2 s). Returns null on failure.
TTDK_EXPORT void* ttdi_create(int rank, int world, int device, long long cap_bytes, long long spin_max) {
  static_assert(sizeof(hipIpcMemHandle_t) == ttdk::kHandleBytes, "IPC handle size");
  if (world < 1 || world > ttdk::kMaxRanks || rank < 0 || rank >= world || cap_bytes <= 0) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  auto* e = new IpcEngine();
  e->rank = rank;
  e->world = world;
  e->device = device;
  e->cap = (cap_bytes + 4095) / 4096 * 4096;
  if (spin_max > 0) e->spin_max = spin_max;
  // the flag words are polled across xGMI by the peers: uncached device memory (no stale line in
  // any L2 between a peer's store and this rank's poll), fine-grained as the fallback
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&e->flags), ttdk::kFlagBytes, hipDeviceMallocUncached) !=
      hipSuccess) {
    (void)hipGetLastError();
    e->flags = nullptr;
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&e->flags), ttdk::kFlagBytes, hipDeviceMallocFinegrained) !=
        hipSuccess) {
      (void)hipGetLastError();
      e->flags = nullptr;
    }
  }
  if (hipMalloc(&e->data, 4 * e->cap) != hipSuccess ||
      (!e->flags && hipMalloc(&e->flags, ttdk::kFlagBytes) != hipSuccess) ||
      hipMalloc(&e->ctr, 2 * sizeof(unsigned)) != hipSuccess ||
      hipHostMalloc(&e->err, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipMemset(e->flags, 0, ttdk::kFlagBytes) != hipSuccess || hipMemset(e->ctr, 0, 2 * sizeof(unsigned)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    if (e->data) (void)hipFree(e->data);
    if (e->flags) (void)hipFree(e->flags);
    if (e->ctr) (void)hipFree(e->ctr);
    if (e->err) (void)hipHostFree(e->err);
    delete e;
    return nullptr;
  }
  *reinterpret_cast<volatile int*>(e->err) = 0;
  e->peers.data[rank] = e->data;
  e->peers.flags[rank] = e->flags;
  return e;
}

// This rank's IPC handles: out[0:64] data, out[64:128] flags.
TTDK_EXPORT int ttdi_handle(void* h, char* out) {
  auto* e = static_cast<IpcEngine*>(h);
  hipIpcMemHandle_t a, f;
  hipError_t rc = hipIpcGetMemHandle(&a, e->data);
  if (rc != hipSuccess) return rc;
  rc = hipIpcGetMemHandle(&f, e->flags);
  if (rc != hipSuccess) return rc;
  std::memcpy(out, &a, ttdk::kHandleBytes);
  std::memcpy(out + ttdk::kHandleBytes, &f, ttdk::kHandleBytes);
  return hipSuccess;
}

// Map every peer: handles = world x 128 bytes (ttdi_handle of each rank, rank order), devices =
// each rank's device ordinal (peer access is enabled for the other devices of this node).
TTDK_EXPORT int ttdi_open(void* h, const char* handles, const int* devices) {
  auto* e = static_cast<IpcEngine*>(h);
  if (hipSetDevice(e->device) != hipSuccess) return hipErrorInvalidDevice;
  for (int p = 0; p < e->world; ++p) {
    if (p == e->rank) continue;
    if (devices[p] != e->device) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, e->device, devices[p]) == hipSuccess && can) {
        const hipError_t pe = hipDeviceEnablePeerAccess(devices[p], 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) return pe;
        (void)hipGetLastError();
      }
    }
    hipIpcMemHandle_t a, f;
    std::memcpy(&a, handles + p * 2 * ttdk::kHandleBytes, ttdk::kHandleBytes);
    std::memcpy(&f, handles + p * 2 * ttdk::kHandleBytes + ttdk::kHandleBytes, ttdk::kHandleBytes);
    void* pd = nullptr;
    void* pf = nullptr;
    hipError_t rc = hipIpcOpenMemHandle(&pd, a, hipIpcMemLazyEnablePeerAccess);
    if (rc != hipSuccess) return rc;
    rc = hipIpcOpenMemHandle(&pf, f, hipIpcMemLazyEnablePeerAccess);
    if (rc != hipSuccess) {
      (void)hipIpcCloseMemHandle(pd);
      return rc;
    }
    e->peers.data[p] = static_cast<char*>(pd);
    e->peers.flags[p] = static_cast<unsigned*>(pf);
    e->opened[p] = true;
  }
  return hipSuccess;
}

// Test helper: make engine `other` (another rank's engine in THIS process, same device) a peer
// of `h` without IPC — one process can then run every rank of a small group on one GPU (each
// rank's kernel on its own stream) to check the barriers and the two-shot exchange.
TTDK_EXPORT int ttdi_link_local(void* h, void* other) {
  auto* e = static_cast<IpcEngine*>(h);
  auto* o = static_cast<IpcEngine*>(other);
  if (o->world != e->world || o->rank == e->rank || o->device != e->device) return hipErrorInvalidValue;
  e->peers.data[o->rank] = o->data;
  e->peers.flags[o->rank] = o->flags;
  return hipSuccess;
}

// In-place SUM all-reduce of `count` elements (dtype 0 fp32, 1 bf16) at `buf` on `st` through
// `path` (ttd_ipc::kOneShot / kTwoShot) with at most `max_blocks` workgroups (the collectives' CTA
// budget; <= 0: ttd_ipc::kMaxBlocks). Every rank must call with the same count / path /
// max_blocks in the same order. The bucket is processed in whole 16-B vectors (count % (16 B /
// element) == 0, 16-B aligned).
TTDK_EXPORT int ttdi_allreduce(void* h, void* buf, long long count, int dtype, int path, int max_blocks,
                               hipStream_t st) {
  auto* e = static_cast<IpcEngine*>(h);
  const int esz = dtype == 0 ? 4 : 2, vec = 16 / esz;
  const long long bytes = count * esz;
  if ((path != ttd_ipc::kOneShot && path != ttd_ipc::kTwoShot) || count <= 0 || bytes > e->cap ||
      (reinterpret_cast<uintptr_t>(buf) & 15) || count % vec)
    return hipErrorInvalidValue;
  for (int p = 0; p < e->world; ++p)
    if (!e->peers.data[p]) return hipErrorNotReady;  // ttdi_open not called
  const int nb = ttd_ipc::blocks_for(bytes, max_blocks);
#define TTDI_LAUNCH(T, PATH)                                                                               \
  hipLaunchKernelGGL((ttdk::ipc_allreduce_kernel<T, PATH>), dim3(nb), dim3(ttdk::kThreads), 0, st, e->peers, \
                     static_cast<T*>(buf), count, e->rank, e->world, e->cap, e->ctr, e->err, e->spin_max)
  if (dtype == 0 && path == ttd_ipc::kOneShot) TTDI_LAUNCH(float, ttd_ipc::kOneShot);
  else if (dtype == 0) TTDI_LAUNCH(float, ttd_ipc::kTwoShot);
  else if (path == ttd_ipc::kOneShot) TTDI_LAUNCH(bf16_t, ttd_ipc::kOneShot);
  else TTDI_LAUNCH(bf16_t, ttd_ipc::kTwoShot);
#undef TTDI_LAUNCH
  return hipGetLastError();
}

// 1 when a barrier of some call that has run so far timed out (a peer never arrived): the host
// word the kernels write, read without any device synchronisation.
TTDK_EXPORT int ttdi_error(void* h) {
  auto* e = static_cast<IpcEngine*>(h);
  return *reinterpret_cast<volatile int*>(e->err);
}

// Clear the error word (tests; a recovered session builds a fresh engine instead). The caller
// makes sure no launch of this engine is still running.
TTDK_EXPORT void ttdi_clear_error(void* h) {
  auto* e = static_cast<IpcEngine*>(h);
  (void)hipSetDevice(e->device);
  (void)hipMemset(e->flags + ttdk::kAbortIdx, 0, sizeof(unsigned));
  (void)hipDeviceSynchronize();
  *reinterpret_cast<volatile int*>(e->err) = 0;
}

TTDK_EXPORT void ttdi_destroy(void* h) {
  auto* e = static_cast<IpcEngine*>(h);
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  for (int p = 0; p < e->world; ++p) {
    if (!e->opened[p]) continue;
    (void)hipIpcCloseMemHandle(e->peers.data[p]);
    (void)hipIpcCloseMemHandle(e->peers.flags[p]);
  }
  (void)hipFree(e->data);
  (void)hipFree(e->flags);
  (void)hipFree(e->ctr);
  (void)hipHostFree(e->err);
  delete e;
}
