"""Native RCCL communicator (csrc/kernels/collective.hip) for the gradient all-reduce.

`BucketedAllReducer` (collective.py) launches its buckets through this engine on GPU process
groups: one RCCL communicator per replica group, created from rank 0's unique id (handed out
over the existing torch process group), with its own HIP stream. A bucket launch is an event
fork from the stream that produced the bucket's last gradient onto the communicator stream,
then the in-place RCCL call(s); `join()` makes the consumer stream wait. No host
synchronisation anywhere on the step path, and the calls are capture-safe (hipGraph).

Co-scheduling policy (MI355X, one process per GPU): the fastest backward kernels are persistent,
one workgroup per CU with a static work split (gemm256p, the pointwise / halo conv kernels), so
a workgroup that finds its CU held by an all-reduce CTA delays the whole launch by a full share.
A small RCCL CTA budget (maxCTAs 8 = 3 % of the 256 CUs) keeps the collectives out of the
compute's way (tools/comm_interference.py: < 1 % step-time cost with 200 us of peer skew) — IF
those 8 channels still carry the step's gradient bytes inside the backward. That is measured,
not assumed: when a multi-rank communicator is created (`for_group`), the engine probes the
all-reduce at 1 MB and 32 MB on RCCL's own CTA choice and on the capped budget (one
communicator each), every rank takes the slowest rank's numbers (so all ranks decide alike),
and `choose_cta_budget` keeps the cap only if the projected per-step all-reduce time at the
capped bandwidth, times a 1.5 margin, fits the backward's overlap window (`overlap_ms`, the
caller's estimate of its backward) — otherwise RCCL's own budget, the faster one. Without an
overlap estimate the cap is kept when it delivers >= 70 % of the default bus bandwidth. The
probe table, the choice and the reason travel with the communicator (`policy`) into the bench
JSON. While the step's buckets are in flight the persistent grids can size themselves to the
remaining CUs (ttdk_set_reserved_cus, opt-in TTD_RESERVE_COMM_CUS=1).
Latency-bound small buckets: when the 1 MB probe runs at < 25 % of the 32 MB bus bandwidth
(per-collective latency dominates), `policy["first_bucket_mb"]` raises the reducer's first
bucket so the first collective is not a latency-bound one.

Tuning knobs (environment, read at communicator creation):
  TTD_RCCL_MAX_CTAS / TTD_RCCL_MIN_CTAS  RCCL's CTA (workgroup) budget per collective: how many
                                         CUs a bucket all-reduce may occupy while it overlaps
                                         the backward GEMMs (unset: chosen by the start-up
                                         probe; 0 = RCCL's own choice, no CU reservation)
  TTD_RCCL_PRIO                          communicator stream priority (default 0 = normal, below
                                         the main chain's high-priority stream)
  TTD_RCCL_TIMEOUT                       seconds before a collective that makes no progress (a
                                         dead peer) is reported as an error (default 300)
  TTD_RCCL_NONBLOCKING=1                 non-blocking communicator: creation polled against the
                                         deadline too (not capture-safe: RCCL may issue from its
                                         own thread)
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_char_p, c_double, c_float, c_int, c_longlong, c_void_p
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .. import _native
from ..utils import errors

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float64: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5}
_OP = {"sum": 0, "avg": 1, "min": 2, "max": 3}
_ALGO = {"allreduce": 0, "hierarchical": 1, "reduce_to_one": 2}

_bound = False


def _lib():
    global _bound
    lib = _native.hip()
    if not _bound:
        lib.ttdc_error.restype = c_char_p
        lib.ttdc_error.argtypes = [c_void_p]
        lib.ttdc_version.restype = c_int
        lib.ttdc_unique_id.restype = c_int
        lib.ttdc_unique_id.argtypes = [c_char_p]
        lib.ttdc_create.restype = c_void_p
        lib.ttdc_create.argtypes = [c_char_p, c_int, c_int, c_int, c_int, c_int, c_int, c_double, c_int]
        lib.ttdc_stream.restype = c_void_p
        lib.ttdc_stream.argtypes = [c_void_p]
        lib.ttdc_bucket.restype = c_int
        lib.ttdc_bucket.argtypes = [c_void_p, c_void_p, c_longlong, c_int, c_int, c_int, c_int, c_void_p]
        lib.ttdc_bucket_nofork.restype = c_int
        lib.ttdc_bucket_nofork.argtypes = [c_void_p, c_void_p, c_longlong, c_int, c_int, c_int, c_int]
        lib.ttdc_join.restype = c_int
        lib.ttdc_join.argtypes = [c_void_p, c_void_p]
        lib.ttdc_arm.restype = c_int
        lib.ttdc_arm.argtypes = [c_void_p, c_void_p]
        lib.ttdc_collective.restype = c_int
        lib.ttdc_collective.argtypes = [c_void_p, c_int, c_void_p, c_longlong, c_int, c_int, c_int, c_void_p]
        lib.ttdc_synchronize.restype = c_int
        lib.ttdc_synchronize.argtypes = [c_void_p]
        lib.ttdc_probe.restype = c_int
        lib.ttdc_probe.argtypes = [c_void_p, c_void_p, c_longlong, c_int, ctypes.POINTER(c_float)]
        lib.ttdc_set_timing.restype = None
        lib.ttdc_set_timing.argtypes = [c_void_p, c_int]
        lib.ttdc_timing.restype = c_int
        lib.ttdc_timing.argtypes = [c_void_p, ctypes.POINTER(c_float), ctypes.POINTER(c_float)]
        lib.ttdc_destroy.restype = None
        lib.ttdc_destroy.argtypes = [c_void_p, c_int]
        lib.ttdc_reserve.restype = c_int
        lib.ttdc_reserve.argtypes = [c_void_p, c_longlong]
        lib.ttdc_aborts.restype = c_int
        lib.ttdc_aborts.argtypes = [c_void_p]
        lib.ttdc_debug_stall.restype = c_int
        lib.ttdc_debug_stall.argtypes = [c_void_p, c_void_p, c_int]
        lib.ttdc_emulate_bucket.restype = c_int
        lib.ttdc_emulate_bucket.argtypes = [c_void_p, c_int, c_double, c_void_p, c_longlong]
        lib.ttdk_set_reserved_cus.restype = c_int
        lib.ttdk_set_reserved_cus.argtypes = [c_int]
        lib.ttdk_persistent_cus.restype = c_int
        lib.ttdk_persistent_cus.argtypes = []
        _bound = True
    return lib


def rccl_version() -> int:
    """Version code of the RCCL the process actually loaded (torch's bundled one when torch
    came first: both export the soname librccl.so.1)."""
    return int(_lib().ttdc_version())


DEFAULT_MAX_CTAS = 8          # the capped budget the start-up probe evaluates
PROBE_BYTES = (1 << 20, 32 << 20)
CAP_MIN_BW_RATIO = 0.70        # no overlap estimate: keep the cap at >= 70 % of default bandwidth
OVERLAP_MARGIN = 1.5
LATENCY_BOUND_RATIO = 0.25     # 1 MB bus bandwidth below this share of 32 MB's: latency-bound


def _ring_ms(nbytes: float, busbw_gbps: float, nranks: int) -> float:
    """Ring all-reduce time of `nbytes` at bus bandwidth `busbw_gbps` (busbw = algbw*2(n-1)/n)."""
    if busbw_gbps <= 0:
        return float("inf")
    return 2.0 * (nranks - 1) / nranks * nbytes / (busbw_gbps * 1e9) * 1e3


def projected_step_ms(probe, bucket_bytes, nranks: int) -> float:
    """Per-step all-reduce time of `bucket_bytes` (one collective each) from a probe table
    [{bytes, ms, busbw_GBps}, ...] of one CTA budget: t(b) = latency + ring time at the largest
    probed size's bandwidth, latency = what the smallest probe took beyond its ring time."""
    pts = sorted(probe, key=lambda d: d["bytes"])
    big, small = pts[-1], pts[0]
    bw = float(big["busbw_GBps"])
    lat = max(0.0, float(small["ms"]) - _ring_ms(small["bytes"], bw, nranks)) if len(pts) > 1 else 0.0
    return sum(lat + _ring_ms(b, bw, nranks) for b in bucket_bytes)


def choose_cta_budget(probes, bucket_bytes, nranks: int, overlap_ms=None, cap: int = DEFAULT_MAX_CTAS,
                      margin: float = OVERLAP_MARGIN):
    """The CTA budget for the gradient communicator from measured probes.

    probes: {ctas: [{"bytes", "ms", "busbw_GBps"}, ...]} with the capped budget `cap` and 0 (RCCL's
    own choice); bucket_bytes: the reducer's per-step collective sizes; overlap_ms: the backward
    time the collectives can hide under (None: unknown). Returns a policy dict:
    {cta_budget, reason, projected_ms: {ctas: ms}, first_bucket_mb (or None), probe}."""
    proj = {c: projected_step_ms(p, bucket_bytes, nranks) for c, p in probes.items()}
    bw = {c: max(float(d["busbw_GBps"]) for d in p) for c, p in probes.items()}
    pol = {"projected_ms": {str(c): round(v, 3) for c, v in proj.items()}, "probe": probes,
           "overlap_ms": overlap_ms, "first_bucket_mb": None}
    if cap not in probes:
        pol.update(cta_budget=0, reason="no probe of the capped budget")
    elif 0 not in probes:
        pol.update(cta_budget=cap, reason="no probe of RCCL's default budget")
    elif overlap_ms is not None and overlap_ms > 0:
        if proj[cap] * margin <= overlap_ms:
            pol.update(cta_budget=cap, reason="capped budget hides %.2f ms x %.1f in the %.1f ms backward"
                       % (proj[cap], margin, overlap_ms))
        else:
            pol.update(cta_budget=0, reason="capped budget needs %.2f ms x %.1f > %.1f ms backward: RCCL default "
                       "(%.2f ms)" % (proj[cap], margin, overlap_ms, proj[0]))
    else:
        ratio = bw[cap] / bw[0] if bw[0] > 0 else 1.0
        if ratio >= CAP_MIN_BW_RATIO:
            pol.update(cta_budget=cap, reason="capped budget delivers %.0f %% of the default bus bandwidth" % (100 * ratio))
        else:
            pol.update(cta_budget=0, reason="capped budget delivers only %.0f %% of the default bus bandwidth"
                       % (100 * ratio))
    # latency-bound small collectives: make the first bucket big enough to leave that regime
    chosen = probes.get(pol["cta_budget"]) or next(iter(probes.values()))
    pts = sorted(chosen, key=lambda d: d["bytes"])
    if len(pts) > 1 and float(pts[-1]["busbw_GBps"]) > 0 and \
            float(pts[0]["busbw_GBps"]) < LATENCY_BOUND_RATIO * float(pts[-1]["busbw_GBps"]):
        pol["first_bucket_mb"] = 8.0
    return pol


def set_reserved_cus(n: int) -> int:
    """CUs the persistent kernels leave to the collective engine's CTAs (0 = none); returns the
    previous value. Host-side, takes effect for kernels launched after the call."""
    return int(_lib().ttdk_set_reserved_cus(int(n)))


def persistent_cus() -> int:
    """CUs the persistent kernels currently size their grids to."""
    return int(_lib().ttdk_persistent_cus())


def emulate_bucket(stream, ctas: int, us: float, buf: torch.Tensor):
    """Queue an emulated bucket all-reduce (`ctas` workgroups streaming over `buf` for `us`
    microseconds) on `stream`: the one-GPU stand-in of an RCCL bucket kernel."""
    rc = _lib().ttdc_emulate_bucket(_stream_ptr(stream), int(ctas), float(us), buf.data_ptr(), buf.numel() * buf.element_size())
    if rc != 0:
        raise errors.InternalError("emulated bucket launch failed (%d)" % rc)


def unique_id() -> bytes:
    lib = _lib()
    buf = ctypes.create_string_buffer(128)
    if lib.ttdc_unique_id(buf) != 128:
        raise errors.InternalError("ncclGetUniqueId failed: %s" % lib.ttdc_error(None).decode())
    return buf.raw


def _stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


class RcclCommunicator:
    """One RCCL communicator + its HIP stream. Create it on every rank of the group with the
    same `uid` (rank 0's `unique_id()`), or through `for_group` which distributes the id."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: torch.device, priority: Optional[int] = None,
                 min_ctas: Optional[int] = None, max_ctas: Optional[int] = None, timeout: Optional[float] = None,
                 nonblocking: Optional[bool] = None):
        lib = _lib()
        env = os.environ.get
        prio = int(env("TTD_RCCL_PRIO", "0")) if priority is None else int(priority)
        min_ctas = int(env("TTD_RCCL_MIN_CTAS", "0")) if min_ctas is None else int(min_ctas)
        if max_ctas is None:
            max_ctas = int(env("TTD_RCCL_MAX_CTAS", "0"))
        max_ctas = int(max_ctas)
        if min_ctas > max_ctas > 0:
            min_ctas = max_ctas
        timeout = float(env("TTD_RCCL_TIMEOUT", "300")) if timeout is None else float(timeout)
        nonblocking = env("TTD_RCCL_NONBLOCKING", "0") == "1" if nonblocking is None else bool(nonblocking)
        self.device = torch.device(device)
        self.rank, self.nranks = int(rank), int(nranks)
        self.max_ctas = max_ctas
        with torch.cuda.device(self.device):
            h = lib.ttdc_create(uid, self.nranks, self.rank, self.device.index, prio, min_ctas, max_ctas, timeout,
                                1 if nonblocking else 0)
        if not h:
            raise errors.UnavailableError("RCCL communicator creation failed: %s"
                                          % lib.ttdc_error(None).decode())
        self._h = h
        self.stream = torch.cuda.ExternalStream(lib.ttdc_stream(h), device=self.device)
        self.policy = None  # set by for_group's start-up probe (choose_cta_budget)

    @classmethod
    def for_group(cls, group=None, device=None, **kw) -> "RcclCommunicator":
        """Collective over `group`: rank 0 draws the unique id, the torch process group carries
        it to the others — together with a status byte, so a failure on rank 0 (no id) reaches
        every rank through the same broadcast and all of them raise (no rank is left waiting in
        a different collective)."""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        (uid,) = broadcast_unique_ids(group, 1, dev)
        return cls(uid, world, rank, dev, **kw)

    # ------------------------------------------------------------------ step path
    def _check(self, rc: int, what: str):
        if rc != 0:
            raise errors.UnavailableError("%s: %s" % (what, self.error))

    @property
    def error(self) -> str:
        return _lib().ttdc_error(self._h).decode("utf-8", "replace") if self._h else "destroyed"

    def bucket(self, t: torch.Tensor, op: str = "sum", algorithm: str = "allreduce", compress: bool = False,
               producer=None, fork: bool = True):
        """In-place reduction of contiguous `t` on the communicator stream, ordered after the
        work already queued on `producer` (default: the current stream). fork=False: no fork
        (the caller ordered `self.stream` itself, e.g. through utils.graphs.fork under a
        segmented capture)."""
        assert t.is_contiguous() and t.device == self.device
        if fork:
            rc = _lib().ttdc_bucket(self._h, t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op], _ALGO[algorithm],
                                    1 if compress else 0, _stream_ptr(producer))
        else:
            rc = _lib().ttdc_bucket_nofork(self._h, t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op], _ALGO[algorithm],
                                           1 if compress else 0)
        self._check(rc, "bucket all-reduce")

    def join(self, consumer=None):
        """`consumer` (default: current stream) waits for every collective queued so far."""
        self._check(_lib().ttdc_join(self._h, _stream_ptr(consumer)), "collective join")

    def arm(self, stream=None):
        """Arm the no-progress watchdog after a hipGraph replay on `stream` (default: current):
        a join captured into the graph records no marker of its own, so without this a replayed
        step whose collectives never finish would hang without a deadline."""
        self._check(_lib().ttdc_arm(self._h, _stream_ptr(stream)), "watchdog arm")

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        """Stream-ordered in-place all-reduce on `stream` (default: current)."""
        assert t.is_contiguous()
        self._check(_lib().ttdc_collective(self._h, 0, t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op], 0,
                                           _stream_ptr(stream)), "all-reduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        assert t.is_contiguous()
        self._check(_lib().ttdc_collective(self._h, 1, t.data_ptr(), t.numel(), _DT[t.dtype], 0, int(root),
                                           _stream_ptr(stream)), "broadcast")
        return t

    def reserve(self, count: int):
        """Pre-size the bf16 staging buffer for compressed buckets of up to `count` fp32
        elements (growing it later would need a stream sync + hipMalloc: illegal in capture)."""
        self._check(_lib().ttdc_reserve(self._h, int(count)), "staging reserve")

    @property
    def aborted(self) -> bool:
        """The watchdog (or a synchronize deadline) aborted this communicator."""
        return bool(self._h) and _lib().ttdc_aborts(self._h) > 0

    def debug_stall(self, flag_ptr: int, max_ms: int):
        """Fault injection: hold the communicator stream until the int at flag_ptr (host memory
        the device can read) is non-zero or max_ms passed."""
        self._check(_lib().ttdc_debug_stall(self._h, flag_ptr, int(max_ms)), "debug stall")

    def synchronize(self):
        """Host wait for the communicator stream with a deadline (a dead peer raises)."""
        self._check(_lib().ttdc_synchronize(self._h), "collective synchronize")

    def set_timing(self, on: bool):
        """Time each following bucket's reduction on the communicator stream (events recorded
        after its fork wait is satisfied); `timing()` reads them after a synchronize."""
        _lib().ttdc_set_timing(self._h, 1 if on else 0)

    def timing(self) -> Dict[str, float]:
        """{buckets, busy_ms (sum of bucket reduction times), span_ms (first start -> last end)}."""
        self.synchronize()
        busy, span = c_float(0.0), c_float(0.0)
        n = _lib().ttdc_timing(self._h, ctypes.byref(busy), ctypes.byref(span))
        if n < 0:
            raise errors.InternalError("hipEventElapsedTime failed")
        return {"buckets": int(n), "busy_ms": round(float(busy.value), 4), "span_ms": round(float(span.value), 4)}

    def probe(self, nbytes: int, iters: int = 5) -> Dict[str, float]:
        """RCCL bus bandwidth of an fp32 all-reduce of `nbytes` on the communicator stream."""
        buf = torch.zeros(max(1, nbytes // 4), dtype=torch.float32, device=self.device)
        ms = c_float(0.0)
        self._check(_lib().ttdc_probe(self._h, buf.data_ptr(), buf.numel(), int(iters), ctypes.byref(ms)), "probe")
        t = float(ms.value)
        bw = 2.0 * (self.nranks - 1) / self.nranks * nbytes / (t * 1e-3) / 1e9 if t > 0 else 0.0
        return {"bytes": int(nbytes), "ms": round(t, 4), "busbw_GBps": round(bw, 1)}

    def destroy(self, abort: bool = False):
        if self._h:
            _lib().ttdc_destroy(self._h, 1 if abort else 0)
            self._h = None

    def __del__(self):
        try:
            import sys
            if sys.is_finalizing():  # the HIP runtime may already be gone: leave it to process exit
                return
            self.destroy(abort=True)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


# one communicator per (process-group generation, group); recovery aborts them (strategy.py)
_COMMS: Dict[tuple, RcclCommunicator] = {}
_FAILED: Dict[tuple, str] = {}


def _key(group):
    from .strategy import _PG
    return (_PG["generation"], id(group) if group is not None else None)


def broadcast_unique_ids(group, n: int, device) -> List[bytes]:
    """`n` RCCL unique ids drawn on rank 0 of `group`, carried to every rank by ONE broadcast of
    the torch process group with a status byte: a failure on rank 0 reaches every rank through
    that same broadcast and all of them raise together."""
    rank = dist.get_rank(group)
    dev = torch.device(device)
    msg = torch.zeros(128 * n + 1, dtype=torch.uint8, device=dev if dist.get_backend(group) == "nccl" else "cpu")
    why = ""
    if rank == 0:
        try:
            for i in range(n):
                msg[128 * i:128 * (i + 1)].copy_(torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8))
            msg[128 * n] = 1
        except Exception as e:  # noqa: BLE001 - reported to every rank below
            why = "%s: %s" % (type(e).__name__, e)
    dist.broadcast(msg, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    host = msg.cpu()
    if int(host[128 * n]) != 1:
        raise errors.UnavailableError("RCCL unique id unavailable on rank 0%s" % (": " + why if why else ""))
    return [bytes(host[128 * i:128 * (i + 1)].tolist()) for i in range(n)]


def _probe_budgets(group, overlap_ms, bucket_bytes, budgets=None, make=None):
    """Create a communicator per candidate CTA budget, probe each, keep the one the policy
    picks (collective: every rank reaches the same choice from the slowest rank's numbers).

    Every rank runs the same torch process-group sequence whatever happens locally: ONE id
    broadcast (all ids at once), then ONE MAX all-reduce whose slot 0 is a failure flag. A rank
    whose communicator creation or probe fails records it, still joins that all-reduce, and every
    rank then raises together (for_group's MIN vote turns that into a common fallback); a
    failure can no longer leave one rank in the flag vote while the others sit in a different
    collective. `make(uid, world, rank, device, max_ctas)` builds a communicator
    (tests inject failures through it)."""
    budgets = tuple(budgets) if budgets is not None else (DEFAULT_MAX_CTAS, 0)
    make = make or (lambda uid, w, r, dev, ctas: RcclCommunicator(uid, w, r, dev, max_ctas=ctas))
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    uids = broadcast_unique_ids(group, len(budgets), dev)
    comms, probes, why = {}, {}, ""
    try:
        for ctas, uid in zip(budgets, uids):
            c = make(uid, world, rank, dev, ctas)
            comms[ctas] = c
            probes[ctas] = [c.probe(nb, iters=5) for nb in PROBE_BYTES]
    except Exception as e:  # noqa: BLE001 - shared through the status slot below
        why = "%s: %s" % (type(e).__name__, e)
    n = len(budgets) * len(PROBE_BYTES)
    t = torch.zeros(1 + n, dtype=torch.float64, device=dev)
    if why:
        t[0] = 1.0
    else:
        t[1:] = torch.tensor([d["ms"] for c in budgets for d in probes[c]], dtype=torch.float64)
    # identical tables everywhere: the slowest rank's time per (budget, size), and any failure
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    th = t.cpu()
    if float(th[0]) > 0:
        for c in comms.values():
            c.destroy(abort=True)
        raise errors.UnavailableError("CTA-budget probe failed %s" % ("on this rank: " + why if why
                                                                      else "on another rank"))
    i = 1
    for c in budgets:
        for d in probes[c]:
            d["ms"] = round(float(th[i]), 4)
            d["busbw_GBps"] = round(2.0 * (world - 1) / world * d["bytes"] / (d["ms"] * 1e-3) / 1e9, 1) \
                if d["ms"] > 0 else 0.0
            i += 1
    pol = choose_cta_budget(probes, bucket_bytes or [32 << 20], world, overlap_ms)
    keep = pol["cta_budget"]
    for ctas, c in comms.items():
        if ctas != keep:
            c.destroy(abort=False)
    comm = comms[keep]
    comm.policy = pol
    return comm


def for_group(group=None, required: bool = False, overlap_ms=None, bucket_bytes=None) -> Optional[RcclCommunicator]:
    """The native communicator of `group` (created and self-checked on first use), or None when
    the native engine does not apply: a non-RCCL group (gloo), a one-rank group, TTD_COLLECTIVE=
    torch, or a failed self-check on ANY rank (every rank then agrees to use the torch process
    group; the reason is kept in `failure_reason`). Collective: all ranks of `group` call it.
    required=True: also on a one-rank group, and raise instead of returning None.
    Multi-rank groups without TTD_RCCL_MAX_CTAS get their CTA budget from the start-up probe
    (module docstring): `overlap_ms` (the backward the collectives hide under) and
    `bucket_bytes` (per-step collective sizes) feed `choose_cta_budget`."""
    if not dist.is_initialized() or dist.get_backend(group) != "nccl":
        if required:
            raise errors.FailedPreconditionError("the native RCCL engine needs an initialised nccl process group")
        return None
    if not required and (dist.get_world_size(group) == 1 or os.environ.get("TTD_COLLECTIVE", "native") == "torch"):
        return None
    k = _key(group)
    if k in _COMMS:
        return _COMMS[k]
    if k in _FAILED:
        return None
    comm, reason = None, ""
    try:
        w = dist.get_world_size(group)
        probe = os.environ.get("TTD_RCCL_PROBE", "1")  # "force": also on one rank (tests)
        if (w > 1 or probe == "force") and "TTD_RCCL_MAX_CTAS" not in os.environ and probe in ("1", "force"):
            comm = _probe_budgets(group, overlap_ms, bucket_bytes)
        else:
            comm = RcclCommunicator.for_group(group)
            comm.policy = {"cta_budget": comm.max_ctas, "reason": "fixed (TTD_RCCL_MAX_CTAS / one rank / "
                           "TTD_RCCL_PROBE=0)", "probe": None, "first_bucket_mb": None}
        # self-check: sum of (rank + 1) over the group, stream-ordered on the current stream
        t = torch.full((1024,), float(dist.get_rank(group) + 1), dtype=torch.float32, device=comm.device)
        comm.all_reduce_(t)
        ok = bool(torch.all(t == w * (w + 1) / 2).item())
        if not ok:
            reason = "self-check all-reduce returned a wrong sum"
    except Exception as e:  # noqa: BLE001 - reported, then every rank falls back together
        ok, reason = False, "%s: %s" % (type(e).__name__, e)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=torch.device("cuda", torch.cuda.current_device()))
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag.item()) == 1:
        _COMMS[k] = comm
        return comm
    if comm is not None:
        comm.destroy(abort=True)
    _FAILED[k] = reason or "self-check failed on another rank"
    if required:
        raise errors.UnavailableError("native RCCL engine unavailable: %s" % _FAILED[k])
    import warnings
    warnings.warn("native RCCL engine unavailable (%s); gradients all-reduce through the torch process group"
                  % _FAILED[k])
    return None


def retune(group, comm: RcclCommunicator, overlap_ms: float, bucket_bytes) -> RcclCommunicator:
    """Re-decide the CTA budget with a MEASURED overlap window (the warm-up step's backward,
    collective.BucketedAllReducer.window_ms, MAX over ranks so every rank decides alike) from the
    start-up probe table already held in `comm.policy`; when the budget changes, a communicator
    with the new budget replaces `comm` (collective: every rank of `group` calls it with the same
    arguments). Returns the communicator to use."""
    pol = getattr(comm, "policy", None) or {}
    probes = pol.get("probe")
    if not probes:
        return comm  # fixed budget (TTD_RCCL_MAX_CTAS / TTD_RCCL_PROBE=0): nothing to re-decide
    new = choose_cta_budget({int(k): v for k, v in probes.items()}, bucket_bytes or [32 << 20],
                            dist.get_world_size(group), overlap_ms)
    new["overlap_source"] = "measured (warm-up step backward, max over ranks)"
    if int(new["cta_budget"]) == int(comm.max_ctas):
        comm.policy = new
        return comm
    (uid,) = broadcast_unique_ids(group, 1, comm.device)
    fresh = RcclCommunicator(uid, dist.get_world_size(group), dist.get_rank(group), comm.device,
                             max_ctas=int(new["cta_budget"]))
    fresh.policy = new
    comm.synchronize()
    comm.destroy(abort=False)
    _COMMS[_key(group)] = fresh
    return fresh


def failure_reason(group=None) -> Optional[str]:
    return _FAILED.get(_key(group))


def abort_all():
    """Abort every native communicator (process-group recovery: the peers may be gone)."""
    for c in list(_COMMS.values()):
        c.destroy(abort=True)
    _COMMS.clear()
    _FAILED.clear()


def shutdown():
    """Orderly end of a run: finalize + destroy every native communicator (all ranks call it,
    before torch.distributed.destroy_process_group)."""
    for c in list(_COMMS.values()):
        c.destroy(abort=False)
    _COMMS.clear()
    _FAILED.clear()


def _at_exit():
    # a run that ended without shutdown() (an exception): abort while the HIP runtime is alive
    try:
        abort_all()
    except Exception:  # noqa: BLE001
        pass


import atexit  # noqa: E402

atexit.register(_at_exit)
