"""Bucketed, backward-overlapped gradient all-reduce over RCCL (xGMI) / gloo.

This is the MirroredStrategy / MultiWorkerMirroredStrategy gradient aggregation of the north
star (BASELINE.json) — the reference itself aggregates through PS accumulators instead
(SyncReplicasOptimizer, /root/reference/distribute_training.py:142-148).

Design for MI355X:
* gradients live in ONE flat fp32 buffer laid out in backward-completion order
  (train/flat.py), so a bucket is a contiguous slice: all-reduce runs in place, no
  pack/unpack copies, no per-tensor launches;
* the model calls `mark_ready(name)` when every gradient up to `name` is final; each bucket
  whose end lies below that watermark is launched immediately with `async_op=True`, so RCCL
  (on its own HIP stream, ordered after the compute stream at launch time) overlaps with the
  rest of backward;
* bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X) and RCCL rings are
  per-link bound, so per-collective latency (tens of us) rather than HBM capacity is the
  constraint. The default (first bucket 4 MB so communication starts early, then 32 MB)
  keeps ResNet-50 (~100 MB of fp32 gradients) at four collectives;
* `finish()` makes the compute stream wait for the collectives (no host sync).

On GPU process groups the buckets go through the native RCCL engine (`rccl.py`,
`csrc/kernels/collective.hip`): its own communicator and HIP stream, an event fork per bucket,
bf16 compression cast on the communicator stream, capture-safe. `TTD_COLLECTIVE=torch` (or a
failed start-up self-check on any rank) routes them through torch.distributed instead.

Gradients are pre-scaled by 1/world (the loss gradient scale), so SUM == mean.

Reduction algorithms (tf.distribute cross-device ops, strategy.py):
* "allreduce"      one RCCL all-reduce per bucket (RcclAllReduce / NcclAllReduce);
* "hierarchical"   reduce-scatter then all-gather per bucket — each rank reduces 1/world of the
                   bucket, the two phases run back to back on the communicator's stream
                   (HierarchicalCopyAllReduce; on one xGMI node both phases are per-link bound like
                   the ring, it exists for its different bandwidth / latency split);
* "reduce_to_one"  reduce to rank 0, then broadcast from it (ReductionToOneDevice).
`num_packs` (TF's RcclAllReduce(num_packs)) splits the gradient buffer into that many
equal-size buckets instead of the bucket_mb sizing.
"""
from __future__ import annotations

import bisect
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


ALGORITHMS = ("allreduce", "hierarchical", "reduce_to_one")


class BucketedAllReducer:
    def __init__(self, flat, group=None, bucket_mb: float = 32.0, first_bucket_mb: float = 4.0,
                 compress_bf16: bool = False, algorithm: str = "allreduce", num_packs: Optional[int] = None,
                 engine: str = "auto", overlap_ms: Optional[float] = None):
        """engine: "auto" (native RCCL engine on GPU process groups of > 1 rank), "native"
        (required; also on a one-rank group — tests), "torch" (torch.distributed calls), "ipc"
        (rehearsal: EVERY bucket on the direct xGMI one-/two-shot kernels over IPC-mapped staging
        buffers, any process group as the control plane — e.g. gloo with several ranks sharing
        one GPU, which RCCL refuses — so the multi-rank step, collectives included, is made of
        stream-ordered GPU kernels and can be hipGraph-captured and replayed like the RCCL one).
        overlap_ms: the caller's estimate of the backward the collectives hide under (the native
        engine's start-up CTA-budget probe uses it, rccl.choose_cta_budget)."""
        if algorithm not in ALGORITHMS:
            raise ValueError("unknown all-reduce algorithm %r (one of %s)" % (algorithm, ALGORITHMS))
        if engine not in ("auto", "native", "torch", "ipc"):
            raise ValueError("unknown reducer engine %r" % engine)
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.compress = compress_bf16
        self.algorithm = algorithm
        if num_packs is not None and num_packs > 0:
            # TF num_packs: that many (roughly equal) buckets over the whole gradient buffer
            bucket_mb = first_bucket_mb = max(flat.numel * 4 / num_packs, 4.0) / (1 << 20)
        # end offset (exclusive) of each variable in layout order, INCLUDING the alignment padding
        # up to the next variable (flat.ALIGN elements): every bucket then starts and ends 256-B
        # aligned (whole 16-B vectors for the direct kernels); the padding's gradient is zero
        starts = [flat.offsets[s.name] for s in flat.specs]
        ends = []
        for i, s in enumerate(flat.specs):
            n = 1
            for d in s.shape:
                n *= int(d)
            nxt = min([o for o in starts if o > starts[i]], default=flat.numel)
            ends.append(max(starts[i] + n, nxt))
        if ends:  # the alignment padding after the last variable rides in the last bucket
            ends[-1] = flat.numel
        self._var_end = {s.name: e for s, e in zip(flat.specs, ends)}
        self._ends = ends
        self.bucket_mb = bucket_mb
        self.first_bucket_mb = first_bucket_mb
        self._make_buckets()
        # GPU process groups: the native RCCL engine (rccl.py / collective.hip) unless
        # TTD_COLLECTIVE=torch or its self-check failed on some rank
        self.comm = None
        if engine == "native" or (engine == "auto" and self.world > 1 and flat.grad.is_cuda):
            from . import rccl
            self.comm = rccl.for_group(group, required=engine == "native", overlap_ms=overlap_ms,
                                       bucket_bytes=[(e - s) * (2 if compress_bf16 else 4) for s, e in self.buckets])
            pol = getattr(self.comm, "policy", None) or {}
            fb = pol.get("first_bucket_mb")
            if fb and num_packs is None and fb > self.first_bucket_mb:
                # the probe found small collectives latency-bound: start with a bigger bucket
                self.first_bucket_mb = fb
                self._make_buckets()
        self.engine = "native-rccl" if self.comm is not None else ("torch-" + dist.get_backend(group)
                                                                   if self.world > 1 else "none")
        self.ipc_stream = None  # engine "ipc": the direct kernels' own communicator stream
        # CUs the persistent kernels leave to the collectives while buckets are in flight
        # (rccl.py: co-scheduling policy). Opt-in: at the default CTA budget the measured
        # interference is < 1 % without it (tools/comm_interference.py)
        import os
        self.reserved_cus = (int(getattr(self.comm, "max_ctas", 0) or 0)
                             if self.world > 1 and os.environ.get("TTD_RESERVE_COMM_CUS", "0") == "1" else 0)
        self._reserved_on = False
        if self.comm is not None and compress_bf16 and self.buckets:
            # the bf16 staging buffer at its final size before any step can be graph-captured
            self.comm.reserve(max(e - s for s, e in self.buckets))
        # direct xGMI all-reduce (parallel/ipc.py) for the first and last buckets of a
        # single-node group: one-shot <= 1 MB, two-shot <= 8 MB; RCCL keeps the rest
        self.ipc = None
        self.ipc_reason = None
        self._paths = [0] * len(self.buckets)
        if self.comm is not None and self.world > 1 and not compress_bf16 and flat.grad.is_cuda:
            from . import ipc as ipcm
            if not ipcm.enabled():
                self.ipc_reason = "off (opt-in: TTD_IPC_AR=1)"
            else:
                same = ipcm.group_same_node(group)
                paths = ipcm.plan_paths([(e - s) * 4 for s, e in self.buckets], self.world, same)
                # whole 16-B vectors at 16-B aligned offsets only (same layout on every rank)
                paths = [p if (s % 4 == 0 and (e - s) % 4 == 0) else ipcm.RCCL
                         for p, (s, e) in zip(paths, self.buckets)]
                if not same:
                    self.ipc_reason = "group spans several nodes"
                elif any(p != ipcm.RCCL for p in paths):
                    try:
                        # no more workgroups per launch than RCCL's CTA budget (co-scheduling)
                        self.ipc = ipcm.IpcAllReducer(group, max_blocks=int(getattr(self.comm, "max_ctas", 0) or 0))
                    except Exception as e:  # noqa: BLE001 - every rank raised together: all use RCCL
                        self.ipc_reason = "%s: %s" % (type(e).__name__, e)
                    if self.ipc is not None:
                        why = self._ipc_selfcheck()
                        if why:
                            self.ipc.destroy()
                            self.ipc, self.ipc_reason = None, why
                        else:
                            self._paths = paths
        if engine == "ipc":
            self._init_ipc_rehearsal(group)
        self._next = 0
        self._works = []
        self._keep = []
        self._timed = None
        self._window = None
        self.launch_log: List[int] = []

    def _init_ipc_rehearsal(self, group):
        """engine "ipc": every bucket through the direct one-shot (<= 1 MB) / two-shot kernels on a
        stream of the reducer's own (staging buffers sized for the largest bucket)."""
        from ..utils import errors
        from . import ipc as ipcm
        if self.world < 2 or not self.flat.grad.is_cuda or self.compress:
            raise errors.FailedPreconditionError("the ipc rehearsal engine wants >= 2 GPU ranks, fp32 buckets")
        if any(s % 4 or (e - s) % 4 for s, e in self.buckets):
            raise errors.FailedPreconditionError("ipc rehearsal: a bucket is not whole 16-B vectors")
        # at least the default staging size: the self-check's two-shot pattern is 3 MB, larger
        # than every bucket of a small model
        cap = max(max(e - s for s, e in self.buckets) * 4, ipcm.default_cap())
        self.ipc = ipcm.IpcAllReducer(group, cap_bytes=cap)
        why = self._ipc_selfcheck()
        if why:
            self.ipc.destroy()
            self.ipc = None
            raise errors.UnavailableError("ipc rehearsal engine: " + why)
        self._paths = [ipcm.ONE_SHOT if (e - s) * 4 <= ipcm.ONE_SHOT_MAX else ipcm.TWO_SHOT
                       for s, e in self.buckets]
        self.ipc_stream = torch.cuda.Stream(device=self.flat.grad.device)
        self.engine = "ipc-rehearsal"

    def _ipc_selfcheck(self) -> Optional[str]:
        """Both direct paths on a known pattern (sum of rank + 1), every rank voting: the paths
        are used only if they return the right sum without a barrier timeout on EVERY rank."""
        from . import ipc as ipcm
        why = ""
        try:
            r = dist.get_rank(self.group)
            want = self.world * (self.world + 1) / 2
            for path, n in ((ipcm.ONE_SHOT, 64 * 1024), (ipcm.TWO_SHOT, 768 * 1024)):
                t = torch.full((n,), float(r + 1), dtype=torch.float32, device=self.flat.grad.device)
                self.ipc.all_reduce_(t, path)
                if not bool(torch.all(t == want).item()):
                    why = "self-check: %s returned a wrong sum" % ipcm.PATH_NAMES[path]
            if not why and self.ipc.timed_out():
                why = "self-check: a barrier timed out"
        except Exception as e:  # noqa: BLE001 - voted below
            why = "self-check: %s: %s" % (type(e).__name__, e)
        flag = torch.tensor([0 if why else 1], dtype=torch.int32, device=self.flat.grad.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1:
            return None
        return why or "self-check failed on another rank"

    @property
    def bucket_paths(self) -> List[str]:
        """Path of every bucket: "ipc_oneshot" / "ipc_twoshot" (direct xGMI), "rccl" (native
        engine), or the torch backend's name."""
        from .ipc import PATH_NAMES
        if self.comm is None and self.ipc_stream is None:
            return [self.engine] * len(self.buckets)
        return [PATH_NAMES[p] for p in self._paths]

    def measure_window(self):
        """Record, in the next step, how long the backward runs on after the first bucket is
        ready (the window the collectives can hide under): `window_ms()` afterwards."""
        if self.flat.grad.is_cuda:
            self._window = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), False]

    def window_ms(self) -> Optional[float]:
        w, self._window = self._window, None
        if w is None or not w[2]:
            return None
        w[1].synchronize()
        return float(w[0].elapsed_time(w[1]))

    def retune(self, overlap_ms: float):
        """Re-decide the native engine's CTA budget from a measured overlap window (collective:
        every rank calls it with the same value, e.g. the MAX over ranks of window_ms())."""
        if self.comm is None:
            return
        from . import rccl
        old = self.comm
        self.comm = rccl.retune(self.group, self.comm, float(overlap_ms),
                                [(e - s) * (2 if self.compress else 4) for s, e in self.buckets])
        if self.comm is not old:
            if self.compress and self.buckets:
                # the fresh communicator's bf16 staging buffer at its final size before any
                # step can be graph-captured (as in __init__)
                self.comm.reserve(max(e - s for s, e in self.buckets))
            if self.ipc is not None:
                self.ipc.max_blocks = int(getattr(self.comm, "max_ctas", 0) or 0)

    def _make_buckets(self):
        """Greedy buckets on variable boundaries: the first `first_bucket_mb` (communication
        starts early), then `bucket_mb` each."""
        self.buckets: List[Tuple[int, int]] = []
        start = 0
        limit = int(self.first_bucket_mb * (1 << 20)) // 4
        for e in self._ends:
            if e - start >= limit:
                self.buckets.append((start, e))
                start = e
                limit = int(self.bucket_mb * (1 << 20)) // 4
        if start < self.flat.numel:
            self.buckets.append((start, self.flat.numel))
        self._bucket_ends = [b[1] for b in self.buckets]

    def policy(self):
        """The native engine's start-up collective policy (CTA budget, probe table, reason), or
        None on the torch / single-rank paths."""
        return getattr(self.comm, "policy", None)

    def bytes_per_step(self) -> int:
        """Bytes each rank hands to the collectives per step (all buckets)."""
        return sum(e - s for s, e in self.buckets) * (2 if self.compress else 4)

    def time_next_step(self):
        """Instrument the next step's collectives (native engine only): `comm_stats()` then
        reports their busy time and how much of it the backward did not hide."""
        if self.comm is None:
            return False
        self.comm.set_timing(True)
        self._timed = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        return True

    def comm_stats(self):
        """After a step run with time_next_step(): {buckets, busy_ms, span_ms, exposed_ms,
        overlap_pct}. exposed_ms = time the consumer stream waited for the collectives after the
        backward's last kernel was queued; overlap_pct = share of the busy time hidden."""
        if self.comm is None or self._timed is None:
            return None
        st = self.comm.timing()
        self.comm.set_timing(False)
        self._timed[1].synchronize()
        exposed = float(self._timed[0].elapsed_time(self._timed[1]))
        self._timed = None
        st["exposed_ms"] = round(exposed, 4)
        st["overlap_pct"] = round(100.0 * max(0.0, 1.0 - exposed / st["busy_ms"]), 1) if st["busy_ms"] > 0 else None
        return st

    def check(self):
        """Raise UnavailableError when a direct-path bucket of a finished call failed (a peer
        missed a barrier: that bucket holds NaN, not a sum). Reads a host-mapped word: no sync."""
        if self.ipc is not None:
            self.ipc.check()

    def begin(self):
        self.check()  # the previous step's direct-path buckets, as far as they have run
        self._next = 0
        self._works = []
        self._keep = []
        self.launch_log = []

    def _reserve(self, on: bool):
        if self.reserved_cus <= 0 or on == self._reserved_on:
            return
        from . import rccl
        rccl.set_reserved_cus(self.reserved_cus if on else 0)
        self._reserved_on = on

    def _launch(self, i):
        s, e = self.buckets[i]
        t = self.flat.grad[s:e]
        self.launch_log.append(i)
        if self.world == 1 and self.comm is None:
            return
        if self.ipc_stream is not None:
            # rehearsal engine: the direct kernel on the reducer's stream, ordered after the
            # producing stream (an event node pair under segmented capture)
            from ..utils import graphs
            graphs.fork(torch.cuda.current_stream(), self.ipc_stream)
            self.ipc.all_reduce_(t, self._paths[i], stream=self.ipc_stream)
            return
        if i == 0:
            # from the first bucket on, RCCL CTAs may hold CUs: persistent grids launched from
            # here to finish() use the remaining ones
            self._reserve(True)
            if self._window is not None:
                self._window[0].record()
        if self.comm is not None:
            # in place on the communicator stream, ordered after the current (producing) stream;
            # under a segmented hipGraph capture the fork is an event node pair and the
            # communicator stream records its own linear graph segments (utils/graphs.py)
            from ..utils import graphs
            if self.ipc is not None and self._paths[i] != 0:
                # direct xGMI one-/two-shot on the communicator stream (same ordering as RCCL)
                graphs.fork(torch.cuda.current_stream(), self.comm.stream)
                self.ipc.all_reduce_(t, self._paths[i], stream=self.comm.stream)
                return
            if graphs.capturing_segmented():
                graphs.fork(torch.cuda.current_stream(), self.comm.stream)
                self.comm.bucket(t, algorithm=self.algorithm, compress=self.compress, fork=False)
            else:
                self.comm.bucket(t, algorithm=self.algorithm, compress=self.compress)
            return
        c = t.to(torch.bfloat16) if self.compress else t
        if self.algorithm == "allreduce":
            w = dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        elif self.algorithm == "reduce_to_one":
            # ops on one communicator run in issue order (RCCL: one stream); gloo's worker
            # threads need the reduce finished before the broadcast reads rank 0's result
            w = dist.reduce(c, dst=0, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if not self._ordered():
                w.wait()
            w = dist.broadcast(c, src=0, group=self.group, async_op=True)
        else:  # hierarchical: reduce-scatter + all-gather over a world-divisible staging buffer
            n = c.numel()
            per = -(-n // self.world)
            if per * self.world == n:
                buf = c
            else:
                buf = torch.zeros(per * self.world, dtype=c.dtype, device=c.device)
                buf[:n].copy_(c)
            part = torch.empty(per, dtype=c.dtype, device=c.device)
            w = dist.reduce_scatter_tensor(part, buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if not self._ordered():
                w.wait()
            w = dist.all_gather_into_tensor(buf, part, group=self.group, async_op=True)
            self._keep.append(part)  # alive until the collective completed (finish)
            if buf is not c:
                self._works.append((w, buf[:n], t))
                return
        self._works.append((w, c if c is not t else None, t if c is not t else None))

    def _ordered(self) -> bool:
        """Whether async collectives of this group complete in issue order (RCCL's single
        communicator stream) — gloo runs them on a thread pool."""
        return dist.get_backend(self.group) == "nccl"

    def mark_ready(self, name: str):
        """All gradients up to and including variable `name` are final."""
        upto = self._var_end[name]
        while self._next < len(self.buckets) and self.buckets[self._next][1] <= upto:
            self._launch(self._next)
            self._next += 1

    def sync_on_read(self):
        """TF SyncOnRead(MEAN) semantics for the non-trainable variables (BatchNorm moving
        mean/variance): every replica updates its own copy from its own batch; reading them in
        cross-replica context (checkpoint save, evaluation) first averages them across replicas."""
        sync_on_read_mean_(self.flat, self.group)

    def finish(self):
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        self._reserve(False)
        if self._window is not None:
            self._window[1].record()  # the backward's last queued work
            self._window[2] = True
        if self.ipc_stream is not None:
            from ..utils import graphs
            graphs.join(torch.cuda.current_stream(), self.ipc_stream)
            if not graphs.capturing_segmented():
                self.check()
            return
        if self.comm is not None:
            if self._timed is not None:
                self._timed[0].record()  # the backward's last queued work
            from ..utils import graphs
            if graphs.capturing_segmented():
                graphs.join(torch.cuda.current_stream(), self.comm.stream)
            else:
                self.comm.join()  # the current stream waits for the buckets (no host sync)
                self.check()
            if self._timed is not None:
                self._timed[1].record()
            return
        works, self._works = self._works, []
        for w, c, t in works:
            try:
                w.wait()
            except Exception as e:  # noqa: BLE001 - an aborted/failed communicator is a preemption
                from .fault import as_preemption_error
                raise as_preemption_error(e) from e
            if c is not None:
                t.copy_(c)
        self._keep = []


def allreduce_mean_(tensor: torch.Tensor, group=None):
    """Blocking mean all-reduce of a small tensor (metrics)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return tensor
    dist.all_reduce(tensor, op=dist.ReduceOp.SUM, group=group)
    tensor /= dist.get_world_size(group)
    return tensor


def broadcast_flat_(flat, src: int = 0, group=None):
    """Replica-0 broadcast of the initial master weights (Mirrored strategies' variable
    synchronisation at creation)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.broadcast(flat.master, src=src, group=group)
    flat.refresh_compute()


def sync_on_read_mean_(flat, group=None):
    """Average the non-trainable variables of a FlatParams store across replicas (one packed
    all-reduce; see BucketedAllReducer.sync_on_read)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    names = [s.name for s in flat.specs if not s.trainable]
    if not names:
        return
    packed = torch.cat([flat.var[n].reshape(-1) for n in names])
    dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
    packed /= dist.get_world_size(group)
    o = 0
    for n in names:
        k = flat.var[n].numel()
        flat.var[n].copy_(packed[o:o + k].view_as(flat.var[n]))
        o += k


def broadcast_state_(flat, opt=None, src: int = 0, group=None):
    """Make every replica hold replica `src`'s training state: master weights (then the bf16
    compute copy), the optimizer's slot buffers and its step counter. Used after a restore
    (only `src` read the checkpoint) and after a recovery (MonitoredTrainingSession)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.broadcast(flat.master, src=src, group=group)
    flat.refresh_compute()
    if opt is None:
        return
    for name in ("mom", "m", "v"):
        buf = getattr(opt, name, None)
        if isinstance(buf, torch.Tensor):
            dist.broadcast(buf, src=src, group=group)
    step = torch.tensor([int(opt._host_step)], dtype=torch.int64, device=flat.master.device)
    dist.broadcast(step, src=src, group=group)
    opt.set_step(int(step.item()))


def broadcast_flag(flag: bool, src: int = 0, group=None, device=None) -> bool:
    """Replica `src`'s value of a host boolean on every replica (e.g. "the checkpoint timer
    fired"), so that decisions taken from per-process clocks stay collective-consistent."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return bool(flag)
    dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                             if dist.get_backend(group) == "nccl" else torch.device("cpu"))
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.broadcast(t, src=src, group=group)
    return bool(t.item())
