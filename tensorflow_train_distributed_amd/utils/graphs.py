"""hipGraph capture of launch-bound training steps.

The ResNet/BERT engines issue a few hundred small kernels per step through ctypes; every
launcher takes PyTorch's *current* stream and performs no host synchronisation (device-side
LR schedule / global step, fused loss sums kept on device), so a whole step can be recorded
once into a hipGraph and replayed with a single launch — the MI355X replacement for the
reference's XLA/graph-mode step ("graph executor").

Rules a captured callable must follow (all framework engines do):
* no `.item()`, `.cpu()`, `torch.cuda.synchronize()` or other host reads inside;
* inputs/outputs live in fixed buffers (refill them in place between replays);
* any step-dependent scalar must be read from device memory (optimizer hyper array, step
  counter), not passed as a kernel argument.

Temporary tensors allocated during capture come from the graph's private memory pool, so
replay reuses exactly the same addresses.
"""
from __future__ import annotations

import ctypes
import os
from typing import Any, Callable, Optional, Tuple

import torch


class CapturedStep:
    """A recorded step: `replay()` re-runs every captured kernel on the current stream."""

    def __init__(self, graph: "torch.cuda.CUDAGraph", outputs: Any):
        self.graph = graph
        self.outputs = outputs

    def replay(self):
        self.graph.replay()
        return self.outputs

    __call__ = replay


def capture(fn: Callable[[], Any], warmup: int = 1, pool=None,
            stream: Optional[torch.cuda.Stream] = None) -> Tuple[CapturedStep, Any]:
    """Run `fn` `warmup` times eagerly on a side stream (so lazily-built state — workspaces,
    chunk tables, split-K slabs — exists before capture), then record one call into a hipGraph.

    Returns (CapturedStep, outputs-of-the-captured-call). NOTE: the warmup calls execute real
    work (e.g. optimizer updates), exactly like eager steps would.
    """
    if not torch.cuda.is_available():
        raise RuntimeError("hipGraph capture needs a GPU")
    s = stream or torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=pool, stream=s):
        out = fn()
    torch.cuda.synchronize()
    return CapturedStep(g, out), out


class GraphedStep:
    """Lazily captured step: the first `eager_steps` calls run eagerly, the next call captures,
    every later call replays. `enabled=False` keeps it eager (debugging, CPU)."""

    def __init__(self, fn: Callable[[], Any], eager_steps: int = 1, enabled: bool = True):
        self.fn = fn
        self.eager_steps = eager_steps
        self.enabled = enabled and torch.cuda.is_available()
        self.calls = 0
        self.captured: Optional[CapturedStep] = None

    def __call__(self):
        if not self.enabled:
            return self.fn()
        if self.captured is not None:
            return self.captured.replay()
        self.calls += 1
        if self.calls <= self.eager_steps:
            return self.fn()
        self.captured, out = capture(self.fn, warmup=0)
        # the capture itself did not execute the step: run it once so call semantics hold
        return self.captured.replay()


# ---------------------------------------------------------------------------------------------
# HIP entry points the torch API does not expose (event nodes, capture dependencies).

_HIP = None
_P = ctypes.c_void_p


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    return _HIP


# ---------------------------------------------------------------------------------------------
# Segmented two-stream capture (what the bench replays).
#
# Stream capture does not carry stream priority into kernel nodes, and per-node priorities
# (hipLaunchAttributePriority + hipGraphInstantiateFlagUseNodePriority) are refused on ROCm 7.2
# (round-3 probe), so a single multi-branch graph lets the main chain and the side-stream weight
# gradients compete as equals and replays slower than the eager two-stream ResNet step. The step
# is instead recorded as LINEAR graphs, one per
# stream, replayed on the very streams the eager step uses (main chain: high priority; weight
# gradients: normal priority) — the hardware sees the eager step's queues and priorities.
# Cross-stream dependencies become event record / wait NODES added to the capture graphs by hand
# (hipEventRecordWithFlags(..., hipEventRecordExternal) is refused under capture on ROCm 7.2),
# and every join (main waits for a side stream) cuts the capture into a new segment, so at replay
# each wait node is enqueued after the record it waits for (segments are launched in capture
# order: main_k, the side streams' segment k, main_k+1, ...). The engines express their stream
# forks and joins through fork() / join() / record() / wait() below, which are plain torch
# events outside such a capture.

_SEG = None  # the active SegmentedCapture


def _ev_create():
    e = _P(0)
    if _hip().hipEventCreateWithFlags(ctypes.byref(e), 2) != 0:  # hipEventDisableTiming
        raise RuntimeError("hipEventCreateWithFlags failed")
    return e


def _add_event_node(stream, ev, wait: bool):
    hip = _hip()
    status, cid, graph, deps, n = ctypes.c_int(0), ctypes.c_ulonglong(0), _P(0), _P(0), ctypes.c_size_t(0)
    rc = hip.hipStreamGetCaptureInfo_v2(_P(stream.cuda_stream), ctypes.byref(status), ctypes.byref(cid),
                                        ctypes.byref(graph), ctypes.byref(deps), ctypes.byref(n))
    if rc != 0 or status.value != 1:
        raise RuntimeError("segmented capture: stream is not capturing (rc %d, status %d)" % (rc, status.value))
    node = _P(0)
    add = hip.hipGraphAddEventWaitNode if wait else hip.hipGraphAddEventRecordNode
    rc = add(ctypes.byref(node), graph, deps, n, ev)
    if rc != 0:
        raise RuntimeError("hipGraphAddEvent%sNode failed (%d)" % ("Wait" if wait else "Record", rc))
    # the node becomes the stream's dependency set: later captured work orders after it
    rc = hip.hipStreamUpdateCaptureDependencies(_P(stream.cuda_stream), ctypes.byref(node), ctypes.c_size_t(1), 1)
    if rc != 0:
        raise RuntimeError("hipStreamUpdateCaptureDependencies failed (%d)" % rc)


class SegmentedCapture:
    """Records `fn` as per-stream linear graph segments (see the comment above)."""

    def __init__(self, main: torch.cuda.Stream):
        self.main = main
        self.pools = {}
        self.segments = []  # (stream, CUDAGraph) in launch order
        self.cur = {}       # stream -> CUDAGraph being captured
        self.events = []    # persistent hipEvent_t (referenced by the graphs)
        self.n_ev = 0
        self.tail = {}      # stream -> event recorded at the end of its last closed segment
        self.seg_index = 0  # segments closed so far (a mark remembers the one it was recorded in)
        # stream -> streams whose record nodes in the CURRENT batch of segments it waits on (forks):
        # the batch is launched in an order where every such record precedes its wait
        self.deps = {}

    # -- capture bookkeeping
    def _begin(self, s):
        key = s.cuda_stream
        if key not in self.pools:
            self.pools[key] = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            g.capture_begin(pool=self.pools[key], capture_error_mode="relaxed")
        self.cur[key] = (s, g)

    def _launch_order(self):
        """Streams of the current batch, main first, then every stream after the streams its
        fork waits read records from. Insertion order alone is wrong when a stream that began
        early (e.g. the communicator stream, forked from main for the first bucket) later waits
        on a stream that began after it (the weight-gradient stream, for the next bucket): its
        segment would be launched before the record it waits for, and the wait would pair with
        the previous replay's record (the rehearsal's replicas diverged that way)."""
        main_key = self.main.cuda_stream
        keys = [main_key] + [k for k in self.cur if k != main_key]
        placed, order = set(), []
        while len(order) < len(keys):
            for k in keys:
                if k not in placed and all(d in placed or d not in self.cur for d in self.deps.get(k, ())):
                    order.append(k)
                    placed.add(k)
                    break
            else:
                raise RuntimeError("segmented capture: cyclic fork dependencies between streams in one segment")
        return order

    def _end_all(self):
        order = self._launch_order()
        main_key = self.main.cuda_stream
        for k in order:
            if k not in self.cur:
                continue
            s, g = self.cur[k]
            if k != main_key:
                # a side segment may end with work main has not waited for yet (a join to an
                # earlier mark cut it): its tail event lets a later join wait for all of it
                ev = self._event()
                _add_event_node(s, ev, wait=False)
                self.tail[k] = ev
            del self.cur[k]
            with torch.cuda.stream(s):
                g.capture_end()
            self.segments.append((s, g))
        self.deps = {}
        self.seg_index += 1

    def _event(self):
        if self.n_ev == len(self.events):
            self.events.append(_ev_create())
        e = self.events[self.n_ev]
        self.n_ev += 1
        return e

    # -- the engine's synchronisation points
    def fork(self, src, dst):
        if dst.cuda_stream not in self.cur:
            self._begin(dst)  # the side stream's next segment starts with this wait
        ev = self._event()
        _add_event_node(src, ev, wait=False)
        _add_event_node(dst, ev, wait=True)
        if src.cuda_stream != dst.cuda_stream:
            self.deps.setdefault(dst.cuda_stream, set()).add(src.cuda_stream)

    def join(self, dst, src):
        if dst.cuda_stream != self.main.cuda_stream:
            raise RuntimeError("segmented capture: joins must target the main stream")
        if src.cuda_stream not in self.cur:
            ev = self.tail.pop(src.cuda_stream, None)
            if ev is not None:  # src's work sits in closed (already launched) segments
                _add_event_node(dst, ev, wait=True)
            return
        self.wait_mark(dst, self.mark(src))

    def mark(self, src):
        """Record a point of src's captured work (a record node)."""
        if src.cuda_stream not in self.cur:
            raise RuntimeError("segmented capture: mark on a stream that is not capturing")
        ev = self._event()
        _add_event_node(src, ev, wait=False)
        return (ev, self.seg_index)

    def wait_mark(self, dst, m):
        if dst.cuda_stream != self.main.cuda_stream:
            raise RuntimeError("segmented capture: joins must target the main stream")
        ev, seg = m
        if seg == self.seg_index:
            # the record sits in a segment still being captured: cut, so that it is launched
            # before the segment holding the wait
            self._end_all()
            self._begin(self.main)
        _add_event_node(dst, ev, wait=True)

    # -- run / replay
    def capture(self, fn):
        global _SEG
        if _SEG is not None:
            raise RuntimeError("nested segmented capture")
        _SEG = self
        try:
            self._begin(self.main)
            with torch.cuda.stream(self.main):
                out = fn()
            self._end_all()
        except BaseException:
            # leave no stream in capture mode behind (the caller may fall back to eager steps)
            for s, g in list(self.cur.values()):
                try:
                    with torch.cuda.stream(s):
                        g.capture_end()
                except Exception:  # noqa: BLE001 - an invalidated capture cannot end cleanly
                    pass
            self.cur.clear()
            raise
        finally:
            _SEG = None
        return out

    def replay(self):
        # ordered after the caller's stream and before its next work (the side streams fork from
        # and join main inside the segments)
        cur = torch.cuda.current_stream()
        if cur != self.main:
            self.main.wait_stream(cur)
        for s, g in self.segments:
            with torch.cuda.stream(s):
                g.replay()
        if cur != self.main:
            cur.wait_stream(self.main)


class SegmentedStep:
    def __init__(self, cap: SegmentedCapture, outputs):
        self.cap = cap
        self.outputs = outputs
        self.info = {"segments": len(cap.segments), "events": cap.n_ev,
                     "streams": len({s.cuda_stream for s, _ in cap.segments})}

    def replay(self):
        self.cap.replay()
        return self.outputs

    __call__ = replay


def capture_segmented(fn: Callable[[], Any], main: torch.cuda.Stream, warmup: int = 1) -> SegmentedStep:
    """Run `fn` `warmup` times eagerly on `main`, then record it as per-stream graph segments
    (the streams it forks through fork() / join() keep their identity and priority at replay).
    .replay() may be called from any stream: the segments launch on their own streams, ordered
    after the caller's earlier work and before its later work."""
    if not torch.cuda.is_available():
        raise RuntimeError("hipGraph capture needs a GPU")
    main.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(main):
        for _ in range(warmup):
            fn()
    torch.cuda.synchronize()
    cap = SegmentedCapture(main)
    out = cap.capture(fn)
    torch.cuda.synchronize()
    return SegmentedStep(cap, out)


def fork(src, dst):
    """dst orders after the work already queued on src (a torch event outside segmented capture)."""
    if _SEG is not None:
        _SEG.fork(src, dst)
        return
    ev = torch.cuda.Event()
    ev.record(src)
    dst.wait_event(ev)


def join(dst, src):
    """dst (the main stream) orders after everything queued on src."""
    if _SEG is not None:
        _SEG.join(dst, src)
        return
    dst.wait_stream(src)


def mark(src):
    """A point of src's queued work that join_mark() can wait for later."""
    if _SEG is not None:
        return _SEG.mark(src)
    ev = torch.cuda.Event()
    ev.record(src)
    return ev


def join_mark(dst, m):
    if _SEG is not None:
        _SEG.wait_mark(dst, m)
        return
    dst.wait_event(m)


def capturing_segmented() -> bool:
    return _SEG is not None


# ---------------------------------------------------------------------------------------------
# CU-masked side streams.
#
# The ResNet/BERT weight gradients run on a normal-priority side stream next to the
# high-priority data-gradient chain. Stream priority only orders dispatch: a side workgroup that
# has started holds its CU until it finishes, so the chain's one-workgroup-per-CU GEMMs wait for
# CUs (measured: the stage-3/4 3x3 data gradients take 1.8x their standalone time in the step).
# A side stream created with a CU mask can only ever occupy those CUs.

def cu_masked_stream(device, cus: int) -> torch.cuda.ExternalStream:
    """A HIP stream whose kernels run only on `cus` of the device's CUs (hipExtStreamCreateWith-
    CUMask), spread over the CU index range with a stride coprime to 8 so every XCD gets its
    share whichever way CU indices map to XCDs. The stream lives for the process."""
    dev = torch.device(device)
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    cus = max(1, min(int(cus), n))
    words = (n + 31) // 32
    mask = [0] * words
    stride = 37 if n % 37 else 41
    for i in range(cus):
        idx = (i * stride + 5) % n
        mask[idx // 32] |= 1 << (idx % 32)
    hip = _hip()
    s = _P(0)
    with torch.cuda.device(dev):
        arr = (ctypes.c_uint32 * words)(*mask)
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), arr)
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed (%d)" % rc)
    return torch.cuda.ExternalStream(s.value, device=dev)
