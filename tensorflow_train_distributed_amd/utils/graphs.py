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

import contextlib
import ctypes
import os
from typing import Any, Callable, List, Optional, Tuple

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
# Priority-preserving capture.
#
# The eager ResNet step runs its main data-gradient chain on a high-priority stream and the
# weight gradients on a normal-priority side stream, so the side stream only takes the CUs the
# main chain's kernels leave idle (their tail waves). Stream capture does not carry stream
# priority into the graph's kernel nodes, so a plain replay lets the two branches compete as
# equals. Here the engine marks its side-stream blocks (side_scope); after capture every kernel
# node gets hipLaunchAttributePriority (side blocks low, everything else high) and the graph is
# instantiated with hipGraphInstantiateFlagUseNodePriority, so replay dispatches like eager.

_HIP = None
_P = ctypes.c_void_p
_KERNEL_NODE = 0             # hipGraphNodeTypeKernel
_ATTR_PRIORITY = 8           # hipLaunchAttributePriority
_FLAG_USE_NODE_PRIORITY = 8  # hipGraphInstantiateFlagUseNodePriority


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    return _HIP


def _capture_graph(stream) -> Optional[int]:
    """The hipGraph_t being captured on `stream` (None when it is not capturing)."""
    hip = _hip()
    status = ctypes.c_int(0)
    cid = ctypes.c_ulonglong(0)
    graph = _P(0)
    deps = _P(0)
    ndeps = ctypes.c_size_t(0)
    rc = hip.hipStreamGetCaptureInfo_v2(_P(stream.cuda_stream), ctypes.byref(status), ctypes.byref(cid), ctypes.byref(graph), ctypes.byref(deps),
            ctypes.byref(ndeps))
    if rc != 0 or status.value != 1 or not graph.value:  # hipStreamCaptureStatusActive
        return None
    return graph.value


def graph_nodes(graph: int) -> List[int]:
    hip = _hip()
    n = ctypes.c_size_t(0)
    if hip.hipGraphGetNodes(_P(graph), None, ctypes.byref(n)) != 0:
        return []
    arr = (_P * n.value)()
    if n.value and hip.hipGraphGetNodes(_P(graph), arr, ctypes.byref(n)) != 0:
        return []
    return [int(a) for a in arr[:n.value] if a]


_SIDE_NODES: Optional[set] = None  # set while a prioritized capture records


@contextlib.contextmanager
def side_scope(stream):
    """Mark the kernels launched in this block (on `stream`, a low-priority side stream) as
    side-branch work for a prioritized capture. Free outside capture."""
    if _SIDE_NODES is None:
        yield
        return
    g = _capture_graph(stream)
    before = set(graph_nodes(g)) if g else None
    try:
        yield
    finally:
        if g:
            _SIDE_NODES.update(set(graph_nodes(g)) - before)


class PrioritizedStep:
    """A captured step replayed from an executable instantiated with per-node priorities."""

    def __init__(self, graph, outputs, prio_exec, info):
        self.graph = graph          # torch CUDAGraph (keeps the memory pool alive)
        self.outputs = outputs
        self.prio_exec = prio_exec  # hipGraphExec_t (None: node priorities unsupported)
        self.info = info

    def replay(self):
        if self.prio_exec is None:
            return self.replay_plain()
        rc = _hip().hipGraphLaunch(_P(self.prio_exec), _P(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError("hipGraphLaunch failed (%d)" % rc)
        return self.outputs

    def replay_plain(self):
        self.graph.replay()
        return self.outputs

    __call__ = replay

    def __del__(self):
        try:
            if self.prio_exec is not None:
                _hip().hipGraphExecDestroy(_P(self.prio_exec))
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def capture_prioritized(fn: Callable[[], Any], warmup: int = 1, stream: Optional[torch.cuda.Stream] = None,
                        pool=None) -> PrioritizedStep:
    """capture() with the eager step's stream priorities kept as node priorities (see above)."""
    global _SIDE_NODES
    if not torch.cuda.is_available():
        raise RuntimeError("hipGraph capture needs a GPU")
    s = stream or torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    _SIDE_NODES = set()
    try:
        with torch.cuda.graph(g, pool=pool, stream=s):
            out = fn()
        side = _SIDE_NODES
    finally:
        _SIDE_NODES = None
    torch.cuda.synchronize()
    g.instantiate()
    hip = _hip()
    lo, hi = torch.cuda.Stream.priority_range()
    raw = g.raw_cuda_graph()
    info = {"kernel_nodes": 0, "side_kernel_nodes": 0, "set_rc": {}}
    ok = True
    for nd in graph_nodes(raw):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(_P(nd), ctypes.byref(t))
        if t.value != _KERNEL_NODE:
            continue
        info["kernel_nodes"] += 1
        is_side = nd in side
        info["side_kernel_nodes"] += int(is_side)
        v = (ctypes.c_char * 64)()
        ctypes.cast(v, ctypes.POINTER(ctypes.c_int))[0] = lo if is_side else hi
        rc = hip.hipGraphKernelNodeSetAttribute(_P(nd), _ATTR_PRIORITY, v)
        info["set_rc"][rc] = info["set_rc"].get(rc, 0) + 1
        ok = ok and rc == 0
    ex = None
    if ok and info["kernel_nodes"]:
        e = _P(0)
        rc = hip.hipGraphInstantiateWithFlags(ctypes.byref(e), _P(raw), ctypes.c_ulonglong(_FLAG_USE_NODE_PRIORITY))
        info["instantiate_rc"] = rc
        if rc == 0:
            ex = e.value
    info["set_rc"] = {str(k): v for k, v in info["set_rc"].items()}
    return PrioritizedStep(g, out, ex, info)
