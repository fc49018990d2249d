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
