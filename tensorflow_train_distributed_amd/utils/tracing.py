"""Tracing and numerics debugging.

The reference has no tracing beyond `log_device_placement=False` and its wall-clock
`sec/batch` print (/root/reference/distribute_training.py:202,229-235). Here:

* `range(name)` / `@traced` — roctx ranges (libroctx64, pushed/popped on the host thread)
  around step phases. `rocprofv3 --marker-trace` shows them on the timeline next to the HIP
  kernels; without the library (CPU box) they are no-ops. The ResNet/BERT engines and the
  optimizer tag their phases with them when `TTD_ROCTX=1`.
* `check_numerics(t, message)` — tf.debugging.check_numerics: raises InvalidArgumentError
  when a tensor holds NaN or Inf (a host sync: debugging only).
* `CheckNumericsHook` — checks every trainable gradient / variable of a FlatParams store
  after each run (one fused finite-check over the flat buffer, not per tensor).
* `launch_blocking()` — whether HIP kernels run synchronously (`HIP_LAUNCH_BLOCKING=1`), the
  mode to use when hunting the kernel behind an asynchronous fault.
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import os
from typing import Optional

import torch

from . import errors

_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


def enabled() -> bool:
    return os.environ.get("TTD_ROCTX", "0") == "1" and _lib() is not None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _lib() if enabled() else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str):
    lib = _lib() if enabled() else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


def traced(name: Optional[str] = None):
    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*a, **kw):
            with range(label):
                return fn(*a, **kw)
        return wrapper
    return deco


def check_numerics(tensor: torch.Tensor, message: str = "") -> torch.Tensor:
    """tf.debugging.check_numerics: returns `tensor` unchanged or raises InvalidArgumentError
    naming the first kind of bad value found (NaN before Inf)."""
    t = tensor.detach()
    if not t.is_floating_point():
        return tensor
    if bool(torch.isnan(t).any()):
        raise errors.InvalidArgumentError("%s : Tensor had NaN values" % message)
    if bool(torch.isinf(t).any()):
        raise errors.InvalidArgumentError("%s : Tensor had Inf values" % message)
    return tensor


def launch_blocking() -> bool:
    return os.environ.get("HIP_LAUNCH_BLOCKING", "0") == "1" or os.environ.get("CUDA_LAUNCH_BLOCKING", "0") == "1"


def _hook_base():
    from ..train.hooks import SessionRunHook
    return SessionRunHook


class CheckNumericsHook(_hook_base()):
    """After every run (or every `every_n_steps`), checks the flat gradient and master buffers
    of `params` (a FlatParams) for NaN/Inf and raises InvalidArgumentError naming the first
    offending variable."""

    def __init__(self, params, every_n_steps: int = 1, check_vars: bool = True):
        self.params = params
        self.every = max(1, int(every_n_steps))
        self.check_vars = check_vars
        self._n = 0

    def after_run(self, run_context, run_values):
        self._n += 1
        if self._n % self.every:
            return
        bufs = [("gradient", self.params.grad)] + ([("variable", self.params.master)] if self.check_vars else [])
        for kind, buf in bufs:
            if bool(torch.isfinite(buf).all()):
                continue
            for s in self.params.specs:  # locate the variable (slow path, only on failure)
                t = (self.params.g if kind == "gradient" else self.params.var)[s.name]
                if not bool(torch.isfinite(t).all()):
                    raise errors.InvalidArgumentError("%s of %s has NaN/Inf values" % (kind, s.name))
            raise errors.InvalidArgumentError("%s buffer has NaN/Inf values" % kind)
