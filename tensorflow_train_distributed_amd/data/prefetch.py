"""Python side of the native batch prefetcher (csrc/runtime/prefetch.cc) and an async
host->device copier.

NativeBatchPrefetcher: a C++ thread gathers shuffled batches (TF next_batch epoch
semantics) into a ring of host buffers, off the Python GIL.
DevicePrefetcher: overlaps the H2D copy of batch k+1 (pinned memory, side HIP stream)
with compute on batch k.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _native


def _lib():
    lib = _native.rt()
    if not getattr(lib, "_pf_sigs", False):
        lib.ttd_prefetch_create.restype = ctypes.c_void_p
        lib.ttd_prefetch_create.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
        lib.ttd_prefetch_next.restype = ctypes.c_int64
        lib.ttd_prefetch_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.ttd_prefetch_destroy.argtypes = [ctypes.c_void_p]
        lib._pf_sigs = True
    return lib


class NativeBatchPrefetcher:
    def __init__(self, images: np.ndarray, labels: np.ndarray, batch: int, depth: int = 4, seed: int = 0):
        self.images = np.ascontiguousarray(images)
        self.labels = np.ascontiguousarray(labels)
        n = self.images.shape[0]
        self.batch = batch
        self._xshape = (batch,) + self.images.shape[1:]
        self._yshape = (batch,) + self.labels.shape[1:]
        xrow = self.images.nbytes // n
        yrow = self.labels.nbytes // n
        self._h = _lib().ttd_prefetch_create(self.images.ctypes.data, self.labels.ctypes.data, n, xrow, yrow, batch,
                                             depth, seed)
        if not self._h:
            raise RuntimeError(_native.rt_error())

    def next(self):
        x = np.empty(self._xshape, dtype=self.images.dtype)
        y = np.empty(self._yshape, dtype=self.labels.dtype)
        ep = _lib().ttd_prefetch_next(self._h, x.ctypes.data, y.ctypes.data)
        return x, y, int(ep)

    def close(self):
        if self._h:
            _lib().ttd_prefetch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DevicePrefetcher:
    """Wraps an iterator of host batches (tuples/dicts of arrays); yields device tensors
    whose H2D copy was issued one step ahead on a side stream."""

    def __init__(self, it, device):
        self.it = iter(it)
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._next = None
        self._preload()

    def _to_dev(self, v):
        t = torch.as_tensor(v)
        if self.stream is None:
            return t
        if not t.is_pinned():
            t = t.pin_memory()
        return t.to(self.device, non_blocking=True)

    def _preload(self):
        try:
            b = next(self.it)
        except StopIteration:
            self._next = None
            return
        if self.stream is None:
            self._next = b
            return
        with torch.cuda.stream(self.stream):
            if isinstance(b, dict):
                self._next = {k: self._to_dev(v) for k, v in b.items()}
            else:
                self._next = tuple(self._to_dev(v) for v in b)

    def __iter__(self):
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        b = self._next
        self._preload()
        return b
