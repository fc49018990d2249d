"""Direct xGMI all-reduce for the small gradient buckets (csrc/kernels/ipc_allreduce.hip).

Every rank of a single-node group allocates staging buffers, exports their IPC handles, and maps
every peer's (hipIpcOpenMemHandle); a bucket all-reduce is then ONE kernel on the communicator
stream that reads the peers' staged data over the point-to-point xGMI links:

  one-shot  (<= 1 MB)  each rank sums the whole bucket from all peers (1 flag barrier);
  two-shot  (<= 8 MB)  reduce-scatter + all-gather through the peers' buffers (2 barriers);
  RCCL      (larger)   the ring / tree engine (rccl.py) keeps the bandwidth-bound buckets.

`choose()` is the per-bucket decision (ipc_plan.h; CPU-tested through libttd_rt.so). The
reducer (collective.BucketedAllReducer) uses this path for its first and last buckets — the
first so communication starts with no ring latency, the last because nothing of the backward
is left to hide it — and records the path of every bucket (`bucket_paths`, in the bench JSON).
Reference aggregation: /root/reference/distribute_training.py:142-148 (PS accumulators; the
Mirrored strategies' all-reduce is the north star's, BASELINE.json).

Failure contract: a barrier whose peer does not arrive within the spin bound (TTD_IPC_SPIN polls,
~1-2 s by default) sets a host-mapped error word and its workgroup writes NaN over its share of
the bucket instead of a sum; every later call of that engine poisons without waiting. The
reducer checks the word at its join points (no device sync) and raises UnavailableError, which
MonitoredTrainingSession turns into a recovery (reference:
/root/reference/distribute_training.py:209-215). A late peer therefore never yields a wrong sum.

Environment: TTD_IPC_AR=1 enables the path (opt-in: it has run on one GPU with two processes,
never on several GPUs); TTD_IPC_AR_CAP_MB sets the staging buffer size (default 8 MB: the
two-shot limit); TTD_IPC_SPIN the barrier poll bound.
"""
from __future__ import annotations

import ctypes
import os
import socket
from ctypes import c_char_p, c_int, c_longlong, c_void_p
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native
from ..utils import errors

RCCL, ONE_SHOT, TWO_SHOT = 0, 1, 2
ONE_SHOT_MAX = 1 << 20  # ipc_plan.h kOneShotMax
PATH_NAMES = {RCCL: "rccl", ONE_SHOT: "ipc_oneshot", TWO_SHOT: "ipc_twoshot"}
HANDLE_BYTES = 128  # data + flags hipIpcMemHandle_t

_bound = False


def _hip():
    global _bound
    lib = _native.hip()
    if not _bound:
        lib.ttdi_create.restype = c_void_p
        lib.ttdi_create.argtypes = [c_int, c_int, c_int, c_longlong, c_longlong]
        lib.ttdi_handle.restype = c_int
        lib.ttdi_handle.argtypes = [c_void_p, c_char_p]
        lib.ttdi_open.restype = c_int
        lib.ttdi_open.argtypes = [c_void_p, c_char_p, ctypes.POINTER(c_int)]
        lib.ttdi_allreduce.restype = c_int
        lib.ttdi_allreduce.argtypes = [c_void_p, c_void_p, c_longlong, c_int, c_int, c_int, c_void_p]
        lib.ttdi_link_local.restype = c_int
        lib.ttdi_link_local.argtypes = [c_void_p, c_void_p]
        lib.ttdi_error.restype = c_int
        lib.ttdi_error.argtypes = [c_void_p]
        lib.ttdi_clear_error.restype = None
        lib.ttdi_clear_error.argtypes = [c_void_p]
        lib.ttdi_destroy.restype = None
        lib.ttdi_destroy.argtypes = [c_void_p]
        _bound = True
    return lib


def _rt():
    lib = _native.rt()
    lib.ttd_ipc_choose.restype = c_int
    lib.ttd_ipc_choose.argtypes = [c_longlong, c_int, c_int, c_longlong]
    lib.ttd_ipc_chunk.restype = None
    lib.ttd_ipc_chunk.argtypes = [c_longlong, c_int, c_int, c_int, ctypes.POINTER(c_longlong),
                                  ctypes.POINTER(c_longlong)]
    lib.ttd_ipc_part.restype = None
    lib.ttd_ipc_part.argtypes = [c_longlong, c_longlong, c_int, c_int, c_int, ctypes.POINTER(c_longlong),
                                 ctypes.POINTER(c_longlong)]
    lib.ttd_ipc_blocks.restype = c_int
    lib.ttd_ipc_blocks.argtypes = [c_longlong, c_int]
    return lib


def default_cap() -> int:
    return int(float(os.environ.get("TTD_IPC_AR_CAP_MB", "8")) * (1 << 20))


def enabled() -> bool:
    return os.environ.get("TTD_IPC_AR", "0") == "1"


def default_spin() -> int:
    """Barrier polls before a peer counts as lost (0: the kernel default, ~1-2 s)."""
    return int(os.environ.get("TTD_IPC_SPIN", "0"))


def choose(nbytes: int, world: int, same_node: bool, cap: Optional[int] = None) -> int:
    """Path of one bucket: RCCL, ONE_SHOT or TWO_SHOT (ipc_plan.h choose)."""
    return int(_rt().ttd_ipc_choose(int(nbytes), int(world), 1 if same_node else 0,
                                    int(default_cap() if cap is None else cap)))


def chunk(count: int, vec: int, world: int, r: int):
    lo, hi = c_longlong(), c_longlong()
    _rt().ttd_ipc_chunk(int(count), int(vec), int(world), int(r), ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def part(lo: int, hi: int, vec: int, nb: int, b: int):
    a, e = c_longlong(), c_longlong()
    _rt().ttd_ipc_part(int(lo), int(hi), int(vec), int(nb), int(b), ctypes.byref(a), ctypes.byref(e))
    return a.value, e.value


def blocks_for(nbytes: int, budget: int = 0) -> int:
    return int(_rt().ttd_ipc_blocks(int(nbytes), int(budget)))


def plan_paths(bucket_bytes: List[int], world: int, same_node: bool, cap: Optional[int] = None,
               edges_only: bool = True) -> List[int]:
    """Path of every bucket of a reducer: with edges_only, only the first and last buckets may
    take the direct path (the large middle ones stay on RCCL, whose ring is bandwidth-optimal)."""
    out = []
    n = len(bucket_bytes)
    for i, b in enumerate(bucket_bytes):
        if edges_only and 0 < i < n - 1:
            out.append(RCCL)
        else:
            out.append(choose(b, world, same_node, cap))
    return out


def group_same_node(group=None) -> bool:
    """Every rank of `group` runs on this host (its peers' GPU memory is mappable)."""
    if not dist.is_initialized():
        return True
    names: List[Optional[str]] = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


class LocalGroup:
    """Every rank of a `world`-rank group as engines of THIS process on one device, peers linked
    by plain pointers (no IPC): tests run the ranks' kernels on separate streams."""

    def __init__(self, world: int, device=None, cap_bytes: Optional[int] = None, spin: Optional[int] = None,
                 max_blocks: int = 0):
        lib = _hip()
        self.world = world
        self.max_blocks = int(max_blocks)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cap = int(default_cap() if cap_bytes is None else cap_bytes)
        self.h = []
        with torch.cuda.device(self.device):
            for r in range(world):
                h = lib.ttdi_create(r, world, self.device.index, self.cap, int(default_spin() if spin is None else spin))
                if not h:
                    self.destroy()
                    raise errors.UnavailableError("ttdi_create failed")
                self.h.append(h)
        for a in range(world):
            for b in range(world):
                if a != b and lib.ttdi_link_local(self.h[a], self.h[b]) != 0:
                    self.destroy()
                    raise errors.InternalError("ttdi_link_local failed")

    def all_reduce_(self, r: int, t: torch.Tensor, path: int, stream) -> torch.Tensor:
        rc = _hip().ttdi_allreduce(self.h[r], t.data_ptr(), t.numel(), 0 if t.dtype == torch.float32 else 1,
                                   int(path), self.max_blocks, stream.cuda_stream)
        if rc != 0:
            raise errors.InternalError("ipc all-reduce launch failed (hipError %d)" % rc)
        return t

    def timed_out(self) -> bool:
        return any(_hip().ttdi_error(h) != 0 for h in self.h)

    def clear_error(self):
        for h in self.h:
            _hip().ttdi_clear_error(h)

    def destroy(self):
        for h in self.h:
            _hip().ttdi_destroy(h)
        self.h = []


class IpcAllReducer:
    """The staging buffers and peer mappings of one group; `all_reduce_(t, path, stream)` runs
    one bucket. Collective construction: every rank of `group` must create it together."""

    def __init__(self, group=None, device=None, cap_bytes: Optional[int] = None, spin: Optional[int] = None,
                 max_blocks: int = 0):
        """max_blocks: workgroups per launch at most (the collectives' CTA budget; 0: no cap
        beyond ipc_plan.h's 64). spin: barrier polls before a peer counts as lost."""
        lib = _hip()
        self.group = group
        self.max_blocks = int(max_blocks)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cap = int(default_cap() if cap_bytes is None else cap_bytes)
        with torch.cuda.device(self.device):
            h = lib.ttdi_create(self.rank, self.world, self.device.index, self.cap,
                                int(default_spin() if spin is None else spin))
        self._h = h
        # every rank learns whether any rank failed, so all of them raise together
        ok = self._all_ok(bool(h))
        if not ok:
            self.destroy()
            raise errors.UnavailableError("IPC all-reduce staging buffers could not be allocated on some rank")
        buf = ctypes.create_string_buffer(HANDLE_BYTES)
        rc = lib.ttdi_handle(h, buf)
        mine = buf.raw if rc == 0 else b""
        if self.world > 1:
            allh: List[Optional[bytes]] = [None] * self.world
            dist.all_gather_object(allh, (mine, self.device.index), group=group)
        else:
            allh = [(mine, self.device.index)]
        if any(len(x[0]) != HANDLE_BYTES for x in allh):
            self.destroy()
            raise errors.UnavailableError("hipIpcGetMemHandle failed on some rank (rc %d here)" % rc)
        handles = b"".join(x[0] for x in allh)
        devs = (c_int * self.world)(*[int(x[1]) for x in allh])
        with torch.cuda.device(self.device):
            rc = lib.ttdi_open(h, handles, devs)
        if not self._all_ok(rc == 0):
            self.destroy()
            raise errors.UnavailableError("hipIpcOpenMemHandle failed on some rank (rc %d here)" % rc)

    def _all_ok(self, ok: bool) -> bool:
        if self.world == 1:
            return ok
        st: List[Optional[bool]] = [None] * self.world
        dist.all_gather_object(st, bool(ok), group=self.group)
        return all(st)

    def all_reduce_(self, t: torch.Tensor, path: int, stream=None) -> torch.Tensor:
        """In-place SUM of `t` (contiguous fp32 / bf16 CUDA tensor, 16-B aligned, a multiple of
        16 B) over the group through `path`, queued on `stream` (default: current)."""
        if t.dtype not in (torch.float32, torch.bfloat16) or not t.is_contiguous():
            raise ValueError("ipc all-reduce wants a contiguous fp32 / bf16 tensor")
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = _hip().ttdi_allreduce(self._h, t.data_ptr(), t.numel(), 0 if t.dtype == torch.float32 else 1, int(path),
                                   self.max_blocks, s.cuda_stream)
        if rc != 0:
            raise errors.InternalError("ipc all-reduce launch failed (hipError %d)" % rc)
        return t

    @staticmethod
    def fits(t: torch.Tensor, cap: int) -> bool:
        """The tensor can take the direct path: 16-B aligned, whole 16-B vectors, <= cap bytes."""
        nb = t.numel() * t.element_size()
        return (t.data_ptr() % 16 == 0 and nb % 16 == 0 and 0 < nb <= cap and t.is_contiguous()
                and t.dtype in (torch.float32, torch.bfloat16))

    def timed_out(self) -> bool:
        """Whether a barrier of some call that has run so far timed out (a peer never arrived):
        a host-mapped word, read without synchronising (calls still queued are not covered)."""
        return bool(self._h) and _hip().ttdi_error(self._h) != 0

    def check(self):
        """Raise UnavailableError when a call has failed (its bucket holds NaN, not a sum)."""
        if self.timed_out():
            raise errors.UnavailableError(
                "direct xGMI all-reduce: a peer did not reach a barrier within the spin bound (lost or "
                "stalled rank); the affected gradient bucket was poisoned with NaN, not summed")

    def clear_error(self):
        if self._h:
            _hip().ttdi_clear_error(self._h)

    def destroy(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            _hip().ttdi_destroy(h)

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
