"""Parameter-server runtime (Python side of csrc/runtime/ps_server.cc).

Covers the reference's TF1 distributed runtime surface:
* `Server(cluster, job_name, task_index)` / `.join()` / `.target`
  (/root/reference/distribute_training.py:175-181,209): a `ps` task runs the native C++
  variable server (TCP, one thread per connection); `join()` blocks until a Shutdown RPC;
* `replica_device_setter(worker_device, cluster)` (:186-188): round-robin placement of
  variables over PS tasks (the global step goes first, on ps task 0);
* `PSClient`: the data plane a worker uses instead of TF's Send/Recv partitions — Pull
  (PS -> worker weights), ApplyGD (Hogwild async update + global_step += 1),
  AccumApply / TakeApply / token dequeue+enqueue (SyncReplicasOptimizer), Save/Restore of
  each task's shard, readiness (session-creation barrier), Shutdown.
A dead PS surfaces as `UnavailableError` so MonitoredTrainingSession can re-create the
session and restore from the latest checkpoint.
"""
from __future__ import annotations

import ctypes
import struct
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native
from ..utils import errors
from .cluster import ClusterSpec, split_address

# wire ops (must match ps_server.cc)
OP_PING, OP_INIT, OP_IS_READY, OP_SET_READY, OP_PULL, OP_APPLY_GD, OP_ACCUM_APPLY, OP_TAKE_APPLY = 1, 2, 3, 4, 5, 6, 7, 8
OP_DEQUEUE, OP_ENQUEUE, OP_CLOSE_QUEUE, OP_GET_GS, OP_SET_GS, OP_SET_ACCUM_STEP = 9, 10, 11, 12, 13, 14
OP_SAVE, OP_RESTORE, OP_SHUTDOWN, OP_LIST, OP_STATS, OP_COUNTER_ADD = 15, 16, 17, 18, 19, 20
ST_OK, ST_ERR, ST_CLOSED, ST_NOT_FOUND, ST_SHUTTING_DOWN = 0, 1, 2, 3, 4

DT_FLOAT, DT_INT64 = 1, 9


def _lib():
    lib = _native.rt()
    if not getattr(lib, "_ps_sigs", False):
        vp = ctypes.c_void_p
        lib.ttd_ps_server_start.restype = vp
        lib.ttd_ps_server_start.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        lib.ttd_ps_server_port.argtypes = [vp]
        lib.ttd_ps_server_join.argtypes = [vp]
        lib.ttd_ps_server_stop.argtypes = [vp]
        lib.ttd_ps_server_stopping.argtypes = [vp]
        lib.ttd_ps_server_destroy.argtypes = [vp]
        lib.ttd_ps_client_connect.restype = vp
        lib.ttd_ps_client_connect.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        lib.ttd_ps_client_call.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(vp),
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        lib.ttd_ps_client_resp.restype = vp
        lib.ttd_ps_client_resp.argtypes = [vp]
        lib.ttd_ps_client_resp_len.restype = ctypes.c_uint64
        lib.ttd_ps_client_resp_len.argtypes = [vp]
        lib.ttd_ps_client_close.argtypes = [vp]
        lib.ttd_ps_client_abort.argtypes = [vp]
        lib._ps_sigs = True
    return lib


# ------------------------------------------------------------------ server
_SERVERS: Dict[str, "Server"] = {}


class Server:
    """tf.train.Server equivalent. For job "ps" it hosts the native variable server on this
    task's port; for "worker" it only records the cluster so `MonitoredTrainingSession(
    master=server.target)` can find the parameter servers."""

    def __init__(self, server_or_cluster_def, job_name: Optional[str] = None, task_index: int = 0,
                 start: bool = True, bind_host: str = "0.0.0.0", config=None):
        self.cluster = ClusterSpec(server_or_cluster_def)
        self.job_name = job_name
        self.task_index = int(task_index)
        self._h = None
        self.port = None
        if job_name == "ps":
            _, port = split_address(self.cluster.task_address("ps", self.task_index))
            if start:
                self.start(bind_host, port)
        self.target = "ttd://%s/%d@%x" % (job_name, self.task_index, id(self))
        _SERVERS[self.target] = self

    def start(self, bind_host="0.0.0.0", port=None):
        if self._h:
            return
        if port is None:
            _, port = split_address(self.cluster.task_address("ps", self.task_index))
        h = _lib().ttd_ps_server_start(bind_host.encode(), int(port), self.task_index)
        if not h:
            raise errors.UnavailableError("cannot start PS task %d: %s" % (self.task_index, _native.rt_error()))
        self._h = h
        self.port = _lib().ttd_ps_server_port(h)

    def join(self):
        """Blocks until a Shutdown RPC (the reference's `server.join()` never returned)."""
        if self._h:
            _lib().ttd_ps_server_join(self._h)

    def stop(self):
        if self._h:
            _lib().ttd_ps_server_destroy(self._h)
            self._h = None

    @staticmethod
    def create_local_server(config=None, start=True):
        return Server(ClusterSpec({"localhost": ["localhost:0"]}), "localhost", 0)


def server_for_target(target: str) -> Optional[Server]:
    return _SERVERS.get(target)


# ------------------------------------------------------------------ client
class PSConnection:
    """One TCP connection to one PS task (thread-safe, calls are serialised)."""

    def __init__(self, address: str, connect_timeout: float = 30.0, retry_interval: float = 0.2):
        self.address = address
        host, port = split_address(address)
        deadline = time.time() + connect_timeout
        lib = _lib()
        while True:
            h = lib.ttd_ps_client_connect(host.encode(), port, 10000)
            if h:
                break
            if time.time() >= deadline:
                raise errors.UnavailableError("PS %s unreachable: %s" % (address, _native.rt_error()))
            time.sleep(retry_interval)
        self._h = h
        self._lock = threading.Lock()

    def call(self, op: int, segs: Sequence = (), timeout_ms: int = 60000) -> Tuple[int, bytes]:
        """segs: bytes objects or (ptr, nbytes) tuples, sent back to back as the body."""
        keep = []
        ptrs = (ctypes.c_void_p * max(1, len(segs)))()
        lens = (ctypes.c_uint64 * max(1, len(segs)))()
        for i, s in enumerate(segs):
            if isinstance(s, (bytes, bytearray)):
                b = ctypes.create_string_buffer(bytes(s), len(s))
                keep.append(b)
                ptrs[i], lens[i] = ctypes.addressof(b), len(s)
            else:
                ptrs[i], lens[i] = s[0], s[1]
        lib = _lib()
        with self._lock:
            if self._h is None:
                raise errors.UnavailableError("connection to %s closed" % self.address)
            st = lib.ttd_ps_client_call(self._h, op, len(segs), ptrs, lens, timeout_ms)
            if st < 0:
                raise errors.UnavailableError("PS %s: %s" % (self.address, _native.rt_error()))
            n = lib.ttd_ps_client_resp_len(self._h)
            body = ctypes.string_at(lib.ttd_ps_client_resp(self._h), n) if n else b""
        return st, body

    def abort(self):
        """Cancel a call blocked on another thread (it raises UnavailableError)."""
        h = self._h
        if h is not None:
            _lib().ttd_ps_client_abort(h)

    def close(self):
        self.abort()
        with self._lock:
            if self._h is not None:
                _lib().ttd_ps_client_close(self._h)
                self._h = None


def _name(n: str) -> bytes:
    b = n.encode()
    return struct.pack("<H", len(b)) + b


def _check(st, body, what):
    if st == ST_OK:
        return body
    if st == ST_CLOSED:
        raise errors.OutOfRangeError("%s: queue closed" % what)
    if st == ST_NOT_FOUND:
        raise errors.NotFoundError("%s: variable %s not found on PS" % (what, body.decode(errors="replace")))
    if st == ST_SHUTTING_DOWN:
        raise errors.AbortedError("%s: PS shutting down" % what)
    raise errors.InternalError("%s failed (status %d) %s" % (what, st, body[:200]))


class PSClient:
    """Variable-store client spanning all PS tasks of a cluster.

    `placement[name] = ps task index` (see replica_device_setter). Host buffers are numpy
    float32 arrays addressed by variable name; the caller owns device<->host staging.
    """

    def __init__(self, cluster: ClusterSpec, placement: Dict[str, int], connect_timeout: float = 60.0):
        self.cluster = cluster
        self.placement = dict(placement)
        self.n_ps = cluster.num_tasks("ps")
        self._connect_timeout = connect_timeout
        self.conns = [PSConnection(a, connect_timeout) for a in cluster.job_tasks("ps")]
        # blocking ops (token dequeue / take) get their own connections so heartbeats and
        # other calls are not stuck behind them
        self._blocking: Dict[tuple, PSConnection] = {}
        self.by_task: List[List[str]] = [[] for _ in range(self.n_ps)]
        for n, t in self.placement.items():
            self.by_task[t].append(n)

    def blocking_conn(self, task: int, purpose: str = "dequeue") -> PSConnection:
        """Dedicated connection per (task, purpose): a worker blocked in the token dequeue
        must not hold the connection the chief's queue-runner thread takes through."""
        key = (task, purpose)
        c = self._blocking.get(key)
        if c is None:
            c = PSConnection(self.cluster.task_address("ps", task), self._connect_timeout)
            self._blocking[key] = c
        return c

    def cancel_blocking(self, purpose: Optional[str] = None):
        for (t, p), c in list(self._blocking.items()):
            if purpose is None or p == purpose:
                c.abort()

    def close(self):
        self.cancel_blocking()
        for c in self.conns + list(self._blocking.values()):
            c.close()

    # -- control
    def ping(self, task: int = 0) -> int:
        st, b = self.conns[task].call(OP_PING, timeout_ms=5000)
        return struct.unpack("<i", _check(st, b, "ping"))[0]

    def is_ready(self) -> bool:
        for c in self.conns:
            st, b = c.call(OP_IS_READY)
            if not _check(st, b, "is_ready")[0]:
                return False
        return True

    def set_ready(self, ready: bool = True):
        for c in self.conns:
            _check(*c.call(OP_SET_READY, [struct.pack("<B", 1 if ready else 0)]), "set_ready")

    def init_vars(self, values: Dict[str, np.ndarray]):
        per = [[] for _ in range(self.n_ps)]
        for name, arr in values.items():
            a = np.ascontiguousarray(arr)
            dt = DT_INT64 if a.dtype == np.int64 else DT_FLOAT
            if dt == DT_FLOAT:
                a = a.astype(np.float32, copy=False)
            hdr = _name(name) + struct.pack("<iI", dt, a.ndim) + struct.pack("<%dq" % a.ndim, *a.shape) + \
                struct.pack("<Q", a.nbytes)
            per[self.placement[name]].append((hdr, a))
        for t, items in enumerate(per):
            if not items:
                continue
            segs = [struct.pack("<I", len(items))]
            keep = []
            for hdr, a in items:
                segs.append(hdr)
                segs.append((a.ctypes.data, a.nbytes))
                keep.append(a)
            _check(*self.conns[t].call(OP_INIT, segs), "init_vars")

    def pull(self, out: Dict[str, np.ndarray]):
        """Fill out[name] (float32 host arrays) with the PS values."""
        for t, names in enumerate(self.by_task):
            names = [n for n in names if n in out]
            if not names:
                continue
            body = _check(*self.conns[t].call(OP_PULL, [struct.pack("<I", len(names))] + [_name(n) for n in names]),
                          "pull")
            off = 0
            mv = memoryview(body)
            for n in names:
                nb = struct.unpack_from("<Q", body, off)[0]
                off += 8
                dst = out[n]
                if dst.nbytes != nb:
                    raise errors.InvalidArgumentError("pull %s: %d bytes, expected %d" % (n, nb, dst.nbytes))
                dst.reshape(-1).view(np.uint8)[:] = np.frombuffer(mv[off:off + nb], dtype=np.uint8)
                off += nb

    def _grad_segs(self, names, grads):
        segs = [struct.pack("<I", len(names))]
        for n in names:
            g = grads[n]
            segs.append(_name(n) + struct.pack("<Q", g.nbytes))
            segs.append((g.ctypes.data, g.nbytes))
        return segs

    def apply_gd(self, lr: float, grads: Dict[str, np.ndarray]) -> int:
        """Async (Hogwild) ApplyGradientDescent on every PS; global_step += 1 on ps 0."""
        gs = None
        for t, names in enumerate(self.by_task):
            names = [n for n in names if n in grads]
            inc = 1 if t == 0 else 0
            if not names and not inc:
                continue
            body = _check(*self.conns[t].call(OP_APPLY_GD, [struct.pack("<fB", lr, inc)] +
                                              self._grad_segs(names, grads)), "apply_gd")
            if t == 0:
                gs = struct.unpack("<q", body)[0]
        return gs

    def accum_apply(self, local_step: int, grads: Dict[str, np.ndarray]) -> int:
        accepted = 0
        for t, names in enumerate(self.by_task):
            names = [n for n in names if n in grads]
            if not names:
                continue
            body = _check(*self.conns[t].call(OP_ACCUM_APPLY, [struct.pack("<q", local_step)] +
                                              self._grad_segs(names, grads)), "accum_apply")
            accepted += struct.unpack("<I", body)[0]
        return accepted

    def take_apply(self, num_required: int, lr: float, tokens_per_step: int, names_per_task=None) -> int:
        """Chief's sync_op: take the mean of `num_required` gradients per variable (blocking),
        apply GD, then (ps 0) global_step += 1 and enqueue `tokens_per_step` tokens."""
        by_task = names_per_task or self.by_task
        # non-global-step tasks first (in parallel), then ps 0 which finalises the step
        threads, errs = [], []

        def run(t):
            try:
                names = by_task[t]
                _check(*self.blocking_conn(t, "take").call(OP_TAKE_APPLY, [struct.pack("<IfBII", num_required, lr, 0, 0,
                                                                               len(names))] +
                                                   [_name(n) for n in names], timeout_ms=0), "take_apply")
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        for t in range(1, self.n_ps):
            th = threading.Thread(target=run, args=(t,), daemon=True)
            th.start()
            threads.append(th)
        for th in threads:
            th.join()
        if errs:
            raise errs[0]
        names = by_task[0]
        body = _check(*self.blocking_conn(0, "take").call(OP_TAKE_APPLY, [struct.pack("<IfBII", num_required, lr, 1,
                                                                              tokens_per_step, len(names))] +
                                                  [_name(n) for n in names], timeout_ms=0), "take_apply")
        return struct.unpack("<q", body)[0]

    def dequeue_token(self) -> int:
        st, b = self.blocking_conn(0).call(OP_DEQUEUE, timeout_ms=0)
        return struct.unpack("<q", _check(st, b, "dequeue_token"))[0]

    def enqueue_tokens(self, n: int, value: int):
        _check(*self.conns[0].call(OP_ENQUEUE, [struct.pack("<Iq", n, value)]), "enqueue_tokens")

    def close_queue(self):
        _check(*self.conns[0].call(OP_CLOSE_QUEUE), "close_queue")

    def global_step(self) -> int:
        return struct.unpack("<q", _check(*self.conns[0].call(OP_GET_GS), "global_step"))[0]

    def set_global_step(self, v: int):
        _check(*self.conns[0].call(OP_SET_GS, [struct.pack("<q", int(v))]), "set_global_step")

    def set_accum_step(self, v: int):
        for c in self.conns:
            _check(*c.call(OP_SET_ACCUM_STEP, [struct.pack("<q", int(v))]), "set_accum_step")

    def counter_add(self, name: str, delta: int = 1, task: int = 0) -> int:
        """Atomically add to a named int64 counter on a PS task; returns the new value."""
        return struct.unpack("<q", _check(*self.conns[task].call(OP_COUNTER_ADD, [_name(name) +
                                                                                  struct.pack("<q", delta)]),
                                           "counter_add"))[0]

    def stats(self, task: int = 0) -> dict:
        d, s, q = struct.unpack("<qqq", _check(*self.conns[task].call(OP_STATS), "stats"))
        return {"dropped": d, "accum_step": s, "queue": q}

    def save_shard(self, task: int, prefix: str, shard: int = 0, num_shards: int = 1, with_global_step=None):
        wgs = (task == 0) if with_global_step is None else with_global_step
        _check(*self.conns[task].call(OP_SAVE, [_name(prefix) + struct.pack("<iiB", shard, num_shards, 1 if wgs else 0)],
                                      timeout_ms=0), "save")

    def restore(self, prefix: str) -> int:
        total = 0
        for c in self.conns:
            body = _check(*c.call(OP_RESTORE, [_name(prefix)], timeout_ms=0), "restore")
            total += struct.unpack("<I", body)[0]
        return total

    def shutdown(self):
        for c in self.conns:
            try:
                c.call(OP_SHUTDOWN, timeout_ms=5000)
            except errors.OpError:
                pass


# ------------------------------------------------------------------ placement
class DeviceSetter:
    """Result of replica_device_setter: assigns each variable (in creation order) to a PS
    task round-robin (TF's _RoundRobinStrategy); ops stay on `worker_device`."""

    def __init__(self, cluster: ClusterSpec, worker_device: str, ps_tasks: int, strategy=None):
        self.cluster = cluster
        self.worker_device = worker_device
        self.ps_tasks = ps_tasks
        self._next = 0
        self.strategy = strategy
        self.placement: Dict[str, int] = {}

    def assign(self, name: str, nbytes: int = 0) -> int:
        if name in self.placement:
            return self.placement[name]
        if self.ps_tasks == 0:
            return -1
        if self.strategy is not None:
            t = self.strategy(name, nbytes)
        else:
            t = self._next % self.ps_tasks
            self._next += 1
        self.placement[name] = t
        return t

    def device_for(self, name: str) -> str:
        t = self.placement.get(name)
        return self.worker_device if t is None else "/job:ps/task:%d" % t


class GreedyLoadBalancingStrategy:
    """tf.contrib.training.GreedyLoadBalancingStrategy: place each variable on the PS task
    with the fewest bytes so far."""

    def __init__(self, num_tasks: int):
        self.load = [0] * num_tasks

    def __call__(self, name, nbytes):
        t = int(np.argmin(self.load))
        self.load[t] += max(1, nbytes)
        return t


def replica_device_setter(ps_tasks: int = 0, ps_device: str = "/job:ps", worker_device: str = "/job:worker",
                          merge_devices: bool = True, cluster=None, ps_ops=None, ps_strategy=None) -> DeviceSetter:
    cluster = ClusterSpec(cluster) if cluster is not None else ClusterSpec({})
    if not ps_tasks:
        ps_tasks = cluster.num_tasks("ps")
    return DeviceSetter(cluster, worker_device, ps_tasks, ps_strategy)


_device_stack = threading.local()


class device:
    """`with device(setter_or_string):` — records the active placement for variables created
    inside (models consult current_device_setter())."""

    def __init__(self, spec):
        self.spec = spec

    def __enter__(self):
        st = getattr(_device_stack, "s", None)
        if st is None:
            st = _device_stack.s = []
        st.append(self.spec)
        return self.spec

    def __exit__(self, *a):
        _device_stack.s.pop()


def current_device_setter() -> Optional[DeviceSetter]:
    for s in reversed(getattr(_device_stack, "s", []) or []):
        if isinstance(s, DeviceSetter):
            return s
    return None


# ------------------------------------------------------------------ tf-named views of the PS primitives
class TokenQueue:
    """The SyncReplicas token queue on parameter-server task 0 (tf.FIFOQueue of int64 tokens,
    shared name `sync_token_q`, distribute_training.py:144-148 via SyncReplicasOptimizer):
    enqueue_many(n, value) / dequeue() (blocks) / close() (wakes blocked dequeues with
    OutOfRangeError) / size()."""

    name = "sync_token_q"

    def __init__(self, client: PSClient):
        self.client = client

    def enqueue_many(self, n: int, value: int):
        self.client.enqueue_tokens(int(n), int(value))

    def dequeue(self) -> int:
        return self.client.dequeue_token()

    def close(self, cancel_pending_enqueues: bool = False):
        self.client.close_queue()

    def size(self) -> int:
        return self.client.stats(0)["queue"]


class ConditionalAccumulatorSet:
    """The per-variable ConditionalAccumulators of SyncReplicasOptimizer (one per trainable
    variable, on the variable's PS task): apply_grad drops gradients whose local_step is older
    than the accumulators' global step; take_apply waits for `num_required` fresh gradients,
    applies their mean with GradientDescent, bumps the global step and enqueues tokens."""

    def __init__(self, client: PSClient):
        self.client = client

    def apply_grad(self, local_step: int, grads: Dict[str, np.ndarray]) -> int:
        return self.client.accum_apply(int(local_step), grads)

    def set_global_step(self, step: int):
        self.client.set_accum_step(int(step))

    def take_apply(self, num_required: int, lr: float, tokens_per_step: int) -> int:
        return self.client.take_apply(int(num_required), float(lr), int(tokens_per_step))

    def num_dropped(self) -> int:
        return self.client.stats(0)["dropped"]
