"""Failure detection and fault injection.

The reference gets failure handling for free from TF1's gRPC runtime: a dead parameter
server surfaces as UnavailableError and MonitoredTrainingSession re-creates the session and
restores the latest checkpoint (/root/reference/distribute_training.py:209-215). It has no
detector of its own: a worker blocked in the SyncReplicas token dequeue
(distribute_training.py:144-148) waits forever when the chief or a PS dies.

This module adds the two pieces the survey asks for:

* `Heartbeat` — a background thread that pings every PS task of a `PSClient` on its own
  connection. After `max_missed` consecutive failed pings the task is declared dead:
  `on_failure(task)` runs and every blocking call of the client (token dequeue, take) is
  cancelled so the blocked thread raises UnavailableError instead of hanging — which the
  recoverable session then turns into a session re-creation. `HeartbeatHook` wires it into
  MonitoredTrainingSession and fails the next `run()` fast with UnavailableError.
* `FaultInjector` — deterministic faults for tests: fail or delay selected PS RPCs of a
  client (by op code and call index), or raise a preemption error at a chosen global step
  through `FaultInjectionHook`. Nothing here is active unless installed explicitly.

RCCL failures (an aborted communicator, a peer that died) are mapped to UnavailableError by
`as_preemption_error` so the same recovery path covers the all-reduce strategies.
"""
from __future__ import annotations

import random
import threading
import time
from typing import Callable, Dict, List, Optional

from ..utils import errors


class Heartbeat:
    def __init__(self, client, interval: float = 1.0, max_missed: int = 3, timeout_ms: int = 2000,
                 on_failure: Optional[Callable[[int], None]] = None):
        from .ps import PSConnection
        self.client = client
        self.interval = float(interval)
        self.max_missed = int(max_missed)
        self.timeout_ms = int(timeout_ms)
        self.on_failure = on_failure
        self.missed = [0] * client.n_ps
        self.last_seen = [time.time()] * client.n_ps
        self.dead: List[int] = []
        self._conns: Dict[int, Optional[PSConnection]] = {}
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    @property
    def healthy(self) -> bool:
        return not self.dead

    def _ping(self, task: int) -> bool:
        from . import ps as PS
        c = self._conns.get(task)
        try:
            if c is None:
                c = PS.PSConnection(self.client.cluster.task_address("ps", task), connect_timeout=0.0)
                self._conns[task] = c
            st, _ = c.call(PS.OP_PING, timeout_ms=self.timeout_ms)
            return st == PS.ST_OK
        except errors.OpError:
            if c is not None:
                c.close()
            self._conns[task] = None
            return False

    def check_once(self):
        """One round of pings (the thread body; callable directly from tests)."""
        for t in range(self.client.n_ps):
            if t in self.dead:
                continue
            if self._ping(t):
                self.missed[t] = 0
                self.last_seen[t] = time.time()
                continue
            self.missed[t] += 1
            if self.missed[t] >= self.max_missed:
                self.dead.append(t)
                self.client.cancel_blocking()
                if self.on_failure is not None:
                    self.on_failure(t)

    def _run(self):
        while not self._stop.wait(self.interval):
            self.check_once()

    def start(self) -> "Heartbeat":
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="ps-heartbeat", daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5 * self.interval + 1)
            self._thread = None
        for c in self._conns.values():
            if c is not None:
                c.close()
        self._conns.clear()


class FaultInjector:
    """Deterministic RPC faults on a PSClient's connections.

    rules are checked in order for every call; a matching `fail` rule raises `error` (default
    UnavailableError, i.e. a preemption) before the request is sent, a `delay` rule sleeps.
    `at` selects 0-based indices among the calls the rule matches (by op code, or all)."""

    def __init__(self, seed: int = 0):
        self.rules: List[dict] = []
        self.log: List[tuple] = []
        self._installed: List[tuple] = []
        self._rng = random.Random(seed)
        self._lock = threading.Lock()

    def fail(self, op: Optional[int] = None, at=(0,), error=errors.UnavailableError, prob: float = 0.0):
        self.rules.append({"kind": "fail", "op": op, "at": set(at or ()), "error": error, "prob": prob, "seen": 0})
        return self

    def delay(self, seconds: float, op: Optional[int] = None, at=None, prob: float = 1.0):
        self.rules.append({"kind": "delay", "op": op, "at": None if at is None else set(at), "sec": seconds,
                           "prob": prob, "seen": 0})
        return self

    def _before(self, address: str, op: int):
        for r in self.rules:
            if r["op"] is not None and r["op"] != op:
                continue
            with self._lock:
                i = r["seen"]
                r["seen"] += 1
                hit = (r["at"] is not None and i in r["at"]) or (r["prob"] > 0 and self._rng.random() < r["prob"])
            if not hit:
                continue
            self.log.append((r["kind"], address, op, i))
            if r["kind"] == "fail":
                raise r["error"]("injected fault: op %d call %d to %s" % (op, i, address))
            time.sleep(r["sec"])

    def install(self, client) -> "FaultInjector":
        conns = list(client.conns) + list(client._blocking.values())
        orig_blocking = client.blocking_conn

        def blocking_conn(task, purpose="dequeue"):
            c = orig_blocking(task, purpose)
            self._wrap(c)
            return c
        client.blocking_conn = blocking_conn
        self._installed.append((client, "blocking_conn", orig_blocking))
        for c in conns:
            self._wrap(c)
        return self

    def _wrap(self, conn):
        if getattr(conn, "_fault_injector", None) is self:
            return
        orig = conn.call

        def call(op, segs=(), timeout_ms=60000):
            self._before(conn.address, op)
            return orig(op, segs, timeout_ms)
        conn.call = call
        conn._fault_injector = self
        self._installed.append((conn, "call", orig))

    def uninstall(self):
        for obj, attr, orig in reversed(self._installed):
            setattr(obj, attr, orig)
            if attr == "call":
                obj._fault_injector = None
        self._installed.clear()


def as_preemption_error(exc: BaseException) -> BaseException:
    """Map a collective-backend failure (RCCL/gloo communicator error, aborted or timed-out
    work) to UnavailableError so MonitoredTrainingSession's recovery treats it like a lost
    parameter server; anything else is returned unchanged."""
    if isinstance(exc, errors.OpError):
        return exc
    import torch.distributed as dist
    backend_err = getattr(dist, "DistBackendError", None)
    msg = str(exc)
    if (backend_err is not None and isinstance(exc, backend_err)) or any(
            s in msg for s in ("NCCL", "RCCL", "Connection reset", "Connection closed", "Gloo", "gloo",
                                 "timed out", "aborted", "closed by peer")):
        err = errors.UnavailableError("collective failed: %s" % msg)
        err.__cause__ = exc
        return err
    return exc


def _hook_base():
    from ..train.hooks import SessionRunHook
    return SessionRunHook


class HeartbeatHook(_hook_base()):
    """Starts a Heartbeat on the session's PS client; a dead PS fails the next run() with
    UnavailableError (-> session re-creation) instead of letting it block."""

    def __init__(self, client_fn: Callable[[], object], interval: float = 1.0, max_missed: int = 3):
        self.client_fn = client_fn
        self.interval = interval
        self.max_missed = max_missed
        self.heartbeat: Optional[Heartbeat] = None

    def after_create_session(self, session, coord):
        if self.heartbeat is not None:
            self.heartbeat.stop()
        client = self.client_fn()
        self.heartbeat = Heartbeat(client, self.interval, self.max_missed).start() if client is not None else None

    def before_run(self, run_context):
        if self.heartbeat is not None and not self.heartbeat.healthy:
            dead = list(self.heartbeat.dead)
            raise errors.UnavailableError("parameter server task(s) %s stopped answering heartbeats" % dead)
        return None

    def end(self, session):
        if self.heartbeat is not None:
            self.heartbeat.stop()
            self.heartbeat = None


class FaultInjectionHook(_hook_base()):
    """Raises `error` (a preemption by default) once, in the first run() that starts at or
    past global step `at_step` — the in-process equivalent of killing a task at step k.
    `action` (e.g. SIGKILL a parameter-server process) runs first."""

    def __init__(self, at_step: int, error=errors.AbortedError, action: Optional[Callable[[], None]] = None):
        self.at_step = int(at_step)
        self.error = error
        self.action = action
        self.fired = False

    def begin(self):
        from ..train import graph as G
        self._gs = G.get_global_step()
        if self._gs is None:
            raise RuntimeError("global step must be created to use FaultInjectionHook")

    def before_run(self, run_context):
        if self.fired:
            return None
        gs = int(self._gs.value())
        if gs >= self.at_step:
            self.fired = True
            if self.action is not None:
                self.action()
            if self.error is not None:
                raise self.error("injected preemption at global step %d" % gs)
        return None
