"""Sessions: MonitoredTrainingSession and friends.

Reference: `tf.train.MonitoredTrainingSession(master=server.target, is_chief, checkpoint_dir,
hooks, save_checkpoint_secs=60, config)` + `should_stop()` / `run(fetches, feed_dict)`
(/root/reference/distribute_training.py:209-226); semantics in SURVEY.md §2.2 T14-T18, §3.5,
§5.3:
* chief: restore the latest checkpoint of checkpoint_dir (or initialise), mark the PS
  variables ready; default chief-only hooks CheckpointSaverHook / SummarySaverHook /
  StepCounterHook;
* non-chief: wait until the chief has initialised the parameter servers (recovery_wait_secs
  polling, up to max_wait_secs);
* run(): hooks' before_run fetches are merged, the TrainOp executes once, fetches are
  evaluated after the step, after_run hooks see their results;
* recovery: an UnavailableError/AbortedError (PS or collective peer lost) closes and
  re-creates the session (the chief restores from the latest checkpoint) and retries;
* close(): hooks' end() (final checkpoint) then Coordinator.join(stop_grace_period_secs).
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..utils import errors
from . import graph as G
from .hooks import (CheckpointSaverHook, SessionRunArgs, SessionRunContext, SessionRunHook, SessionRunValues,
                    StepCounterHook, SummarySaverHook)

log = logging.getLogger("tensorflow_train_distributed_amd")

USE_DEFAULT = object()


class Coordinator:
    def __init__(self, clean_stop_exception_types=(errors.OutOfRangeError,)):
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._exc = None
        self._clean = clean_stop_exception_types

    def request_stop(self, ex=None):
        if ex is not None and not isinstance(ex, self._clean) and self._exc is None:
            self._exc = ex
        self._stop.set()

    def should_stop(self) -> bool:
        return self._stop.is_set()

    def wait_for_stop(self, timeout=None) -> bool:
        return self._stop.wait(timeout)

    def clear_stop(self):
        self._stop.clear()
        self._exc = None

    def register_thread(self, t):
        self._threads.append(t)

    def raise_requested_exception(self):
        if self._exc is not None:
            raise self._exc

    def join(self, threads=None, stop_grace_period_secs=120, ignore_live_threads=False):
        threads = list(threads or []) + self._threads
        deadline = time.time() + stop_grace_period_secs
        for t in threads:
            t.join(max(0.0, deadline - time.time()))
        live = [t.name for t in threads if t.is_alive()]
        if live and not ignore_live_threads:
            log.warning("threads still running after grace period: %s", live)
        self.raise_requested_exception()

    @property
    def joined(self):
        return not any(t.is_alive() for t in self._threads)


# ---------------------------------------------------------------------------------------
def _flatten(x, out):
    if isinstance(x, dict):
        for k in sorted(x, key=str):
            _flatten(x[k], out)
    elif isinstance(x, (list, tuple)):
        for v in x:
            _flatten(v, out)
    elif x is not None:
        out.append(x)
    return out


def _pack(x, it):
    if isinstance(x, dict):
        keys = sorted(x, key=str)
        vals = {k: _pack(x[k], it) for k in keys}
        return {k: vals[k] for k in x}
    if isinstance(x, (list, tuple)):
        r = [_pack(v, it) for v in x]
        return type(x)(r) if isinstance(x, tuple) and not hasattr(x, "_fields") else (
            type(x)(*r) if hasattr(x, "_fields") else r)
    if x is None:
        return None
    return next(it)


def _host(v):
    if isinstance(v, torch.Tensor):
        return v.detach().float().item() if v.numel() == 1 else v.detach().cpu().numpy()
    return v


class _CoreSession:
    """The innermost session (tf.Session analogue): executes TrainOps and evaluates fetch
    handles. In parameter-server mode it owns the PSClient."""

    def __init__(self, graph: G.Graph, target: str = "", config=None, is_chief: bool = True,
                 checkpoint_dir: Optional[str] = None, max_wait_secs: float = 7200, recovery_wait_secs: float = 0.5,
                 scaffold=None):
        from .checkpoint import Saver
        self.graph = graph
        self.target = target
        self.config = config
        self.is_chief = is_chief
        self.checkpoint_dir = checkpoint_dir
        self.train_ops = graph.get_collection(G.TRAIN_OP)
        self.ps_ops = [op for op in self.train_ops if op.mode == "ps"]
        # all-reduce replicas (Mirrored / MultiWorkerMirrored): replica 0 restores and writes
        # checkpoints, every replica takes part in the state broadcast and the save collectives
        self.strategy = mirrored_strategy(self.train_ops)
        self.replica_id = self.strategy.replica_id if self.strategy is not None else 0
        self.client = None
        self._closed = False
        self.scaffold = scaffold
        if self.ps_ops:
            self._connect()
            self._prepare_ps(max_wait_secs, recovery_wait_secs)
        else:
            self._prepare_local()

    # -- creation
    def _cluster(self):
        from ..parallel.ps import server_for_target
        srv = server_for_target(self.target) if self.target else None
        if srv is not None and srv.cluster:
            return srv.cluster
        return self.ps_ops[0].setter.cluster

    def _connect(self):
        from ..parallel.ps import PSClient
        placement = {}
        for op in self.ps_ops:
            placement.update(op.placement)
        self.client = PSClient(self._cluster(), placement)
        for op in self.ps_ops:
            op.attach_ps(self.client)

    def _prepare_ps(self, max_wait_secs, recovery_wait_secs):
        from .checkpoint import latest_checkpoint
        c = self.client
        if self.is_chief:
            init = {}
            for op in self.ps_ops:
                init.update(op.initial_values())
            c.init_vars(init)
            c.set_global_step(0)
            ckpt = latest_checkpoint(self.checkpoint_dir) if self.checkpoint_dir else None
            if ckpt:
                n = c.restore(ckpt)
                log.info("Restored %d tensors from %s", n, ckpt)
            c.set_ready(True)
        else:
            deadline = time.time() + max_wait_secs
            while not c.is_ready():
                if time.time() > deadline:
                    raise errors.DeadlineExceededError("chief did not initialise the PS within %ss" % max_wait_secs)
                time.sleep(recovery_wait_secs)

    def _prepare_local(self):
        from .checkpoint import latest_checkpoint
        if self.checkpoint_dir and self.replica_id == 0:
            ckpt = latest_checkpoint(self.checkpoint_dir)
            if ckpt:
                self.default_saver().restore(None, ckpt, strict=False)
                log.info("Restored from %s", ckpt)
        if self.strategy is not None:
            # replica 0's (restored or initial) weights, optimizer slots and global step
            from ..parallel.collective import broadcast_state_
            for op in self.train_ops:
                if op.mode == "mirrored":
                    broadcast_state_(op.params, op.flat, group=self.strategy.group)
                    op.reducer = None  # rebuilt against the current process group on first use

    @property
    def is_checkpoint_writer(self) -> bool:
        return self.replica_id == 0

    def agree(self, flag: bool) -> bool:
        """Replica 0's value of a per-process decision (a timer firing) on every replica."""
        if self.strategy is None:
            return bool(flag)
        from ..parallel.collective import broadcast_flag
        return broadcast_flag(flag, group=self.strategy.group)

    # -- checkpointing
    def default_saver(self):
        from .checkpoint import Saver
        if self.ps_ops:
            return Saver([])
        items = []
        for op in self.train_ops:
            items += _saver_items(op)
        gs = self.graph.global_step
        extra = {}
        if gs is not None and not any(n == "global_step" for n, _, _ in items):
            items.append(("global_step", lambda: np.asarray(gs.value(), dtype=np.int64),
                          lambda a: gs.assign(int(np.asarray(a)))))
        return Saver(items, extra=extra, on_restore=[op.params.refresh_compute for op in self.train_ops])

    def save_checkpoint(self, saver, basename, step):
        """Collective on all-reduce replicas: every replica averages its SyncOnRead variables
        (BN moving statistics), replica 0 alone writes, then all wait for the write."""
        if self.strategy is not None:
            from ..parallel.collective import sync_on_read_mean_
            for op in self.train_ops:
                if op.mode == "mirrored":
                    sync_on_read_mean_(op.params, self.strategy.group)
            path = saver.save(None, basename, global_step=step) if self.replica_id == 0 else None
            self.strategy.barrier()
            return path
        if self.ps_ops:
            n = self.client.n_ps
            return saver.save(None, basename, global_step=step,
                              shard_writers=[lambda p, t=t: self.client.save_shard(t, p) for t in range(n)])
        return saver.save(None, basename, global_step=step)

    # -- execution
    def _feed(self, feed_dict):
        out = {}
        for k, v in (feed_dict or {}).items():
            name = k.name if isinstance(k, G.Placeholder) else str(k)
            out[name] = v
        return out

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        feed = self._feed(feed_dict)
        flat = _flatten(fetches, [])
        for op in dict.fromkeys(f for f in flat if hasattr(f, "run") and hasattr(f, "optimizer")):
            op.run(feed)
        vals = [self._eval(f, feed) for f in flat]
        return _pack(fetches, iter(vals))

    def _eval(self, f, feed):
        from .optimizers import TrainOp
        if isinstance(f, TrainOp):
            return None
        if isinstance(f, G.Fetch):
            v = f.op.outputs.get(f.key)
            if v is None:
                raise errors.InvalidArgumentError("%s has no output %r (run the train op first)" % (f.op.name, f.key))
            return _host(v)
        if isinstance(f, G.GlobalStep):
            return f.value()
        if isinstance(f, G.Placeholder):
            return feed.get(f.name)
        if isinstance(f, G._AddN):
            return sum(self._eval(v, feed) for v in f.values)
        if callable(f):
            return _host(f())
        return _host(f)

    def close(self):
        if self._closed:
            return
        self._closed = True
        if self.client is not None:
            self.client.close()


def mirrored_strategy(train_ops):
    """The strategy of the first train op that all-reduces over more than one replica."""
    for op in train_ops:
        if getattr(op, "mode", None) == "mirrored" and op.strategy is not None \
                and op.strategy.num_replicas_in_sync > 1:
            return op.strategy
    return None


def _saver_items(op):
    """Name-based Saver items for a TrainOp: every model variable (TF layout) + optimizer
    slots with TF1 slot names (<var>/Momentum, <var>/Adam, <var>/Adam_1)."""
    from .checkpoint import export_value, import_value
    P = op.params
    items = []
    for s in P.specs:
        items.append((s.name, (lambda s=s: export_value(s, P.var[s.name])),
                      (lambda a, s=s: import_value(s, a, P.var[s.name]))))
    flat = op.flat
    if flat is not None:
        names = {"mom": "Momentum", "m": "Adam", "v": "Adam_1"}
        if type(flat).__name__ == "FlatLAMB":
            names = {"m": "LAMB", "v": "LAMB_1"}
        for attr, suffix in names.items():
            buf = getattr(flat, attr, None)
            if not isinstance(buf, torch.Tensor):
                continue
            for s in P.specs:
                if not s.trainable:
                    continue
                o, n = P.offsets[s.name], int(np.prod(s.shape))
                v = buf[o:o + n].view(tuple(s.shape))
                items.append(("%s/%s" % (s.name, suffix), (lambda s=s, v=v: export_value(s, v)),
                              (lambda a, s=s, v=v: import_value(s, a, v))))
    return items


class _HookedSession:
    def __init__(self, sess: _CoreSession, hooks: List[SessionRunHook]):
        self._sess = sess
        self._hooks = hooks
        self._should_stop = False

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        actual = SessionRunArgs(fetches, feed_dict, options)
        ctx = SessionRunContext(actual, self._sess)
        hook_args = [h.before_run(ctx) for h in self._hooks]
        feed = dict(feed_dict or {})
        for a in hook_args:
            if a is not None and a.feed_dict:
                for k in a.feed_dict:
                    if k in feed:
                        raise RuntimeError("same tensor fed by a hook and by the caller: %s" % k)
                feed.update(a.feed_dict)
        combined = {"caller": fetches, "hooks": [a.fetches if a is not None else None for a in hook_args]}
        out = self._sess.run(combined, feed_dict=feed, options=options)
        for h, r in zip(self._hooks, out["hooks"]):
            h.after_run(ctx, SessionRunValues(r, options, run_metadata))
        self._should_stop = self._should_stop or ctx.stop_requested
        return out["caller"]


class MonitoredSession:
    """Recoverable, coordinated, hooked session (tf.train.MonitoredSession)."""

    def __init__(self, session_creator=None, hooks=None, stop_grace_period_secs=120, graph=None):
        self._creator = session_creator or ChiefSessionCreator()
        self._hooks = list(hooks or [])
        self._grace = stop_grace_period_secs
        self._graph = graph or G.get_default_graph()
        for h in self._hooks:
            h.begin()
        self._graph.finalized = True
        self.coord = Coordinator()
        self._sess = None
        self._hooked = None
        self._closed = False
        self.recoveries = 0
        self._create()

    def _create(self):
        # as TF's _RecoverableSession._create_session: creating (or re-creating) the session
        # retries while a task is still unreachable (e.g. a replacement PS that is starting)
        delay = 0.2
        while True:
            try:
                self._sess = self._creator.create_session(self._graph)
                break
            except errors.PREEMPTION_ERRORS as e:
                log.warning("%s while creating the session: %s — retrying", type(e).__name__, e)
                time.sleep(delay)
                delay = min(2 * delay, 5.0)
        self._hooked = _HookedSession(self._sess, self._hooks)
        for h in self._hooks:
            h.after_create_session(self._sess, self.coord)

    def should_stop(self) -> bool:
        if self._closed:
            return True
        return self.coord.should_stop() or (self._hooked is not None and self._hooked._should_stop)

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        while True:
            try:
                out = self._hooked.run(fetches, feed_dict, options, run_metadata)
                if self._hooked._should_stop:
                    self.coord.request_stop()
                return out
            except errors.PREEMPTION_ERRORS as e:
                log.warning("%s: %s — recreating the session", type(e).__name__, e)
                self.recoveries += 1
                strategy = getattr(self._sess, "strategy", None)
                try:
                    self._sess.close()
                except Exception:  # noqa: BLE001
                    pass
                if strategy is not None:
                    # a failed collective leaves the communicator unusable: rebuild the process
                    # group (next generation) before the new session restores + broadcasts
                    strategy.recover()
                self._create()
            except Exception as e:
                self.coord.request_stop(e)
                raise

    def run_step_fn(self, step_fn):
        class StepContext:
            def __init__(s, sess):
                s.session = sess

            def run_with_hooks(s, *a, **kw):
                return self.run(*a, **kw)

            def request_stop(s):
                self.coord.request_stop()
        return step_fn(StepContext(self._sess))

    def close(self):
        if self._closed:
            return
        try:
            for h in self._hooks:
                h.end(self._sess)
        finally:
            self._closed = True
            self.coord.request_stop()
            try:
                self.coord.join(stop_grace_period_secs=self._grace, ignore_live_threads=True)
            finally:
                if self._sess is not None:
                    self._sess.close()

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type in (errors.OutOfRangeError, StopIteration):
            exc_type = None
        try:
            self.close()
        except Exception:
            if exc_type is None:
                raise
        return exc_type is None and exc is not None and isinstance(exc, (errors.OutOfRangeError, StopIteration))


class SessionCreator:
    def create_session(self, graph) -> _CoreSession:
        raise NotImplementedError


class ChiefSessionCreator(SessionCreator):
    def __init__(self, scaffold=None, master="", config=None, checkpoint_dir=None, checkpoint_filename_with_path=None):
        self.master, self.config, self.checkpoint_dir, self.scaffold = master, config, checkpoint_dir, scaffold

    def create_session(self, graph):
        return _CoreSession(graph, self.master, self.config, True, self.checkpoint_dir, scaffold=self.scaffold)


class WorkerSessionCreator(SessionCreator):
    def __init__(self, scaffold=None, master="", config=None, max_wait_secs=7200, recovery_wait_secs=0.5):
        self.master, self.config, self.max_wait, self.recovery_wait = master, config, max_wait_secs, recovery_wait_secs
        self.scaffold = scaffold

    def create_session(self, graph):
        return _CoreSession(graph, self.master, self.config, False, None, self.max_wait, self.recovery_wait,
                            scaffold=self.scaffold)


def MonitoredTrainingSession(master="", is_chief=True, checkpoint_dir=None, scaffold=None, hooks=None,
                             chief_only_hooks=None, save_checkpoint_secs=USE_DEFAULT, save_summaries_steps=USE_DEFAULT,
                             save_summaries_secs=USE_DEFAULT, config=None, stop_grace_period_secs=120,
                             log_step_count_steps=100, max_wait_secs=7200, save_checkpoint_steps=USE_DEFAULT,
                             summary_dir=None, recovery_wait_secs=0.5) -> MonitoredSession:
    if save_summaries_steps is USE_DEFAULT and save_summaries_secs is USE_DEFAULT:
        save_summaries_steps, save_summaries_secs = 100, None
    elif save_summaries_steps is USE_DEFAULT:
        save_summaries_steps = None
    elif save_summaries_secs is USE_DEFAULT:
        save_summaries_secs = None
    if save_checkpoint_secs is USE_DEFAULT and save_checkpoint_steps is USE_DEFAULT:
        save_checkpoint_secs, save_checkpoint_steps = 600, None
    elif save_checkpoint_secs is USE_DEFAULT:
        save_checkpoint_secs = None
    elif save_checkpoint_steps is USE_DEFAULT:
        save_checkpoint_steps = None
    all_hooks = []
    mirror = mirrored_strategy(G.get_default_graph().get_collection(G.TRAIN_OP))
    if mirror is not None and checkpoint_dir and ((save_checkpoint_secs and save_checkpoint_secs > 0) or
                                                  (save_checkpoint_steps and save_checkpoint_steps > 0)):
        # all-reduce replicas: the checkpoint hook runs on EVERY replica (its save is a
        # collective; replica 0 writes), whichever of them the caller marked chief
        all_hooks.append(CheckpointSaverHook(checkpoint_dir, save_secs=save_checkpoint_secs,
                                             save_steps=save_checkpoint_steps))
        save_checkpoint_secs = save_checkpoint_steps = None
    if is_chief:
        creator = ChiefSessionCreator(scaffold, master, config, checkpoint_dir)
        all_hooks.extend(chief_only_hooks or [])
        summary_dir = summary_dir or checkpoint_dir
        if mirror is not None and mirror.replica_id != 0:
            summary_dir = None  # one event-file writer per job
        if summary_dir:
            if log_step_count_steps and log_step_count_steps > 0:
                all_hooks.append(StepCounterHook(output_dir=summary_dir, every_n_steps=log_step_count_steps))
            if (save_summaries_steps and save_summaries_steps > 0) or (save_summaries_secs and save_summaries_secs > 0):
                all_hooks.append(SummarySaverHook(save_steps=save_summaries_steps, save_secs=save_summaries_secs,
                                                  output_dir=summary_dir))
        if checkpoint_dir and ((save_checkpoint_secs and save_checkpoint_secs > 0) or
                               (save_checkpoint_steps and save_checkpoint_steps > 0)):
            all_hooks.append(CheckpointSaverHook(checkpoint_dir, save_secs=save_checkpoint_secs,
                                                 save_steps=save_checkpoint_steps))
    else:
        creator = WorkerSessionCreator(scaffold, master, config, max_wait_secs, recovery_wait_secs)
    all_hooks.extend(hooks or [])
    return MonitoredSession(creator, all_hooks, stop_grace_period_secs)


def SingularMonitoredSession(hooks=None, scaffold=None, master="", config=None, checkpoint_dir=None,
                             stop_grace_period_secs=120):
    return MonitoredSession(ChiefSessionCreator(scaffold, master, config, checkpoint_dir), hooks,
                            stop_grace_period_secs)


class Scaffold:
    def __init__(self, init_op=None, saver=None, summary_op=None, ready_op=None, local_init_op=None):
        self.init_op, self.saver, self.summary_op = init_op, saver, summary_op

    def finalize(self):
        return self


class SessionConfig:
    """tf.ConfigProto subset (:201-202): soft placement = CPU fallback for ops without a HIP
    kernel; log_device_placement prints each variable's owner."""

    def __init__(self, allow_soft_placement=True, log_device_placement=False, **kw):
        self.allow_soft_placement = allow_soft_placement
        self.log_device_placement = log_device_placement
        self.extra = kw


ConfigProto = SessionConfig
