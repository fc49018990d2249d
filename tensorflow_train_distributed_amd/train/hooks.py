"""SessionRunHook protocol and the standard hooks.

Reference: the reference passes `StopAtStepHook(last_step=2000)` and (sync mode) the
SyncReplicasOptimizer hook (/root/reference/distribute_training.py:193-199) to
MonitoredTrainingSession, which adds the chief-only CheckpointSaverHook (save every 60 s),
SummarySaverHook (every 100 steps) and StepCounterHook.
Hook protocol: begin() -> after_create_session(session, coord) ->
[before_run(run_context) -> SessionRunArgs | None, after_run(run_context, run_values)]* -> end(session).
"""
from __future__ import annotations

import json
import logging
import math
import os
import threading
import time
from collections import namedtuple
from typing import Callable, Dict, List, Optional

from ..utils import errors
from . import graph as G

log = logging.getLogger("tensorflow_train_distributed_amd")


class SessionRunArgs(namedtuple("SessionRunArgs", ["fetches", "feed_dict", "options"])):
    def __new__(cls, fetches, feed_dict=None, options=None):
        return super().__new__(cls, fetches, feed_dict, options)


class SessionRunValues(namedtuple("SessionRunValues", ["results", "options", "run_metadata"])):
    pass


class SessionRunContext:
    def __init__(self, original_args: SessionRunArgs, session):
        self._original_args = original_args
        self._session = session
        self._stop_requested = False

    @property
    def original_args(self):
        return self._original_args

    @property
    def session(self):
        return self._session

    @property
    def stop_requested(self):
        return self._stop_requested

    def request_stop(self):
        self._stop_requested = True


class SessionRunHook:
    def begin(self):
        pass

    def after_create_session(self, session, coord):
        pass

    def before_run(self, run_context) -> Optional[SessionRunArgs]:
        return None

    def after_run(self, run_context, run_values):
        pass

    def end(self, session):
        pass


class SecondOrStepTimer:
    def __init__(self, every_secs=None, every_steps=None):
        if (every_secs is None) == (every_steps is None):
            raise ValueError("exactly one of every_secs / every_steps")
        self._every_secs = every_secs
        self._every_steps = every_steps
        self._last_time = None
        self._last_step = None

    def should_trigger_for_step(self, step):
        if self._last_step is None:
            return True
        if self._last_step == step:
            return False
        if self._every_secs is not None:
            return time.time() >= self._last_time + self._every_secs
        return step >= self._last_step + self._every_steps

    def update_last_triggered_step(self, step):
        now = time.time()
        elapsed = (now - self._last_time, step - self._last_step) if self._last_time is not None else (None, None)
        self._last_time, self._last_step = now, step
        return elapsed

    def last_triggered_step(self):
        return self._last_step


class StopAtStepHook(SessionRunHook):
    def __init__(self, num_steps=None, last_step=None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("exactly one of num_steps / last_step")
        self._num_steps = num_steps
        self._last_step = last_step

    def begin(self):
        self._gs = G.get_global_step()
        if self._gs is None:
            raise RuntimeError("global step must be created to use StopAtStepHook")

    def after_create_session(self, session, coord):
        if self._last_step is None:
            self._last_step = self._gs.value() + self._num_steps

    def before_run(self, run_context):
        return SessionRunArgs(self._gs)

    def after_run(self, run_context, run_values):
        # fetches are evaluated after the step, so results is the post-update global step
        if run_values.results >= self._last_step:
            run_context.request_stop()

    @property
    def last_step(self):
        return self._last_step


class CheckpointSaverListener:
    def begin(self):
        pass

    def before_save(self, session, global_step_value):
        pass

    def after_save(self, session, global_step_value):
        return False

    def end(self, session, global_step_value):
        pass


class CheckpointSaverHook(SessionRunHook):
    """Saves `<checkpoint_dir>/model.ckpt-<step>` every save_secs / save_steps, at session
    creation and at end(). The saver is supplied by the session (name-based Saver over every
    variable; sharded per PS task in parameter-server mode)."""

    def __init__(self, checkpoint_dir, save_secs=None, save_steps=None, saver=None,
                 checkpoint_basename="model.ckpt", scaffold=None, listeners=None):
        self._dir = checkpoint_dir
        self._timer = SecondOrStepTimer(every_secs=save_secs, every_steps=save_steps)
        self._saver = saver
        self._basename = checkpoint_basename
        self._listeners = listeners or []
        self.saved_paths: List[str] = []
        self.agree_every = max(1, int(os.environ.get("TTD_CKPT_AGREE_STEPS", "50")))

    def begin(self):
        if self._dir:
            os.makedirs(self._dir, exist_ok=True)
        self._gs = G.get_global_step()
        for l in self._listeners:
            l.begin()

    def after_create_session(self, session, coord):
        if self._saver is None:
            self._saver = session.default_saver()
        step = self._gs.value()
        self._save(session, step)
        self._timer.update_last_triggered_step(step)

    def before_run(self, run_context):
        return SessionRunArgs(self._gs)

    def after_run(self, run_context, run_values):
        step = run_values.results
        fire = self._timer.should_trigger_for_step(step)
        agree = getattr(run_context.session, "agree", None)
        if agree is not None and self._timer._every_secs is not None:
            # all-reduce replicas: replica 0's clock decides for everyone. The agreement is a
            # broadcast + host sync, so it runs only on every agree_every-th global step (the
            # replicas see the same global steps, so they all take part in the same ones); the
            # save lands at most agree_every steps after the timer fired, and every other step
            # keeps the host running ahead of the GPU.
            fire = agree(fire) if step % self.agree_every == 0 else False
        if fire:
            self._timer.update_last_triggered_step(step)
            if self._save(run_context.session, step):
                run_context.request_stop()

    def end(self, session):
        step = self._gs.value()
        if step != self._timer.last_triggered_step():
            self._save(session, step)
        for l in self._listeners:
            l.end(session, step)

    def _save(self, session, step):
        for l in self._listeners:
            l.before_save(session, step)
        path = session.save_checkpoint(self._saver, os.path.join(self._dir or ".", self._basename), step)
        if path is not None:  # None: an all-reduce replica other than replica 0 (not a writer)
            self.saved_paths.append(path)
            log.info("Saving checkpoints for %d into %s.", step, path)
        stop = False
        for l in self._listeners:
            stop = l.after_save(session, step) or stop
        return stop


class SummarySaverHook(SessionRunHook):
    """Writes the graph's scalar summaries (SUMMARIES collection) every save_steps/secs."""

    def __init__(self, save_steps=None, save_secs=None, output_dir=None, summary_writer=None, scaffold=None,
                 summary_op=None):
        self._timer = SecondOrStepTimer(every_secs=save_secs, every_steps=save_steps)
        self._output_dir = output_dir
        self._writer = summary_writer
        self._summary_op = summary_op
        self._request = False

    def begin(self):
        from ..summary import FileWriterCache
        if self._writer is None and self._output_dir:
            self._writer = FileWriterCache.get(self._output_dir)
        self._gs = G.get_global_step()
        self._next_step = None

    def before_run(self, run_context):
        self._request = self._next_step is None or self._timer.should_trigger_for_step(self._next_step)
        fetches = {"global_step": self._gs}
        if self._request:
            summ = self._summary_op if self._summary_op is not None else G.get_collection(G.SUMMARIES)
            fetches["summaries"] = [s.value for s in summ]
            self._tags = [s.tag for s in summ]
        return SessionRunArgs(fetches)

    def after_run(self, run_context, run_values):
        step = run_values.results["global_step"]
        if self._next_step is None:
            self._next_step = step
        if self._request and self._writer is not None:
            self._timer.update_last_triggered_step(step)
            vals = run_values.results["summaries"]
            self._writer.add_scalars(list(zip(self._tags, [float(v) for v in vals])), step)
        self._next_step = step + 1

    def end(self, session=None):
        if self._writer is not None:
            self._writer.flush()


class StepCounterHook(SessionRunHook):
    """Logs and summarises `global_step/sec` every N steps."""

    def __init__(self, every_n_steps=100, every_n_secs=None, output_dir=None, summary_writer=None,
                 steps_per_run=1):
        self._timer = SecondOrStepTimer(every_steps=every_n_steps, every_secs=every_n_secs) \
            if every_n_secs is None else SecondOrStepTimer(every_secs=every_n_secs)
        self._output_dir = output_dir
        self._writer = summary_writer
        self.rates: List[float] = []

    def begin(self):
        from ..summary import FileWriterCache
        if self._writer is None and self._output_dir:
            self._writer = FileWriterCache.get(self._output_dir)
        self._gs = G.get_global_step()

    def before_run(self, run_context):
        return SessionRunArgs(self._gs)

    def after_run(self, run_context, run_values):
        step = run_values.results
        if self._timer.should_trigger_for_step(step):
            dt, ds = self._timer.update_last_triggered_step(step)
            if dt:
                rate = ds / dt
                self.rates.append(rate)
                log.info("global_step/sec: %g", rate)
                if self._writer is not None:
                    self._writer.add_scalars([("global_step/sec", rate)], step)


class LoggingTensorHook(SessionRunHook):
    def __init__(self, tensors, every_n_iter=None, every_n_secs=None, at_end=False, formatter=None):
        self._tensors = tensors if isinstance(tensors, dict) else {getattr(t, "name", str(t)): t for t in tensors}
        self._timer = SecondOrStepTimer(every_secs=every_n_secs, every_steps=every_n_iter) \
            if (every_n_iter or every_n_secs) else None
        self._at_end = at_end
        self._formatter = formatter
        self._iter = 0
        self.logged: List[Dict] = []

    def before_run(self, run_context):
        self._should = self._timer is not None and self._timer.should_trigger_for_step(self._iter)
        return SessionRunArgs(self._tensors) if self._should else None

    def after_run(self, run_context, run_values):
        if self._should:
            self._timer.update_last_triggered_step(self._iter)
            vals = run_values.results
            self.logged.append(vals)
            msg = self._formatter(vals) if self._formatter else ", ".join("%s = %s" % kv for kv in vals.items())
            log.info(msg)
        self._iter += 1

    def end(self, session):
        if self._at_end:
            vals = session.run(self._tensors)
            self.logged.append(vals)


class NanLossDuringTrainingError(RuntimeError):
    pass


class NanTensorHook(SessionRunHook):
    def __init__(self, loss_tensor, fail_on_nan_loss=True):
        self._loss = loss_tensor
        self._fail = fail_on_nan_loss

    def before_run(self, run_context):
        return SessionRunArgs(self._loss)

    def after_run(self, run_context, run_values):
        if not math.isfinite(float(run_values.results)):
            if self._fail:
                raise NanLossDuringTrainingError("NaN loss during training.")
            log.warning("NaN loss; stopping.")
            run_context.request_stop()


class GlobalStepWaiterHook(SessionRunHook):
    """Delays a worker until the global step reaches `wait_until_step`."""

    def __init__(self, wait_until_step, poll_secs=0.5):
        self._wait = wait_until_step
        self._poll = poll_secs

    def begin(self):
        self._gs = G.get_global_step()

    def before_run(self, run_context):
        while self._gs.value() < self._wait:
            time.sleep(self._poll)
        return None


class FeedFnHook(SessionRunHook):
    def __init__(self, feed_fn):
        self.feed_fn = feed_fn

    def before_run(self, run_context):
        return SessionRunArgs(fetches=None, feed_dict=self.feed_fn())


class FinalOpsHook(SessionRunHook):
    def __init__(self, final_ops, final_ops_feed_dict=None):
        self._ops = final_ops
        self._feed = final_ops_feed_dict
        self.final_ops_values = None

    def end(self, session):
        if self._ops is not None:
            self.final_ops_values = session.run(self._ops, feed_dict=self._feed)


class ProfilerHook(SessionRunHook):
    """Every save_steps, records one step with torch.profiler (HIP kernels via roctracer on
    ROCm) and writes `timeline-<step>.json` (Chrome trace) to output_dir; falls back to a
    host-phase trace when the profiler is unavailable."""

    def __init__(self, save_steps=None, save_secs=None, output_dir="", show_dataflow=True, show_memory=False):
        self._timer = SecondOrStepTimer(every_secs=save_secs, every_steps=save_steps)
        self._dir = output_dir
        self._prof = None
        self.written: List[str] = []

    def begin(self):
        self._gs = G.get_global_step()
        self._next = None

    def before_run(self, run_context):
        step = self._gs.value()
        self._active = self._timer.should_trigger_for_step(step + 1)
        if self._active:
            self._t0 = time.time()
            try:
                import torch.profiler as tp
                acts = [tp.ProfilerActivity.CPU]
                import torch
                if torch.cuda.is_available():
                    acts.append(tp.ProfilerActivity.CUDA)
                self._prof = tp.profile(activities=acts)
                self._prof.__enter__()
            except Exception:  # noqa: BLE001
                self._prof = None
        return SessionRunArgs(self._gs)

    def after_run(self, run_context, run_values):
        if not self._active:
            return
        step = run_values.results
        self._timer.update_last_triggered_step(step)
        os.makedirs(self._dir, exist_ok=True)
        path = os.path.join(self._dir, "timeline-%d.json" % step)
        if self._prof is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            self._prof.export_chrome_trace(path)
            self._prof = None
        else:
            t1 = time.time()
            json.dump({"traceEvents": [{"name": "step", "ph": "X", "ts": self._t0 * 1e6, "dur": (t1 - self._t0) * 1e6,
                                        "pid": os.getpid(), "tid": 0}]}, open(path, "w"))
        self.written.append(path)


class SyncReplicasOptimizerHook(SessionRunHook):
    """Session setup for SyncReplicasOptimizer (tf _SyncReplicasOptimizerHook):
    chief: accumulators' step := global_step, enqueue the initial tokens, start the chief
    queue-runner thread running sync_op (take mean of N grads -> apply -> global_step += 1 ->
    enqueue tokens_per_step tokens); workers: local_step := global_step.
    end(): the chief closes the token queue so blocked workers exit."""

    def __init__(self, sync_optimizer, is_chief, num_tokens=-1):
        self._opt = sync_optimizer
        self._is_chief = is_chief
        self._num_tokens = num_tokens
        self._thread = None
        self._stop = threading.Event()
        self.applied_steps = 0

    def after_create_session(self, session, coord):
        op = self._opt._train_op
        if op is None or op.mode != "ps":
            return
        client = op.client
        gs = client.global_step()
        op.local_step = gs
        if not self._is_chief:
            return
        client.set_accum_step(gs)
        n = self._opt.replicas_to_aggregate if self._num_tokens == -1 else self._num_tokens
        if n < self._opt.replicas_to_aggregate - self._opt.total_num_replicas:
            raise errors.InvalidArgumentError("too few initial tokens")
        if n > 0:
            client.enqueue_tokens(n, gs)
        self._coord = coord
        self._thread = threading.Thread(target=self._queue_runner, args=(op,), name="sync_replicas_qr", daemon=True)
        if coord is not None:
            coord.register_thread(self._thread)
        self._thread.start()

    def _queue_runner(self, op):
        client = op.client
        try:
            while not self._stop.is_set():
                gs = client.global_step()
                lr = self._opt.schedule.value(gs)
                client.take_apply(self._opt.replicas_to_aggregate, lr, self._opt.tokens_per_step)
                self.applied_steps += 1
        except errors.OpError as e:
            if not self._stop.is_set():
                log.warning("sync replicas queue runner stopped: %s", e)

    def end(self, session):
        self._stop.set()
        op = self._opt._train_op
        if self._is_chief and op is not None and op.client is not None:
            try:
                op.client.close_queue()
            except errors.OpError:
                pass
            op.client.cancel_blocking("take")  # unblock the queue runner's pending take
            if self._thread is not None:
                self._thread.join(10)
