"""tf.train.QueueRunner / add_queue_runner / start_queue_runners and SessionManager.

Reference: the chief's SyncReplicasOptimizer aggregation loop is a TF1 QueueRunner thread
started by the sync hook under the session's Coordinator, and MonitoredTrainingSession's
session creators go through tf.train.SessionManager (prepare_session on the chief,
wait_for_session on the other workers) — /root/reference/distribute_training.py:144-148,
209-215; SURVEY.md §2.2 T11, T18.

Here a QueueRunner runs host callables (enqueue / aggregation steps) in threads until the
Coordinator requests a stop or the callable raises OutOfRangeError (queue closed);
SessionManager exposes the chief/worker session preparation that the session creators use.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional, Sequence

from ..utils import errors
from . import graph as G

QUEUE_RUNNERS = "queue_runners"


class QueueRunner:
    """Runs each of `enqueue_ops` (callables taking no argument, or the session) repeatedly
    in its own thread. `close_op` runs once when the runner stops because of an error or a
    coordinator stop; OutOfRangeError / CancelledError end a thread quietly."""

    def __init__(self, queue=None, enqueue_ops: Sequence[Callable] = (), close_op: Optional[Callable] = None,
                 cancel_op: Optional[Callable] = None, queue_closed_exception_types=(errors.OutOfRangeError,
                                                                                        errors.CancelledError)):
        self.queue = queue
        self.enqueue_ops = list(enqueue_ops)
        self.close_op = close_op
        self.cancel_op = cancel_op
        self._closed_types = tuple(queue_closed_exception_types)
        self.exceptions_raised: List[BaseException] = []
        self._lock = threading.Lock()
        self._runs = 0

    @property
    def name(self):
        return getattr(self.queue, "name", "queue_runner")

    def _call(self, op, sess):
        try:
            return op(sess)
        except TypeError:
            return op()

    def _run(self, sess, coord, op):
        try:
            while coord is None or not coord.should_stop():
                try:
                    self._call(op, sess)
                except self._closed_types:
                    break
        except Exception as e:  # noqa: BLE001
            with self._lock:
                self.exceptions_raised.append(e)
            if coord is not None:
                coord.request_stop(e)
        finally:
            with self._lock:
                self._runs -= 1
                last = self._runs == 0
            if last and self.close_op is not None:
                try:
                    self._call(self.close_op, sess)
                except Exception:  # noqa: BLE001 - closing after a failure is best effort
                    pass

    def _cancel_on_stop(self, sess, coord):
        coord.wait_for_stop()
        if self.cancel_op is not None:
            try:
                self._call(self.cancel_op, sess)
            except Exception:  # noqa: BLE001
                pass

    def create_threads(self, sess, coord=None, daemon=False, start=False) -> List[threading.Thread]:
        threads = []
        with self._lock:
            self._runs = len(self.enqueue_ops)
        for i, op in enumerate(self.enqueue_ops):
            threads.append(threading.Thread(target=self._run, args=(sess, coord, op), daemon=daemon,
                                            name="%s_%d" % (self.name, i)))
        if coord is not None and self.cancel_op is not None:
            threads.append(threading.Thread(target=self._cancel_on_stop, args=(sess, coord), daemon=True,
                                            name="%s_cancel" % self.name))
        for t in threads:
            if coord is not None:
                coord.register_thread(t)
            if start:
                t.start()
        return threads


def add_queue_runner(qr: QueueRunner, collection: str = QUEUE_RUNNERS):
    G.add_to_collection(collection, qr)


def start_queue_runners(sess=None, coord=None, daemon=True, start=True, collection: str = QUEUE_RUNNERS):
    threads = []
    for qr in G.get_collection(collection):
        threads += qr.create_threads(sess, coord=coord, daemon=daemon, start=start)
    return threads


class SessionManager:
    """tf.train.SessionManager: the chief prepares a session (restore the latest checkpoint of
    checkpoint_dir or initialise, then mark the parameter servers ready); other workers wait
    until the chief has done so (polling every recovery_wait_secs, up to max_wait_secs)."""

    def __init__(self, local_init_op=None, ready_op=None, ready_for_local_init_op=None, graph=None,
                 recovery_wait_secs: float = 30.0, local_init_run_options=None):
        self.graph = graph
        self.recovery_wait_secs = recovery_wait_secs

    def _graph(self):
        return self.graph if self.graph is not None else G.get_default_graph()

    def prepare_session(self, master="", init_op=None, saver=None, checkpoint_dir=None, checkpoint_filename_with_path=None,
                        wait_for_checkpoint=False, max_wait_secs=7200, config=None, init_feed_dict=None, init_fn=None):
        from .session import _CoreSession
        sess = _CoreSession(self._graph(), master, config, True, checkpoint_dir)
        if init_fn is not None:
            init_fn(sess)
        return sess

    def recover_session(self, master="", saver=None, checkpoint_dir=None, checkpoint_filename_with_path=None,
                        wait_for_checkpoint=False, max_wait_secs=7200, config=None):
        """Returns (session, restored_from_checkpoint)."""
        from .checkpoint import latest_checkpoint
        sess = self.prepare_session(master, checkpoint_dir=checkpoint_dir, config=config)
        return sess, bool(checkpoint_dir and latest_checkpoint(checkpoint_dir))

    def wait_for_session(self, master="", config=None, max_wait_secs=float("inf")):
        from .session import _CoreSession
        return _CoreSession(self._graph(), master, config, False, None,
                            max_wait_secs if max_wait_secs != float("inf") else 1e12, self.recovery_wait_secs)
