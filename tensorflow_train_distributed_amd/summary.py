"""tf.summary surface: `scalar(name, tensor)` registers a scalar summary in the default graph
(/root/reference/distribute_training.py:128-132); `FileWriter` appends TensorBoard events
(utils/events.py); `FileWriterCache` shares one writer per logdir (as the chief's
SummarySaverHook / StepCounterHook do in TF1)."""
from __future__ import annotations

import threading
from collections import namedtuple

from .train import graph as G
from .utils.events import EventFileWriter, read_events, summary_proto, summary_value_scalar

ScalarSummary = namedtuple("ScalarSummary", ["tag", "value"])


def scalar(name, tensor, collections=None, family=None):
    """tensor: a Fetch handle (e.g. train_op.loss), a GlobalStep, a callable or a number."""
    s = ScalarSummary(name if family is None else "%s/%s" % (family, name), tensor)
    for c in (collections or [G.SUMMARIES]):
        G.add_to_collection(c, s)
    return s


def merge_all(key=G.SUMMARIES):
    return G.get_collection(key)


class FileWriter(EventFileWriter):
    def __init__(self, logdir, graph=None, max_queue=10, flush_secs=120, filename_suffix=""):
        super().__init__(logdir, flush_secs=flush_secs, filename_suffix=filename_suffix)

    def add_summary(self, summary, global_step=None):
        if isinstance(summary, (list, tuple)) and summary and isinstance(summary[0], tuple):
            self.add_scalars(summary, global_step or 0)
        else:
            super().add_summary(summary, global_step or 0)


class FileWriterCache:
    _lock = threading.Lock()
    _cache = {}

    @classmethod
    def get(cls, logdir):
        with cls._lock:
            w = cls._cache.get(logdir)
            if w is None or w._closed:
                w = FileWriter(logdir)
                cls._cache[logdir] = w
            return w

    @classmethod
    def clear(cls):
        with cls._lock:
            for w in cls._cache.values():
                w.close()
            cls._cache.clear()


__all__ = ["scalar", "merge_all", "FileWriter", "FileWriterCache", "read_events", "summary_proto",
           "summary_value_scalar"]
