"""Graph-lite state: the default "graph" holding the global step, placeholders, collections
and summaries — the eager-framework equivalent of the TF1 graph-construction calls the
reference makes (`tf.placeholder` :191-192, `tf.train.get_or_create_global_step` :116,
`tf.add_to_collection('losses', ...)` :83, `tf.summary.scalar` :129,132).

Nothing is traced: a training step is executed by a TrainOp (train/optimizers.py) and the
"tensors" a session can fetch are handles (Fetch) naming one of its outputs.
"""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional

import torch

GLOBAL_STEP = "global_step"
SUMMARIES = "summaries"
LOSSES = "losses"
TRAIN_OP = "train_op"
REGULARIZATION_LOSSES = "regularization_losses"


class Placeholder:
    """Feed slot (tf.placeholder). `feed_dict={ph: value}` or `{ph.name: value}`."""

    def __init__(self, dtype=torch.float32, shape=None, name: Optional[str] = None):
        self.dtype = dtype
        self.shape = shape
        self.name = name or "placeholder"

    def __repr__(self):
        return "Placeholder(%s, %s, %s)" % (self.name, self.dtype, self.shape)


class Fetch:
    """Handle to a named output of a TrainOp (e.g. train_op.loss)."""

    def __init__(self, op, key: str):
        self.op = op
        self.key = key
        self.name = key

    def __repr__(self):
        return "Fetch(%s)" % self.key


class GlobalStep:
    """int64 global step. Its value lives wherever the training runtime keeps it: a host
    counter (local), the optimizer's device counter, or parameter-server task 0."""

    def __init__(self, name="global_step"):
        self.name = name
        self._value = 0
        self._getter = None
        self._setter = None
        self.device = None

    def bind(self, getter=None, setter=None):
        self._getter, self._setter = getter, setter

    def value(self) -> int:
        return int(self._getter()) if self._getter else self._value

    def numpy(self):
        import numpy as np
        return np.asarray(self.value(), dtype=np.int64)

    def assign(self, v):
        v = int(v if not hasattr(v, "item") else v.item())
        if self._setter:
            self._setter(v)
        self._value = v

    def assign_add(self, d=1):
        self.assign(self.value() + d)

    def __int__(self):
        return self.value()

    def __index__(self):
        return self.value()

    def __repr__(self):
        return "GlobalStep(%d)" % self.value()


class Graph:
    def __init__(self):
        self.collections: Dict[str, List[Any]] = {}
        self.global_step: Optional[GlobalStep] = None
        self.placeholders: Dict[str, Placeholder] = {}
        self.models: List[Any] = []
        self.finalized = False

    def add_to_collection(self, name, value):
        self.collections.setdefault(name, []).append(value)

    def get_collection(self, name) -> List[Any]:
        return list(self.collections.get(name, []))

    def as_default(self):
        return _GraphContext(self)


_local = threading.local()
_default = Graph()


class _GraphContext:
    def __init__(self, g):
        self.g = g

    def __enter__(self):
        st = getattr(_local, "stack", None)
        if st is None:
            st = _local.stack = []
        st.append(self.g)
        return self.g

    def __exit__(self, *a):
        _local.stack.pop()


def get_default_graph() -> Graph:
    st = getattr(_local, "stack", None)
    return st[-1] if st else _default


def reset_default_graph():
    global _default
    _default = Graph()


def placeholder(dtype=torch.float32, shape=None, name=None) -> Placeholder:
    p = Placeholder(dtype, shape, name)
    get_default_graph().placeholders[p.name] = p
    return p


def get_or_create_global_step(graph: Optional[Graph] = None) -> GlobalStep:
    g = graph or get_default_graph()
    if g.global_step is None:
        g.global_step = GlobalStep()
        g.add_to_collection(GLOBAL_STEP, g.global_step)
    return g.global_step


def get_global_step(graph: Optional[Graph] = None) -> Optional[GlobalStep]:
    return (graph or get_default_graph()).global_step


def add_to_collection(name, value):
    get_default_graph().add_to_collection(name, value)


def get_collection(name):
    return get_default_graph().get_collection(name)


def add_n(values):
    """tf.add_n over host/device scalars or Fetch handles (sum evaluated at fetch time)."""
    return _AddN(list(values))


class _AddN:
    def __init__(self, values):
        self.values = values
