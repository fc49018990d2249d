"""`ttd.regularizers` — weight penalties.

The reference builds `tf.contrib.layers.l1_regularizer(0.01)` for every hidden kernel
(/root/reference/distribute_training.py:50,55); tf.layers puts the penalty into the
REGULARIZATION_LOSSES collection, which the reference never adds to its loss (§2.9 Q1).
Layers here do the same: `layer.losses` / the collection hold the penalties and the caller
decides whether to add them (`ttd.train.get_regularization_loss()`).
"""
from __future__ import annotations


class Regularizer:
    def __call__(self, w):
        raise NotImplementedError


class L1(Regularizer):
    def __init__(self, scale=0.01):
        self.scale = float(scale)

    def __call__(self, w):
        return self.scale * w.abs().sum()


class L2(Regularizer):
    """Keras convention: scale * sum(w^2) (tf.nn.l2_loss would be 0.5 * sum(w^2))."""

    def __init__(self, scale=0.01):
        self.scale = float(scale)

    def __call__(self, w):
        return self.scale * (w * w).sum()


class L1L2(Regularizer):
    def __init__(self, l1=0.0, l2=0.0):
        self.l1, self.l2 = float(l1), float(l2)

    def __call__(self, w):
        return self.l1 * w.abs().sum() + self.l2 * (w * w).sum()


def l1_regularizer(scale, scope=None):
    return L1(scale)


def l2_regularizer(scale, scope=None):
    return L2(scale)


l1 = L1
l2 = L2
