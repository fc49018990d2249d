"""`ttd.initializers` — TF-compatible variable initializers.

`variance_scaling_initializer()` with TF1 defaults (factor 2.0, FAN_IN, truncated normal)
is what the reference's hidden layers use (/root/reference/distribute_training.py:49): a
+-2 sigma truncated normal with sigma = sqrt(1.3 * factor / fan) (the 1.3 undoes the
truncation's variance loss). Initializers are callables (shape, generator) -> fp32 tensor.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch


def _fans(shape: Sequence[int]):
    shape = tuple(int(s) for s in shape)
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    receptive = 1
    for s in shape[:-2]:
        receptive *= s
    return shape[-2] * receptive, shape[-1] * receptive  # conv kernels [..., in, out]


def _truncated(shape, std, gen):
    t = torch.empty(tuple(shape), dtype=torch.float32)
    torch.nn.init.trunc_normal_(t, 0.0, std, -2 * std, 2 * std, generator=gen)
    return t


class Initializer:
    def __call__(self, shape, gen: Optional[torch.Generator] = None) -> torch.Tensor:
        raise NotImplementedError


class Zeros(Initializer):
    def __call__(self, shape, gen=None):
        return torch.zeros(tuple(shape), dtype=torch.float32)


class Ones(Initializer):
    def __call__(self, shape, gen=None):
        return torch.ones(tuple(shape), dtype=torch.float32)


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = float(value)

    def __call__(self, shape, gen=None):
        return torch.full(tuple(shape), self.value, dtype=torch.float32)


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05):
        self.mean, self.stddev = float(mean), float(stddev)

    def __call__(self, shape, gen=None):
        return torch.empty(tuple(shape)).normal_(self.mean, self.stddev, generator=gen)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05):
        self.mean, self.stddev = float(mean), float(stddev)

    def __call__(self, shape, gen=None):
        return _truncated(shape, self.stddev, gen) + self.mean


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05):
        self.minval, self.maxval = float(minval), float(maxval)

    def __call__(self, shape, gen=None):
        return torch.empty(tuple(shape)).uniform_(self.minval, self.maxval, generator=gen)


class VarianceScaling(Initializer):
    """tf.contrib.layers.variance_scaling_initializer (factor/mode/uniform) and
    tf.keras VarianceScaling (scale/mode/distribution) semantics."""

    def __init__(self, factor=2.0, mode="FAN_IN", uniform=False, distribution=None):
        self.factor = float(factor)
        self.mode = mode.upper()
        self.uniform = bool(uniform) or distribution == "uniform"
        self.distribution = distribution

    def __call__(self, shape, gen=None):
        fan_in, fan_out = _fans(shape)
        n = {"FAN_IN": fan_in, "FAN_OUT": fan_out, "FAN_AVG": (fan_in + fan_out) / 2.0}[self.mode]
        if self.uniform:
            lim = math.sqrt(3.0 * self.factor / n)
            return torch.empty(tuple(shape)).uniform_(-lim, lim, generator=gen)
        if self.distribution == "untruncated_normal":
            return torch.empty(tuple(shape)).normal_(0.0, math.sqrt(self.factor / n), generator=gen)
        return _truncated(shape, math.sqrt(1.3 * self.factor / n), gen)


def variance_scaling_initializer(factor=2.0, mode="FAN_IN", uniform=False, seed=None, dtype=None):
    return VarianceScaling(factor, mode, uniform)


class GlorotUniform(VarianceScaling):
    def __init__(self):
        super().__init__(1.0, "FAN_AVG", uniform=True)


class GlorotNormal(VarianceScaling):
    def __init__(self):
        super().__init__(1.0, "FAN_AVG", uniform=False)


class HeNormal(VarianceScaling):
    def __init__(self):
        super().__init__(2.0, "FAN_IN", uniform=False)


def get(identifier):
    if identifier is None:
        return None
    if isinstance(identifier, Initializer) or callable(identifier):
        return identifier
    table = {"zeros": Zeros(), "ones": Ones(), "glorot_uniform": GlorotUniform(), "glorot_normal": GlorotNormal(),
             "he_normal": HeNormal(), "truncated_normal": TruncatedNormal(), "random_normal": RandomNormal(),
             "variance_scaling": VarianceScaling()}
    return table[identifier]
