"""A small tf.data-style Dataset (host side) + replica sharding for the strategies, and the
synthetic ImageNet / BERT inputs of the north-star benchmarks (no network here).
"""
from __future__ import annotations

import itertools
from typing import Callable, Iterable, Iterator, Optional

import numpy as np
import torch


class Dataset:
    def __init__(self, gen_fn: Callable[[], Iterator]):
        self._gen_fn = gen_fn

    def __iter__(self):
        return iter(self._gen_fn())

    # -- sources
    @staticmethod
    def from_tensor_slices(tensors):
        if isinstance(tensors, dict):
            n = len(next(iter(tensors.values())))
            return Dataset(lambda: ({k: v[i] for k, v in tensors.items()} for i in range(n)))
        if isinstance(tensors, (tuple, list)):
            n = len(tensors[0])
            return Dataset(lambda: (tuple(t[i] for t in tensors) for i in range(n)))
        return Dataset(lambda: (tensors[i] for i in range(len(tensors))))

    @staticmethod
    def from_generator(gen: Callable[[], Iterable]):
        return Dataset(lambda: iter(gen()))

    @staticmethod
    def range(*args):
        return Dataset(lambda: iter(range(*args)))

    # -- transformations
    def map(self, fn):
        return Dataset(lambda: (fn(*x) if isinstance(x, tuple) else fn(x) for x in self))

    def filter(self, pred):
        return Dataset(lambda: (x for x in self if pred(x)))

    def repeat(self, count: Optional[int] = None):
        def gen():
            it = itertools.count() if count is None or count < 0 else range(count)
            for _ in it:
                yield from self
        return Dataset(gen)

    def take(self, n: int):
        return Dataset(lambda: itertools.islice(iter(self), n))

    def skip(self, n: int):
        return Dataset(lambda: itertools.islice(iter(self), n, None))

    def shuffle(self, buffer_size: int, seed: Optional[int] = None):
        def gen():
            rng = np.random.RandomState(seed)
            buf = []
            for x in self:
                buf.append(x)
                if len(buf) >= buffer_size:
                    i = rng.randint(len(buf))
                    buf[i], buf[-1] = buf[-1], buf[i]
                    yield buf.pop()
            rng.shuffle(buf)
            yield from buf
        return Dataset(gen)

    def batch(self, batch_size: int, drop_remainder: bool = False):
        def collate(items):
            first = items[0]
            if isinstance(first, dict):
                return {k: np.stack([np.asarray(it[k]) for it in items]) for k in first}
            if isinstance(first, tuple):
                return tuple(np.stack([np.asarray(it[j]) for it in items]) for j in range(len(first)))
            return np.stack([np.asarray(it) for it in items])

        def gen():
            buf = []
            for x in self:
                buf.append(x)
                if len(buf) == batch_size:
                    yield collate(buf)
                    buf = []
            if buf and not drop_remainder:
                yield collate(buf)
        return Dataset(gen)

    def shard(self, num_shards: int, index: int):
        return Dataset(lambda: itertools.islice(iter(self), index, None, num_shards))

    def prefetch(self, buffer_size: int = 1):
        return self  # host pipeline is synchronous; device prefetch: data.prefetch.DevicePrefetcher

    def cache(self):
        items = []
        done = [False]

        def gen():
            if done[0]:
                yield from items
                return
            for x in self:
                items.append(x)
                yield x
            done[0] = True
        return Dataset(gen)


class DistributedDataset:
    """Splits every global batch along axis 0 into `world` contiguous shards; this replica
    gets shard `rank` (tf.distribute experimental_distribute_dataset semantics)."""

    def __init__(self, dataset, world: int, rank: int):
        self.dataset = dataset
        self.world = world
        self.rank = rank

    def _slice(self, v):
        n = v.shape[0]
        if n % self.world:
            raise ValueError("global batch %d not divisible by %d replicas" % (n, self.world))
        k = n // self.world
        return v[self.rank * k:(self.rank + 1) * k]

    def __iter__(self):
        for b in self.dataset:
            if isinstance(b, dict):
                yield {k: self._slice(v) for k, v in b.items()}
            elif isinstance(b, tuple):
                yield tuple(self._slice(v) for v in b)
            else:
                yield self._slice(b)


def synthetic_imagenet(batch: int, image_size: int = 224, num_classes: int = 1000, device="cpu", seed: int = 0,
                       dtype=torch.bfloat16):
    """One resident random batch (NHWC) repeated forever — the tf_cnn_benchmarks
    `--data_name=imagenet` synthetic input (no decode/augment in the timed loop)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn((batch, image_size, image_size, 3), generator=g, device=device).to(dtype)
    y = torch.randint(0, num_classes, (batch,), generator=g, device=device, dtype=torch.int32)
    return Dataset(lambda: itertools.repeat({"images": x, "labels": y}))


def synthetic_bert(batch: int, seq_len: int = 512, vocab: int = 30522, max_predictions: int = 76, device="cpu",
                   seed: int = 0):
    """Random BERT pre-training batch (MLM + NSP) of the given shape, repeated forever."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    ids = torch.randint(0, vocab, (batch, seq_len), generator=g, device=device, dtype=torch.int32)
    seg = torch.zeros((batch, seq_len), device=device, dtype=torch.int32)
    seg[:, seq_len // 2:] = 1
    mask = torch.ones((batch, seq_len), device=device, dtype=torch.int32)
    pos = torch.stack([torch.randperm(seq_len, generator=torch.Generator().manual_seed(seed + i))[:max_predictions]
                       for i in range(batch)]).to(device=device, dtype=torch.int32)
    mlm_ids = torch.randint(0, vocab, (batch, max_predictions), generator=g, device=device, dtype=torch.int32)
    nsp = torch.randint(0, 2, (batch,), generator=g, device=device, dtype=torch.int32)
    b = {"input_ids": ids, "segment_ids": seg, "input_mask": mask, "masked_lm_positions": pos,
         "masked_lm_ids": mlm_ids, "next_sentence_labels": nsp}
    return Dataset(lambda: itertools.repeat(b))
