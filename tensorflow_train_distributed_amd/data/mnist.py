"""MNIST reader with the semantics of TF1's `tensorflow.examples.tutorials.mnist.input_data`.

Reference: `input_data.read_data_sets(DATA_PATH)` + `mnist.train.next_batch(128)`
(/root/reference/distribute_training.py:6,184,224); SURVEY.md §2.2 T27:
* IDX files `train-images-idx3-ubyte.gz`, `train-labels-idx1-ubyte.gz`,
  `t10k-images-idx3-ubyte.gz`, `t10k-labels-idx1-ubyte.gz` (gzip or raw);
* split train 55,000 / validation 5,000 (validation_size) / test 10,000;
* images float32 [N, 784] scaled to [0, 1]; labels uint8 (dense) or one-hot;
* next_batch: shuffle at the first epoch and every epoch boundary; a batch that crosses the
  boundary concatenates the tail of the old permutation and the head of the new one.
There is no network here: when files are missing, `read_data_sets` can write a
deterministic, learnable synthetic MNIST (class prototypes + noise) in the same IDX format.
The batch gather can run in the native prefetch thread (csrc/runtime/prefetch.cc) — the
README's multi-threaded "ReadByQueue" variant.
"""
from __future__ import annotations

import gzip
import os
import struct
from collections import namedtuple
from typing import Optional

import numpy as np

FILES = {
    "train_images": "train-images-idx3-ubyte.gz",
    "train_labels": "train-labels-idx1-ubyte.gz",
    "test_images": "t10k-images-idx3-ubyte.gz",
    "test_labels": "t10k-labels-idx1-ubyte.gz",
}

Datasets = namedtuple("Datasets", ["train", "validation", "test"])


def _open(path):
    if os.path.exists(path):
        return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")
    raw = path[:-3] if path.endswith(".gz") else path + ".gz"
    if os.path.exists(raw):
        return gzip.open(raw, "rb") if raw.endswith(".gz") else open(raw, "rb")
    raise FileNotFoundError(path)


def read_idx(path) -> np.ndarray:
    with _open(path) as f:
        data = f.read()
    zero, dtype_code, ndim = struct.unpack_from(">HBB", data, 0)
    if zero != 0 or dtype_code != 0x08:
        raise ValueError("%s: not an unsigned-byte IDX file (magic %04x%02x%02x)" % (path, zero, dtype_code, ndim))
    dims = struct.unpack_from(">%dI" % ndim, data, 4)
    off = 4 + 4 * ndim
    return np.frombuffer(data, dtype=np.uint8, offset=off, count=int(np.prod(dims))).reshape(dims).copy()


def write_idx(path, arr: np.ndarray):
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    hdr = struct.pack(">HBB", 0, 0x08, arr.ndim) + struct.pack(">%dI" % arr.ndim, *arr.shape)
    if path.endswith(".gz"):
        with gzip.open(path, "wb", compresslevel=1) as f:
            f.write(hdr + arr.tobytes())
    else:
        with open(path, "wb") as f:
            f.write(hdr + arr.tobytes())


def write_synthetic(train_dir: str, n_train: int = 60000, n_test: int = 10000, seed: int = 0, noise: float = 0.35):
    """Deterministic learnable stand-in for MNIST: 10 random smooth 28x28 prototypes per class,
    each sample = a random prototype of its class + pixel noise + random 0-2 px shift."""
    rng = np.random.RandomState(seed)
    os.makedirs(train_dir, exist_ok=True)
    protos = rng.rand(10, 3, 28, 28)
    k = np.ones(5) / 5.0
    for c in range(10):
        for p in range(3):
            img = protos[c, p]
            img = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 0, img)
            img = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, img)
            img = (img - img.min()) / (img.max() - img.min() + 1e-9)
            protos[c, p] = (img > 0.55).astype(np.float64)

    def make(n):
        labels = rng.randint(0, 10, size=n).astype(np.uint8)
        which = rng.randint(0, 3, size=n)
        imgs = protos[labels, which]
        sh = rng.randint(-2, 3, size=(n, 2))
        out = np.empty((n, 28, 28), dtype=np.float32)
        for dy in range(-2, 3):  # vectorised per distinct shift
            for dx in range(-2, 3):
                sel = (sh[:, 0] == dy) & (sh[:, 1] == dx)
                out[sel] = np.roll(np.roll(imgs[sel], dy, axis=1), dx, axis=2)
        out = np.clip(out + noise * rng.randn(n, 28, 28).astype(np.float32), 0.0, 1.0)
        return (out * 255).astype(np.uint8), labels

    tr_x, tr_y = make(n_train)
    te_x, te_y = make(n_test)
    write_idx(os.path.join(train_dir, FILES["train_images"]), tr_x)
    write_idx(os.path.join(train_dir, FILES["train_labels"]), tr_y)
    write_idx(os.path.join(train_dir, FILES["test_images"]), te_x)
    write_idx(os.path.join(train_dir, FILES["test_labels"]), te_y)


def dense_to_one_hot(labels, num_classes=10):
    out = np.zeros((labels.shape[0], num_classes), dtype=np.float32)
    out[np.arange(labels.shape[0]), labels.astype(np.int64)] = 1.0
    return out


class DataSet:
    def __init__(self, images: np.ndarray, labels: np.ndarray, one_hot: bool = False, reshape: bool = True,
                 dtype=np.float32, seed: Optional[int] = None, native_prefetch: bool = False, prefetch_depth: int = 4):
        assert images.shape[0] == labels.shape[0]
        self._num_examples = images.shape[0]
        if reshape and images.ndim == 4:
            images = images.reshape(images.shape[0], -1)
        elif reshape and images.ndim == 3:
            images = images.reshape(images.shape[0], images.shape[1] * images.shape[2])
        if dtype == np.float32 and images.dtype == np.uint8:
            images = images.astype(np.float32) * (1.0 / 255.0)
        self._images = np.ascontiguousarray(images)
        self._labels = np.ascontiguousarray(dense_to_one_hot(labels) if one_hot else labels)
        self._epochs_completed = 0
        self._index_in_epoch = 0
        self._rng = np.random.RandomState(seed)
        self._perm = None
        self._native = None
        self._native_cfg = (native_prefetch, prefetch_depth, seed)

    @property
    def images(self):
        return self._images

    @property
    def labels(self):
        return self._labels

    @property
    def num_examples(self):
        return self._num_examples

    @property
    def epochs_completed(self):
        return self._epochs_completed

    def _shuffle(self):
        perm = np.arange(self._num_examples)
        self._rng.shuffle(perm)
        self._images_s = self._images[perm]
        self._labels_s = self._labels[perm]

    def next_batch(self, batch_size: int, fake_data: bool = False, shuffle: bool = True):
        if self._native_cfg[0] and shuffle:
            return self._next_native(batch_size)
        start = self._index_in_epoch
        if self._epochs_completed == 0 and start == 0:
            if shuffle:
                self._shuffle()
            else:
                self._images_s, self._labels_s = self._images, self._labels
        if start + batch_size > self._num_examples:
            self._epochs_completed += 1
            rest = self._num_examples - start
            img_rest = self._images_s[start:self._num_examples]
            lab_rest = self._labels_s[start:self._num_examples]
            if shuffle:
                self._shuffle()
            start = 0
            self._index_in_epoch = batch_size - rest
            end = self._index_in_epoch
            return (np.concatenate((img_rest, self._images_s[start:end]), axis=0),
                    np.concatenate((lab_rest, self._labels_s[start:end]), axis=0))
        self._index_in_epoch += batch_size
        end = self._index_in_epoch
        return self._images_s[start:end], self._labels_s[start:end]

    def _next_native(self, batch_size):
        from .prefetch import NativeBatchPrefetcher
        if self._native is None or self._native.batch != batch_size:
            _, depth, seed = self._native_cfg
            self._native = NativeBatchPrefetcher(self._images, self._labels, batch_size, depth=depth,
                                                 seed=0 if seed is None else seed)
        x, y, epochs = self._native.next()
        self._epochs_completed = epochs
        return x, y


def read_data_sets(train_dir: str, fake_data: bool = False, one_hot: bool = False, dtype=np.float32,
                   reshape: bool = True, validation_size: int = 5000, seed: Optional[int] = None,
                   synthetic_if_missing: bool = True, native_prefetch: bool = False) -> Datasets:
    if fake_data:
        def fake():
            return DataSet(np.zeros((0, 784), np.float32), np.zeros((0,), np.uint8), one_hot=one_hot)
        return Datasets(fake(), fake(), fake())
    path = os.path.join(train_dir, FILES["train_images"])
    try:
        read_idx(path)
    except FileNotFoundError:
        if not synthetic_if_missing:
            raise
        write_synthetic(train_dir)
    tr_x = read_idx(os.path.join(train_dir, FILES["train_images"]))
    tr_y = read_idx(os.path.join(train_dir, FILES["train_labels"]))
    te_x = read_idx(os.path.join(train_dir, FILES["test_images"]))
    te_y = read_idx(os.path.join(train_dir, FILES["test_labels"]))
    if not 0 <= validation_size <= len(tr_x):
        raise ValueError("validation_size must be in [0, %d]" % len(tr_x))
    va_x, va_y = tr_x[:validation_size], tr_y[:validation_size]
    tr_x, tr_y = tr_x[validation_size:], tr_y[validation_size:]
    kw = dict(one_hot=one_hot, reshape=reshape, dtype=dtype, seed=seed)
    return Datasets(DataSet(tr_x, tr_y, native_prefetch=native_prefetch, **kw), DataSet(va_x, va_y, **kw),
                    DataSet(te_x, te_y, **kw))
