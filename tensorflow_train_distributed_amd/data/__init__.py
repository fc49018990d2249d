"""Input pipelines: MNIST (IDX) reader with TF next_batch semantics, a small tf.data-style
Dataset, synthetic ImageNet/BERT inputs, native batch prefetch and device prefetch."""
from . import mnist
from .dataset import Dataset, DistributedDataset, synthetic_bert, synthetic_imagenet
from .prefetch import DevicePrefetcher, NativeBatchPrefetcher
