"""tensorflow_train_distributed_amd — an MI355X-native distributed training framework.

Capabilities of boyuanf/tensorflow_train_distributed (a TF1 parameter-server trainer,
/root/reference/distribute_training.py) re-designed for AMD Instinct MI355X (gfx950):
PyTorch-ROCm tensors, hand-written CDNA4 HIP kernels, RCCL collectives over xGMI, a native
C++ runtime (parameter server, checkpoint/event IO, data prefetch) and a
tf.distribute/tf.train-shaped public API:

    import tensorflow_train_distributed_amd as ttd
    ttd.train.MonitoredTrainingSession / ttd.train.SyncReplicasOptimizer / ttd.train.Server
    ttd.distribute.MirroredStrategy / MultiWorkerMirroredStrategy / ParameterServerStrategy
    ttd.train.Checkpoint / CheckpointManager (TensorBundle V2 on disk)
"""
__version__ = "0.1.0"

from . import data, distribute, initializers, layers, models, nn, parallel, regularizers, summary, train  # noqa: E402
from .parallel.ps import device  # noqa: E402
from .utils import app, errors, flags, tracing  # noqa: E402
from .utils.run_config import RunConfig  # noqa: E402
from .utils import tracing as debugging  # noqa: E402  (tf.debugging.check_numerics)
from .utils import tracing as profiler  # noqa: E402  (roctx ranges)
from .train.graph import placeholder  # noqa: E402
from .train.tape import GradientTape, clip_by_global_norm  # noqa: E402
from .nn import reduce_mean, matmul, sigmoid, tanh  # noqa: E402  (tf.reduce_mean / tf.matmul / tf.sigmoid / tf.tanh)
