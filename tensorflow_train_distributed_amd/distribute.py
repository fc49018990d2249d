"""tf.distribute-shaped alias of `parallel` (MirroredStrategy, MultiWorkerMirroredStrategy,
ParameterServerStrategy, ReduceOp, cluster resolvers, cross-device ops)."""
from .parallel import *  # noqa: F401,F403
from .parallel.cluster import TFConfigClusterResolver as cluster_resolver_TFConfig  # noqa: F401


class cluster_resolver:  # tf.distribute.cluster_resolver.TFConfigClusterResolver
    from .parallel.cluster import TFConfigClusterResolver
