"""Distribution: cluster spec / TF_CONFIG, parameter-server runtime, bucketed RCCL
all-reduce and the tf.distribute-compatible strategies."""
from .cluster import ClusterSpec, TFConfigClusterResolver, make_tf_config
from .collective import BucketedAllReducer, allreduce_mean_, broadcast_flat_
from .ps import (DeviceSetter, GreedyLoadBalancingStrategy, PSClient, Server, current_device_setter, device,
                 replica_device_setter)
from .strategy import (CommunicationImplementation, CommunicationOptions, CrossDeviceOps, HierarchicalCopyAllReduce,
                       InputContext, MirroredStrategy, MultiWorkerMirroredStrategy, NcclAllReduce, OneDeviceStrategy,
                       ParameterServerStrategy, RcclAllReduce, ReduceOp, ReductionToOneDevice, Strategy,
                       get_strategy, has_strategy, in_cross_replica_context)
from .fault import FaultInjectionHook, FaultInjector, Heartbeat, HeartbeatHook, as_preemption_error
