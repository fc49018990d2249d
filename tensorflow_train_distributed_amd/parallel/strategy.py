"""tf.distribute.Strategy-compatible API, MI355X-native underneath.

* MirroredStrategy — synchronous data parallelism across the GPUs of one node. MI355X-first
  design: ONE PROCESS PER GPU (launch with torch.distributed.run), each process one replica;
  gradient aggregation is the bucketed, backward-overlapped RCCL all-reduce over xGMI
  (parallel/collective.py). A single process without a launcher is a 1-replica mirror.
* MultiWorkerMirroredStrategy — the same across nodes, cluster from TF_CONFIG
  (rank = worker index, rendezvous at worker 0's address).
* OneDeviceStrategy, ParameterServerStrategy (variables on PS tasks via
  replica_device_setter; see parallel/ps.py) and the cross-replica helpers
  (reduce / gather / experimental_distribute_dataset / run).
CPU replicas use gloo (BASELINE.json config 1: MNIST MirroredStrategy on CPU).
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist

from .cluster import ClusterSpec, TFConfigClusterResolver, split_address


class ReduceOp:
    SUM = "SUM"
    MEAN = "MEAN"


class CommunicationImplementation:
    AUTO = "AUTO"
    RING = "RING"
    NCCL = "NCCL"  # == RCCL on ROCm
    RCCL = "NCCL"


class CommunicationOptions:
    def __init__(self, bytes_per_pack: int = 32 << 20, timeout_seconds: Optional[float] = None,
                 implementation: str = CommunicationImplementation.AUTO):
        self.bytes_per_pack = bytes_per_pack
        self.timeout_seconds = timeout_seconds
        self.implementation = implementation


class CrossDeviceOps:
    """Gradient aggregation policy (tf.distribute cross-device ops): reduction algorithm, bucket
    sizing (bucket_mb, or TF's num_packs = number of equal buckets) and optional bf16 compression
    on the wire. The algorithms are parallel/collective.py's BucketedAllReducer ALGORITHMS."""

    algorithm = "allreduce"

    def __init__(self, bucket_mb: float = 32.0, first_bucket_mb: float = 4.0, compress_bf16: bool = False,
                 num_packs: Optional[int] = None):
        self.bucket_mb = bucket_mb
        self.first_bucket_mb = first_bucket_mb
        self.compress_bf16 = compress_bf16
        self.num_packs = num_packs


class RcclAllReduce(CrossDeviceOps):
    """One RCCL all-reduce per bucket. num_packs=None keeps the overlap-oriented bucket sizing
    (first bucket small so communication starts early); num_packs=k packs the gradients into
    k equal buckets (TF semantics)."""

    def __init__(self, num_packs: Optional[int] = None, bucket_mb: float = 32.0, **kw):
        super().__init__(bucket_mb=bucket_mb, num_packs=num_packs, **kw)


NcclAllReduce = RcclAllReduce


class HierarchicalCopyAllReduce(CrossDeviceOps):
    """Reduce-scatter + all-gather per bucket (each replica reduces its 1/N shard)."""

    algorithm = "hierarchical"

    def __init__(self, num_packs: Optional[int] = None, **kw):
        super().__init__(num_packs=num_packs, **kw)


class ReductionToOneDevice(CrossDeviceOps):
    """Reduce every bucket onto replica 0, then broadcast it back (TF's ReductionToOneDevice)."""

    algorithm = "reduce_to_one"

    def __init__(self, reduce_to_device=None, accumulation_fn=None, **kw):
        super().__init__(**kw)
        self.reduce_to_device = reduce_to_device


_tls = threading.local()


def get_strategy(allow_default: bool = False) -> Optional["Strategy"]:
    st = getattr(_tls, "stack", None)
    if st:
        return st[-1]
    return None if allow_default else _default_strategy()


_DEFAULT = None


def _default_strategy():
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = OneDeviceStrategy("cuda:0" if torch.cuda.is_available() else "cpu")
    return _DEFAULT


def has_strategy() -> bool:
    return bool(getattr(_tls, "stack", None))


def in_cross_replica_context() -> bool:
    return has_strategy() and not getattr(_tls, "in_replica", False)


class InputContext:
    def __init__(self, num_input_pipelines=1, input_pipeline_id=0, num_replicas_in_sync=1):
        self.num_input_pipelines = num_input_pipelines
        self.input_pipeline_id = input_pipeline_id
        self.num_replicas_in_sync = num_replicas_in_sync

    def get_per_replica_batch_size(self, global_batch_size: int) -> int:
        if global_batch_size % self.num_replicas_in_sync:
            raise ValueError("global batch %d not divisible by %d replicas" % (global_batch_size,
                                                                               self.num_replicas_in_sync))
        return global_batch_size // self.num_replicas_in_sync


class _Extended:
    def __init__(self, strategy):
        self._s = strategy

    @property
    def worker_devices(self):
        return (str(self._s.device),)

    @property
    def parameter_devices(self):
        return (str(self._s.device),)

    def _num_replicas(self):
        return self._s.num_replicas_in_sync


class Strategy:
    def __init__(self, device, group=None, cross_device_ops: Optional[CrossDeviceOps] = None):
        self.device = torch.device(device)
        self.group = group
        self.cross_device_ops = cross_device_ops or RcclAllReduce()
        self.extended = _Extended(self)
        self.cluster_resolver = None

    # -- topology
    @property
    def num_replicas_in_sync(self) -> int:
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    @property
    def replica_id(self) -> int:
        return dist.get_rank(self.group) if dist.is_initialized() else 0

    @property
    def is_chief(self) -> bool:
        return self.replica_id == 0

    # -- scope
    @contextlib.contextmanager
    def scope(self):
        st = getattr(_tls, "stack", None)
        if st is None:
            st = _tls.stack = []
        st.append(self)
        try:
            if self.device.type == "cuda":
                with torch.cuda.device(self.device):
                    yield self
            else:
                yield self
        finally:
            st.pop()

    # -- replica execution
    def run(self, fn: Callable, args=(), kwargs=None):
        from ..train.optimizers import TrainOp
        kwargs = kwargs or {}
        _tls.in_replica = True
        try:
            with self.scope():
                if isinstance(fn, TrainOp):
                    return fn.run(*args, **kwargs)
                return fn(*args, **kwargs)
        finally:
            _tls.in_replica = False

    def make_reducer(self, params):
        from .collective import BucketedAllReducer, broadcast_flat_
        broadcast_flat_(params, group=self.group)
        c = self.cross_device_ops
        return BucketedAllReducer(params, group=self.group, bucket_mb=c.bucket_mb, first_bucket_mb=c.first_bucket_mb,
                                  compress_bf16=c.compress_bf16, algorithm=c.algorithm, num_packs=c.num_packs)

    def grad_scale(self, feed) -> float:
        n = None
        for v in feed.values():
            if hasattr(v, "shape") and len(v.shape) > 0:
                n = int(v.shape[0])
                break
        return 1.0 / (max(1, n or 1) * self.num_replicas_in_sync)

    # -- cross-replica ops
    def reduce(self, reduce_op, value, axis=None):
        if isinstance(value, dict):
            return {k: self.reduce(reduce_op, v, axis) for k, v in value.items()}
        t = torch.as_tensor(value, dtype=torch.float32)
        t = t.to(self._comm_device())
        if axis is not None:
            n_local = t.shape[axis]
            t = t.sum(dim=axis)
        else:
            n_local = 1
        if dist.is_initialized() and self.num_replicas_in_sync > 1:
            t = t.clone()
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        if reduce_op == ReduceOp.MEAN:
            t = t / (self.num_replicas_in_sync * (n_local if axis is not None else 1))
        return t

    def all_reduce(self, reduce_op, value):
        return self.reduce(reduce_op, value, axis=None)

    def gather(self, value, axis=0):
        t = torch.as_tensor(value).to(self._comm_device())
        if not dist.is_initialized() or self.num_replicas_in_sync == 1:
            return t
        parts = [torch.empty_like(t) for _ in range(self.num_replicas_in_sync)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim=axis)

    def barrier(self):
        if dist.is_initialized():
            dist.barrier(group=self.group)

    def recover(self):
        """Rebuild this strategy's communicator after a collective failure (next process-group
        generation, same ranks). The caller then restores + broadcasts the training state."""
        if self.group is None and reinit_process_group():
            self.recoveries = getattr(self, "recoveries", 0) + 1

    def experimental_local_results(self, value):
        return (value,)

    def experimental_distribute_dataset(self, dataset, options=None):
        from ..data.dataset import DistributedDataset
        return DistributedDataset(dataset, self.num_replicas_in_sync, self.replica_id)

    def distribute_datasets_from_function(self, dataset_fn, options=None):
        ctx = InputContext(self.num_replicas_in_sync, self.replica_id, self.num_replicas_in_sync)
        return dataset_fn(ctx)

    def _comm_device(self):
        if dist.is_initialized() and dist.get_backend(self.group) == "nccl":
            return self.device
        return torch.device("cpu")

    def __enter__(self):
        self._cm = self.scope()
        return self._cm.__enter__()

    def __exit__(self, *a):
        return self._cm.__exit__(*a)


_PG = {"store": None, "generation": 0, "args": None}


def _base_store(rank, world, init_method, timeout):
    """The rendezvous key-value store, created once per process and kept across process-group
    generations (recovery re-creates the group, not the store)."""
    if _PG["store"] is None:
        if init_method and init_method.startswith("tcp://"):
            host, port = init_method[len("tcp://"):].rsplit(":", 1)
            is_master, port = rank == 0, int(port)
        else:  # env:// (torch.distributed.run, or a launcher exporting MASTER_ADDR/PORT)
            host, port = os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ.get("MASTER_PORT", "29500"))
            # under torch.distributed.run the agent hosts the store; ranks are clients
            is_master = rank == 0 and os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() != "true"
        _PG["store"] = dist.TCPStore(host, port, world, is_master, timeout=timeout,
                                     wait_for_workers=False)
    return _PG["store"]


def _init_pg(rank, world, init_method=None, timeout_s=1800):
    """Default process group of this replica (RCCL on GPUs, gloo on the CPU), on a key prefix
    of the current generation so `reinit_process_group` can build a fresh one after a failure."""
    if dist.is_initialized():
        return
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count()))))
    timeout = datetime.timedelta(seconds=timeout_s)
    store = dist.PrefixStore("ttd_pg_gen%d" % _PG["generation"], _base_store(rank, world, init_method, timeout))
    _PG["args"] = (rank, world, init_method, timeout_s)
    dist.init_process_group(backend, store=store, rank=rank, world_size=world, timeout=timeout, **kw)


def reinit_process_group():
    """Tear down the (failed) default process group and build the next generation with the same
    ranks — the collective-side half of MonitoredTrainingSession's recovery."""
    if _PG["args"] is None:
        return False
    from . import rccl
    rccl.abort_all()  # the native communicators of the failed generation (peers may be gone)
    try:
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - an aborted communicator may fail to shut down cleanly
        pass
    _PG["generation"] += 1
    _init_pg(*_PG["args"])
    return True


def _launch_replicas(n: int):
    """MirroredStrategy() over n > 1 GPUs in a process that no launcher started: become the
    launcher (one process per GPU is the MI355X design). The script is re-run as n ranks by
    torch.distributed.run on 127.0.0.1 and this process exits with their status. Runs before
    anything touches a GPU (device_count() does not initialise one). TTD_MIRRORED_SPAWN=0
    raises instead; a script that cannot be re-run (interactive, -c) raises too."""
    if n <= 1:
        return
    import subprocess
    import sys
    script = sys.argv[0] if sys.argv else ""
    main = sys.modules.get("__main__")
    spec = getattr(main, "__spec__", None)
    # `python -m pkg.mod`: re-run as a module (a file path would break its relative imports)
    entry = ["-m", spec.name] if spec is not None and spec.name not in ("__main__", None) else [script]
    refuse = (os.environ.get("TTD_MIRRORED_SPAWN", "1") == "0" or not script or script == "-c"
              or not os.path.exists(script)
              # a test runner / an embedding process: relaunching would re-run the whole session
              or os.path.basename(script).startswith(("pytest", "py.test")) or "pytest" in sys.modules
              or (spec is not None and spec.name.split(".")[0] in ("pytest", "IPython", "ipykernel")))
    if refuse:
        raise RuntimeError("MirroredStrategy over %d GPUs needs one process per GPU: launch the script with "
                           "`python -m torch.distributed.run --nproc-per-node %d ...` (or pass devices=[...] "
                           "with one device)" % (n, n))
    import socket
    sck = socket.socket()
    sck.bind(("127.0.0.1", 0))
    port = sck.getsockname()[1]
    sck.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + entry + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


class MirroredStrategy(Strategy):
    """Synchronous all-reduce data parallelism on one node, one process per GPU."""

    def __init__(self, devices=None, cross_device_ops: Optional[CrossDeviceOps] = None):
        if "WORLD_SIZE" not in os.environ:
            _launch_replicas(len(devices) if isinstance(devices, (list, tuple)) else
                             (1 if devices is not None else torch.cuda.device_count()))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if devices:
            dev = torch.device(devices[local % len(devices)] if isinstance(devices, (list, tuple)) else devices)
        else:
            dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        if world > 1:
            _init_pg(rank, world)
        super().__init__(dev, cross_device_ops=cross_device_ops)


class MultiWorkerMirroredStrategy(Strategy):
    """All-reduce data parallelism across workers described by TF_CONFIG (every worker task
    is one process/GPU; worker 0 hosts the rendezvous)."""

    def __init__(self, cluster_resolver: Optional[TFConfigClusterResolver] = None,
                 communication_options: Optional[CommunicationOptions] = None):
        cr = cluster_resolver or TFConfigClusterResolver()
        spec = cr.cluster_spec()
        workers = spec.job_tasks("worker") if "worker" in spec.jobs else []
        chief = spec.job_tasks("chief") if "chief" in spec.jobs else []
        tasks = chief + workers
        world = max(1, len(tasks))
        rank = (cr.task_id + len(chief)) if cr.task_type == "worker" else 0
        opts = communication_options or CommunicationOptions()
        if world > 1:
            host, port = split_address(tasks[0])
            _init_pg(rank, world, init_method="tcp://%s:%d" % ("127.0.0.1" if host == "localhost" else host, port),
                     timeout_s=int(opts.timeout_seconds or 1800))
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
            dev = torch.device("cuda", local)
            torch.cuda.set_device(dev)
        else:
            dev = torch.device("cpu")
        super().__init__(dev, cross_device_ops=RcclAllReduce(bucket_mb=opts.bytes_per_pack / (1 << 20)))
        self.cluster_resolver = cr


class OneDeviceStrategy(Strategy):
    def __init__(self, device):
        super().__init__(device)

    @property
    def num_replicas_in_sync(self) -> int:
        return 1


class ParameterServerStrategy(Strategy):
    """Variables on `ps` tasks (round-robin), compute on this worker; updates through the
    native PS runtime (async Hogwild GD, or SyncReplicasOptimizer for synchronous)."""

    def __init__(self, cluster_resolver: Optional[TFConfigClusterResolver] = None, variable_partitioner=None):
        from .ps import replica_device_setter
        cr = cluster_resolver or TFConfigClusterResolver()
        self.cluster = cr.cluster_spec()
        # one worker process per GPU: a launcher's LOCAL_RANK, else the task index over the
        # node's GPUs (the same mapping as examples/distribute_training.py --device gpu)
        if torch.cuda.is_available():
            n = max(1, torch.cuda.device_count())
            dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", cr.task_id % n)))
            torch.cuda.set_device(dev)
        else:
            dev = torch.device("cpu")
        super().__init__(dev)
        self.cluster_resolver = cr
        self.device_setter = replica_device_setter(cluster=self.cluster,
                                                   worker_device="/job:worker/task:%d" % cr.task_id,
                                                   ps_strategy=variable_partitioner)

    @property
    def num_replicas_in_sync(self) -> int:
        return max(1, self.cluster.num_tasks("worker"))

    @contextlib.contextmanager
    def scope(self):
        from .ps import device
        with super().scope(), device(self.device_setter):
            yield self
