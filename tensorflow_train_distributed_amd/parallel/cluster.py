"""Cluster description: `tf.train.ClusterSpec` and the `TF_CONFIG` resolver.

Reference: `tf.train.ClusterSpec({"ps": ps_hosts, "worker": worker_hosts})` built from the
comma-separated `--ps_hosts/--worker_hosts` flags (/root/reference/distribute_training.py:
170-173); the task index is the position in the job's list. `TF_CONFIG`
(`{"cluster": {...}, "task": {"type": "worker", "index": 0}}`) is how
MultiWorkerMirroredStrategy / ParameterServerStrategy discover their cluster (north star).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Union


class ClusterSpec:
    def __init__(self, cluster: Union[Dict[str, Union[List[str], Dict[int, str]]], "ClusterSpec", None] = None):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        self._jobs: Dict[str, Dict[int, str]] = {}
        for job, tasks in (cluster or {}).items():
            if isinstance(tasks, dict):
                self._jobs[job] = {int(k): v for k, v in tasks.items()}
            else:
                self._jobs[job] = {i: a for i, a in enumerate(tasks)}

    @property
    def jobs(self) -> List[str]:
        return sorted(self._jobs)

    def num_tasks(self, job: str) -> int:
        return len(self._jobs.get(job, {}))

    def task_indices(self, job: str) -> List[int]:
        return sorted(self._jobs.get(job, {}))

    def task_address(self, job: str, index: int) -> str:
        try:
            return self._jobs[job][int(index)]
        except KeyError:
            raise ValueError("no task %s:%d in cluster %s" % (job, index, self.as_dict()))

    def job_tasks(self, job: str) -> List[str]:
        return [self._jobs[job][i] for i in self.task_indices(job)]

    def as_dict(self) -> Dict[str, List[str]]:
        return {j: self.job_tasks(j) for j in self.jobs}

    def as_cluster_def(self):
        return self.as_dict()

    def __bool__(self):
        return bool(self._jobs)

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and self.as_dict() == other.as_dict()

    def __repr__(self):
        return "ClusterSpec(%r)" % self.as_dict()


def split_address(addr: str):
    host, _, port = addr.rpartition(":")
    if not host:
        raise ValueError("address %r needs host:port" % addr)
    return host, int(port)


class TFConfigClusterResolver:
    """Reads TF_CONFIG (or an explicit dict)."""

    def __init__(self, tf_config: Optional[Union[str, dict]] = None, rpc_layer: str = "grpc"):
        if tf_config is None:
            tf_config = os.environ.get("TF_CONFIG", "{}")
        cfg = json.loads(tf_config) if isinstance(tf_config, str) else dict(tf_config)
        self._cfg = cfg
        self.rpc_layer = rpc_layer
        task = cfg.get("task", {})
        self.task_type = task.get("type")
        self.task_id = int(task.get("index", 0))

    def cluster_spec(self) -> ClusterSpec:
        return ClusterSpec(self._cfg.get("cluster", {}))

    def master(self, task_type=None, task_id=None) -> str:
        t = task_type or self.task_type
        i = self.task_id if task_id is None else task_id
        if not t:
            return ""
        return "%s://%s" % (self.rpc_layer, self.cluster_spec().task_address(t, i))

    def num_accelerators(self):
        import torch
        return {"GPU": torch.cuda.device_count()} if torch.cuda.is_available() else {}

    @property
    def environment(self):
        return self._cfg.get("environment", "")


def make_tf_config(cluster: Union[ClusterSpec, dict], task_type: str, task_index: int) -> str:
    c = cluster.as_dict() if isinstance(cluster, ClusterSpec) else cluster
    return json.dumps({"cluster": c, "task": {"type": task_type, "index": task_index}})
