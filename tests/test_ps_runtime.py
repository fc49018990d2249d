"""Native parameter-server runtime: variable store, Hogwild apply, ConditionalAccumulator
stale-drop + mean, token queue, sharded save/merge/restore, shutdown (no GPU)."""
import socket
import threading
import time

import numpy as np
import pytest

from tensorflow_train_distributed_amd.parallel import ps as PS
from tensorflow_train_distributed_amd.parallel.cluster import ClusterSpec
from tensorflow_train_distributed_amd.train import checkpoint as C
from tensorflow_train_distributed_amd.utils import errors


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


@pytest.fixture
def cluster2():
    ports = free_ports(3)
    cluster = ClusterSpec({"ps": ["127.0.0.1:%d" % ports[0], "127.0.0.1:%d" % ports[1]],
                           "worker": ["127.0.0.1:%d" % ports[2]]})
    servers = [PS.Server(cluster, "ps", i) for i in range(2)]
    yield cluster, servers
    for s in servers:
        s.stop()


def test_init_pull_apply_gd(cluster2):
    cluster, servers = cluster2
    setter = PS.replica_device_setter(cluster=cluster)
    for n in ["global_step", "a/kernel", "a/bias", "b/kernel"]:
        setter.assign(n)
    assert setter.placement == {"global_step": 0, "a/kernel": 1, "a/bias": 0, "b/kernel": 1}
    vals = {"a/kernel": np.arange(6, dtype=np.float32).reshape(2, 3), "a/bias": np.ones(3, np.float32),
            "b/kernel": np.full(4, 2.0, np.float32)}
    cl = PS.PSClient(cluster, {k: setter.placement[k] for k in vals})
    assert not cl.is_ready()
    cl.init_vars(vals)
    cl.set_ready()
    assert cl.is_ready()
    out = {k: np.zeros_like(v) for k, v in vals.items()}
    cl.pull(out)
    for k in vals:
        np.testing.assert_array_equal(out[k], vals[k])
    grads = {k: np.ones_like(v) for k, v in vals.items()}
    assert cl.apply_gd(0.5, grads) == 1
    assert cl.apply_gd(0.5, grads) == 2
    cl.pull(out)
    np.testing.assert_allclose(out["a/kernel"], vals["a/kernel"] - 1.0)
    assert cl.global_step() == 2
    cl.close()


def test_sync_replicas_accumulator_semantics(cluster2):
    cluster, _ = cluster2
    vals = {"w": np.zeros(4, np.float32), "v": np.zeros(2, np.float32)}
    cl = PS.PSClient(cluster, {"w": 0, "v": 1})
    cl.init_vars(vals)
    cl.set_accum_step(0)
    # two fresh gradients for step 0
    assert cl.accum_apply(0, {"w": np.full(4, 1.0, np.float32), "v": np.full(2, 2.0, np.float32)}) == 2
    assert cl.accum_apply(0, {"w": np.full(4, 3.0, np.float32), "v": np.full(2, 4.0, np.float32)}) == 2
    gs = cl.take_apply(2, 0.1, tokens_per_step=2)
    assert gs == 1
    out = {k: np.zeros_like(v) for k, v in vals.items()}
    cl.pull(out)
    np.testing.assert_allclose(out["w"], -0.1 * 2.0)  # mean(1, 3)
    np.testing.assert_allclose(out["v"], -0.1 * 3.0)
    assert cl.dequeue_token() == 1 and cl.dequeue_token() == 1
    # a gradient computed at the old step is stale now and silently dropped
    assert cl.accum_apply(0, {"w": np.ones(4, np.float32)}) == 0
    assert cl.stats()["dropped"] >= 1
    # take blocks until enough fresh gradients arrive
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("gs", cl.take_apply(1, 0.1, 1)))
    th.start()
    time.sleep(0.3)
    assert th.is_alive()
    cl2 = PS.PSClient(cluster, {"w": 0, "v": 1})
    cl2.accum_apply(1, {"w": np.ones(4, np.float32), "v": np.ones(2, np.float32)})
    th.join(10)
    assert res["gs"] == 2
    cl.close_queue()
    with pytest.raises(errors.OutOfRangeError):
        cl2.dequeue_token()  # token from step 2 was... consumed below? queue has 1 token
        cl2.dequeue_token()
    cl.close()
    cl2.close()


def test_sync_replicas_backup_worker_semantics(cluster2):
    """SyncReplicasOptimizer(replicas_to_aggregate=2, total_num_replicas=3) (SURVEY.md §4.2
    fault injection): the chief applies as soon as 2 fresh gradients are in — the slow (or dead)
    third worker does not block the step — every worker still gets a token, and the straggler's
    gradient for the old step is dropped as stale."""
    cluster, _ = cluster2
    vals = {"w": np.zeros(4, np.float32), "v": np.zeros(2, np.float32)}
    workers = [PS.PSClient(cluster, {"w": 0, "v": 1}) for _ in range(3)]
    chief = workers[0]
    chief.init_vars(vals)
    chief.set_accum_step(0)
    assert workers[0].accum_apply(0, {"w": np.full(4, 2.0, np.float32), "v": np.full(2, 2.0, np.float32)}) == 2
    assert workers[1].accum_apply(0, {"w": np.full(4, 4.0, np.float32), "v": np.full(2, 4.0, np.float32)}) == 2
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("gs", chief.take_apply(2, 0.5, tokens_per_step=3)))
    th.start()
    th.join(10)
    assert not th.is_alive() and res["gs"] == 1  # did not wait for the third replica
    out = {k: np.zeros_like(v) for k, v in vals.items()}
    chief.pull(out)
    np.testing.assert_allclose(out["w"], -0.5 * 3.0)  # mean of the two fresh gradients
    # the straggler computed against step 0: stale now, dropped
    assert workers[2].accum_apply(0, {"w": np.full(4, 100.0, np.float32), "v": np.ones(2, np.float32)}) == 0
    assert all(w.dequeue_token() == 1 for w in workers)  # one token per replica (total_num_replicas)
    chief.pull(out)
    np.testing.assert_allclose(out["w"], -0.5 * 3.0)
    for w in workers:
        w.close()


def test_sharded_save_merge_restore(cluster2, tmp_path):
    cluster, _ = cluster2
    vals = {"x": np.arange(5, dtype=np.float32), "y": np.full(3, 7.0, np.float32)}
    cl = PS.PSClient(cluster, {"x": 0, "y": 1})
    cl.init_vars(vals)
    cl.set_global_step(42)
    saver = C.Saver([])
    prefix = saver.save(None, str(tmp_path / "model.ckpt"), global_step=42,
                        shard_writers=[lambda p, t=t: cl.save_shard(t, p) for t in range(2)])
    r = C.BundleReader(prefix)
    assert r.num_shards == 2
    np.testing.assert_array_equal(r.read("x"), vals["x"])
    np.testing.assert_array_equal(r.read("y"), vals["y"])
    assert int(r.read("global_step")) == 42
    r.close()
    assert C.latest_checkpoint(str(tmp_path)) == prefix
    cl.apply_gd(1.0, {"x": np.ones(5, np.float32), "y": np.ones(3, np.float32)})
    cl.set_global_step(0)
    assert cl.restore(prefix) == 3
    out = {k: np.zeros_like(v) for k, v in vals.items()}
    cl.pull(out)
    np.testing.assert_array_equal(out["x"], vals["x"])
    assert cl.global_step() == 42
    cl.close()


def test_shutdown_unblocks_join_and_dead_ps_is_unavailable(cluster2):
    cluster, servers = cluster2
    cl = PS.PSClient(cluster, {})
    assert cl.ping(1) == 1
    t = threading.Thread(target=servers[1].join)
    t.start()
    cl.conns[1].call(PS.OP_SHUTDOWN)
    t.join(10)
    assert not t.is_alive()
    with pytest.raises(errors.UnavailableError):
        for _ in range(3):
            cl.ping(1)
            time.sleep(0.1)
    cl.close()
