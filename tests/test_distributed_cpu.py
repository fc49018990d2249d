"""Multi-process distributed tests on localhost (CPU, gloo / native PS transport):
* the flag-compatible reference example, 1 PS + 2 workers, async and --sync_replicas;
* MirroredStrategy over gloo with world_size 2 (BASELINE config 1): replicas stay identical
  and match a single process that sees the concatenated batch;
* MultiWorkerMirroredStrategy from TF_CONFIG;
* PS failure: a parameter server is killed mid-training and restarted; the chief's session
  recovers and restores from the latest checkpoint.
"""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = [sys.executable, "-m", "tensorflow_train_distributed_amd.examples.distribute_training"]


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


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    from tensorflow_train_distributed_amd.data import mnist
    d = str(tmp_path_factory.mktemp("mnist"))
    mnist.write_synthetic(d, n_train=8000, n_test=500)
    return d


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    e["OMP_NUM_THREADS"] = "2"
    return e


def _run_cluster(tmp_path, mnist_dir, extra, steps=60):
    p = free_ports(3)
    common = ["--ps_hosts=127.0.0.1:%d" % p[0], "--worker_hosts=127.0.0.1:%d,127.0.0.1:%d" % (p[1], p[2]),
              "--checkpoint_dir=%s" % (tmp_path / "ck"), "--data_dir=%s" % mnist_dir,
              "--training_steps=%d" % steps, "--log_every=20", "--save_checkpoint_secs=1"] + extra
    env = _env()
    ps = subprocess.Popen(EXAMPLE + common + ["--job_name=ps", "--task_id=0"], env=env, cwd=REPO,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    time.sleep(0.5)
    w1 = subprocess.Popen(EXAMPLE + common + ["--job_name=worker", "--task_id=1"], env=env, cwd=REPO,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    w0 = subprocess.Popen(EXAMPLE + common + ["--job_name=worker", "--task_id=0"], env=env, cwd=REPO,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    outs = []
    try:
        for proc in (w0, w1, ps):
            out, _ = proc.communicate(timeout=180)
            outs.append(out)
            assert proc.returncode == 0, out[-3000:]
    finally:
        for proc in (w0, w1, ps):
            if proc.poll() is None:
                proc.kill()
    return outs


def _final_gs(out):
    line = [l for l in out.splitlines() if l.startswith("total step")][-1]
    return int(line.split("global_step:")[1])


@pytest.mark.slow
def test_reference_example_async(tmp_path, mnist_dir):
    from tensorflow_train_distributed_amd.train import checkpoint as C
    w0, w1, _ = _run_cluster(tmp_path, mnist_dir, [], steps=80)
    assert "session started" in w0 and "session started" in w1
    # async: every worker step increments the global step; both stop once it reaches 80
    assert _final_gs(w0) >= 80 and _final_gs(w1) >= 80
    latest = C.latest_checkpoint(str(tmp_path / "ck"))
    assert latest is not None
    keys = dict(C.list_variables(latest))
    assert {"hidden1/kernel", "output/bias", "global_step"} <= set(keys)
    assert int(C.load_variable(latest, "global_step")) >= 80


@pytest.mark.slow
def test_reference_example_sync_replicas(tmp_path, mnist_dir):
    w0, w1, _ = _run_cluster(tmp_path, mnist_dir, ["--sync_replicas"], steps=40)
    # sync: the global step counts aggregated updates; it ends exactly at the last step and the
    # non-chief worker is released by the closed token queue instead of hanging (Q6).
    assert _final_gs(w0) == 40
    assert "total step" in w1


MIRRORED_SCRIPT = r'''
import os, sys, json
import numpy as np, torch
import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.data import mnist
strategy = ttd.distribute.MirroredStrategy() if os.environ.get("MODE") == "mirrored" else \
    ttd.distribute.MultiWorkerMirroredStrategy()
rank, world = strategy.replica_id, strategy.num_replicas_in_sync
data = mnist.read_data_sets(sys.argv[1], seed=123)  # same stream on every replica
with strategy.scope():
    model = ttd.models.mnist_mlp(seed=7, dropout_rate=0.0)
    op = ttd.train.GradientDescentOptimizer(0.05).minimize(model)
losses = []
for step in range(5):
    bx, by = data.train.next_batch(64)  # global batch; each replica takes its shard
    feed = next(iter(strategy.experimental_distribute_dataset([(bx, by)])))
    out = strategy.run(op, args=({"x-input": feed[0], "y-input": feed[1]},))
    losses.append(float(strategy.reduce(ttd.distribute.ReduceOp.MEAN, out["loss"])))
w = model.params.master.clone()
ws = strategy.gather(w[None], axis=0)
json.dump({"rank": rank, "world": world, "losses": losses, "max_rep_diff": float((ws - ws[0]).abs().max()),
           "w": w[:2000].tolist()}, open(sys.argv[2] + "/r%d.json" % rank, "w"))
'''


def _launch_torchrun(tmp_path, mnist_dir, n, env_extra):
    script = tmp_path / "mirrored.py"
    script.write_text(MIRRORED_SCRIPT)
    port = free_ports(1)[0]
    env = _env()
    env.update(env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(script), mnist_dir, str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stdout[-3000:]
    return [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(n)]


@pytest.mark.slow
def test_mirrored_strategy_gloo_matches_single_process(tmp_path, mnist_dir):
    res = _launch_torchrun(tmp_path, mnist_dir, 2, {"MODE": "mirrored", "CUDA_VISIBLE_DEVICES": ""})
    assert res[0]["world"] == 2 and res[0]["max_rep_diff"] == 0.0
    # single process, full global batch, same init -> same weights (all-reduce mean == big batch)
    import tensorflow_train_distributed_amd as ttd
    from tensorflow_train_distributed_amd.data import mnist
    ttd.train.reset_default_graph()
    data = mnist.read_data_sets(mnist_dir, seed=123)
    model = ttd.models.mnist_mlp(seed=7, dropout_rate=0.0)
    op = ttd.train.GradientDescentOptimizer(0.05).minimize(model)
    for _ in range(5):
        bx, by = data.train.next_batch(64)
        op.run({"x-input": bx, "y-input": by})
    np.testing.assert_allclose(np.array(res[0]["w"]), model.params.master[:2000].numpy(), atol=2e-5)


@pytest.mark.slow
def test_multiworker_mirrored_from_tf_config(tmp_path, mnist_dir):
    ports = free_ports(2)
    cluster = {"worker": ["127.0.0.1:%d" % ports[0], "127.0.0.1:%d" % ports[1]]}
    script = tmp_path / "mirrored.py"
    script.write_text(MIRRORED_SCRIPT)
    procs = []
    for i in range(2):
        env = _env()
        env["TF_CONFIG"] = json.dumps({"cluster": cluster, "task": {"type": "worker", "index": i}})
        env["MODE"] = "multiworker"
        env["CUDA_VISIBLE_DEVICES"] = ""
        procs.append(subprocess.Popen([sys.executable, str(script), mnist_dir, str(tmp_path)], env=env, cwd=REPO,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out[-3000:]
    r0 = json.load(open(tmp_path / "r0.json"))
    r1 = json.load(open(tmp_path / "r1.json"))
    assert r0["world"] == 2 and r0["max_rep_diff"] == 0.0 and r0["losses"] == r1["losses"]


RECOVERY_SCRIPT = r'''
import os, sys, time, json
import numpy as np
import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.data import mnist
ps_addr, ckdir, data_dir, out = sys.argv[1:5]
cluster = ttd.train.ClusterSpec({"ps": [ps_addr], "worker": ["127.0.0.1:1"]})
server = ttd.train.Server(cluster, "worker", 0)
data = mnist.read_data_sets(data_dir, seed=0)
with ttd.device(ttd.train.replica_device_setter(cluster=cluster)):
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(seed=3)
    op = ttd.train.GradientDescentOptimizer(0.05).minimize(model, global_step=gs)
    steps = []
    with ttd.train.MonitoredTrainingSession(master=server.target, is_chief=True, checkpoint_dir=ckdir,
                                            hooks=[ttd.train.StopAtStepHook(last_step=int(sys.argv[5]))],
                                            save_checkpoint_steps=10) as sess:
        while not sess.should_stop():
            bx, by = data.train.next_batch(32)
            g = sess.run(gs, feed_dict={"x-input": bx, "y-input": by}) if False else \
                sess.run([op, gs], feed_dict={"x-input": bx, "y-input": by})[1]
            steps.append(g)
            time.sleep(0.01)
        json.dump({"steps": steps, "recoveries": sess.recoveries}, open(out, "w"))
'''

PS_SCRIPT = r'''
import sys
import tensorflow_train_distributed_amd as ttd
cluster = ttd.train.ClusterSpec({"ps": [sys.argv[1]], "worker": ["127.0.0.1:1"]})
s = ttd.train.Server(cluster, "ps", 0)
print("ready", flush=True)
s.join()
'''


@pytest.mark.slow
def test_ps_failure_recovery_restores_checkpoint(tmp_path, mnist_dir):
    port = free_ports(1)[0]
    addr = "127.0.0.1:%d" % port
    (tmp_path / "ps.py").write_text(PS_SCRIPT)
    (tmp_path / "chief.py").write_text(RECOVERY_SCRIPT)
    env = _env()

    def start_ps():
        p = subprocess.Popen([sys.executable, str(tmp_path / "ps.py"), addr], env=env, cwd=REPO,
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        assert p.stdout.readline().strip() == "ready"
        return p
    ps = start_ps()
    out = tmp_path / "res.json"
    chief = subprocess.Popen([sys.executable, str(tmp_path / "chief.py"), addr, str(tmp_path / "ck"), mnist_dir,
                              str(out), "400"], env=env, cwd=REPO, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True)
    try:
        from tensorflow_train_distributed_amd.train import checkpoint as C
        deadline = time.time() + 60
        while time.time() < deadline:  # wait for a checkpoint past step 30
            lc = C.latest_checkpoint(str(tmp_path / "ck"))
            if lc and int(lc.rsplit("-", 1)[1]) >= 30:
                break
            time.sleep(0.1)
        ps.send_signal(signal.SIGKILL)  # parameter server lost
        ps.wait()
        time.sleep(0.5)
        ps = start_ps()  # replacement task on the same address (state is gone)
        text, _ = chief.communicate(timeout=180)
        assert chief.returncode == 0, text[-3000:]
    finally:
        for p in (chief, ps):
            if p.poll() is None:
                p.kill()
    res = json.load(open(out))
    assert res["recoveries"] >= 1
    steps = res["steps"]
    assert steps[-1] == 400
    # after the PS restart the global step continued from a restored checkpoint (>= 30), it
    # did not restart from 0 with re-initialised variables
    first = next(i for i, s in enumerate(steps) if s >= 30)
    assert min(steps[first:]) >= 30


def _sync_on_read_worker(rank, world, store_path, q):
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel.collective import sync_on_read_mean_
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    dist.init_process_group("gloo", store=dist.FileStore(store_path, world), rank=rank, world_size=world)
    specs = [ParamSpec("w", (3,), None, True), ParamSpec("bn/moving_mean", (4,), None, False, trainable=False)]
    p = FlatParams(specs, "cpu", compute_dtype=None)
    p.var["w"].fill_(1.0 + rank)
    p.var["bn/moving_mean"].fill_(10.0 * (rank + 1))
    sync_on_read_mean_(p)
    q.put((rank, p.var["w"].tolist(), p.var["bn/moving_mean"].tolist()))
    dist.destroy_process_group()


def test_sync_on_read_averages_non_trainable_only(tmp_path):
    """BN moving statistics follow TF's SyncOnRead(MEAN): averaged across replicas when read
    for a checkpoint; trainable variables are left alone (they are kept identical by the
    gradient all-reduce)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sync_on_read_worker, args=(r, 2, str(tmp_path / "store"), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res[0][2] == [15.0] * 4 and res[1][2] == [15.0] * 4
    assert res[0][1] == [1.0] * 3 and res[1][1] == [2.0] * 3
