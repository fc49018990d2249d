"""Failure detection and fault injection: PS heartbeat that unblocks a
worker stuck in the SyncReplicas token dequeue when the PS dies (the reference hangs there,
SURVEY §2.9 Q6), injected RPC failures/delays, preemption at a chosen global step with
MonitoredTrainingSession recovery, and collective-error mapping (no GPU)."""
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.parallel import fault
from tensorflow_train_distributed_amd.parallel import ps as PS
from tensorflow_train_distributed_amd.parallel.cluster import ClusterSpec
from tensorflow_train_distributed_amd.utils import errors


def _cluster():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cluster = ClusterSpec({"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1"]})
    return cluster, PS.Server(cluster, "ps", 0)


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PS_MAIN = """
import sys
from tensorflow_train_distributed_amd.parallel import ps as PS
from tensorflow_train_distributed_amd.parallel.cluster import ClusterSpec
s = PS.Server(ClusterSpec({"ps": [sys.argv[1]], "worker": ["127.0.0.1:1"]}), "ps", 0)
print("ready", flush=True)
s.join()
"""


def test_heartbeat_unblocks_token_dequeue_when_ps_hangs():
    cluster, server = _cluster()
    server.stop()  # free the port; the PS runs in a child process that gets SIGKILLed
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    proc = subprocess.Popen([sys.executable, "-c", PS_MAIN, cluster.task_address("ps", 0)], env=env,
                            stdout=subprocess.PIPE, text=True)
    assert proc.stdout.readline().strip() == "ready"
    client = PS.PSClient(cluster, {})
    failed = []
    hb = fault.Heartbeat(client, interval=0.05, max_missed=2, timeout_ms=500, on_failure=failed.append)
    hb.check_once()
    assert hb.healthy and hb.missed == [0]
    result = {}

    def worker():
        try:
            client.dequeue_token()  # blocks: the queue is empty and nobody will enqueue
        except errors.OpError as e:
            result["err"] = e
    t = threading.Thread(target=worker)
    t.start()
    time.sleep(0.2)
    assert t.is_alive()
    hb.start()
    # the PS host hangs (no TCP reset reaches the worker, so only the heartbeat can notice)
    proc.send_signal(signal.SIGSTOP)
    try:
        t.join(15)
    finally:
        hb.stop()
        proc.kill()
        proc.wait()
    assert not t.is_alive(), "dequeue still blocked after the PS died"
    assert isinstance(result.get("err"), errors.UnavailableError)
    assert failed == [0] and not hb.healthy
    client.close()


def test_fault_injector_fails_and_delays_selected_rpcs():
    cluster, server = _cluster()
    try:
        client = PS.PSClient(cluster, {"v": 0})
        client.init_vars({"v": np.zeros(4, np.float32)})
        inj = fault.FaultInjector().fail(op=PS.OP_APPLY_GD, at=(1,)).delay(0.05, op=PS.OP_PING, at=(0,))
        inj.install(client)
        g = {"v": np.ones(4, np.float32)}
        assert client.apply_gd(0.1, g) == 1
        with pytest.raises(errors.UnavailableError, match="injected"):
            client.apply_gd(0.1, g)
        assert client.apply_gd(0.1, g) == 2  # the failed call never reached the PS
        t0 = time.time()
        client.ping(0)
        assert time.time() - t0 >= 0.05
        assert [k for k, *_ in inj.log] == ["fail", "delay"]
        inj.uninstall()
        client.ping(0)
        assert len(inj.log) == 2
        client.close()
    finally:
        server.stop()


def test_injected_preemption_recovers_session_from_checkpoint(tmp_path):
    ttd.train.reset_default_graph()
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(seed=0, dropout_rate=0.0)
    op = ttd.train.GradientDescentOptimizer(0.05).minimize(model, global_step=gs)
    x = ttd.placeholder(None, [None, 784], "x-input")
    y = ttd.placeholder(None, [None], "y-input")
    rng = np.random.default_rng(0)
    inj = fault.FaultInjectionHook(at_step=12)
    steps = []
    with ttd.train.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), save_checkpoint_steps=5,
                                            hooks=[ttd.train.StopAtStepHook(last_step=20), inj]) as sess:
        while not sess.should_stop():
            bx = rng.random((16, 784), dtype=np.float32)
            by = rng.integers(0, 10, 16)
            _, g = sess.run([op, gs], feed_dict={x: bx, y: by})
            steps.append(g)
        recoveries = sess.recoveries
    assert inj.fired and recoveries == 1
    assert steps[-1] == 20
    # the preempted run never executed; the re-created session restored checkpoint 10, so
    # global steps 11 and 12 are trained a second time
    assert steps[:12] == list(range(1, 13))
    assert steps[12:] == list(range(11, 21)), steps
    ttd.train.reset_default_graph()


def test_collective_errors_map_to_preemption():
    import torch.distributed as dist
    e = fault.as_preemption_error(RuntimeError("NCCL communicator was aborted on rank 3"))
    assert isinstance(e, errors.UnavailableError)
    if hasattr(dist, "DistBackendError"):
        assert isinstance(fault.as_preemption_error(dist.DistBackendError("x")), errors.UnavailableError)
    v = ValueError("shape mismatch")
    assert fault.as_preemption_error(v) is v
