"""tf.train.QueueRunner / start_queue_runners / SessionManager / SummaryWriterCache and the
tf-named PS views (token queue, accumulators) — SURVEY.md §2.2 T8-T11, T16, T18 (no GPU)."""
import socket
import threading
import time

import numpy as np
import pytest

import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.parallel import ps as PS
from tensorflow_train_distributed_amd.parallel.cluster import ClusterSpec
from tensorflow_train_distributed_amd.utils import errors


def test_queue_runner_runs_until_stop_and_closes():
    ttd.train.reset_default_graph()
    items, closed = [], []

    def enqueue():
        items.append(1)
        time.sleep(0.001)
        if len(items) >= 50:
            raise errors.OutOfRangeError("queue closed")
    qr = ttd.train.QueueRunner(enqueue_ops=[enqueue], close_op=lambda: closed.append(True))
    ttd.train.add_queue_runner(qr)
    coord = ttd.train.Coordinator()
    threads = ttd.train.start_queue_runners(coord=coord)
    for t in threads:
        t.join(10)
    assert len(items) == 50 and closed == [True] and not qr.exceptions_raised
    # a coordinator stop ends an endless runner; an error is reported through the coordinator
    qr2 = ttd.train.QueueRunner(enqueue_ops=[lambda: time.sleep(0.001)])
    coord2 = ttd.train.Coordinator()
    th = qr2.create_threads(None, coord=coord2, start=True)
    coord2.request_stop()
    coord2.join(th, stop_grace_period_secs=5)

    def bad():
        raise ValueError("boom")
    qr3 = ttd.train.QueueRunner(enqueue_ops=[bad])
    coord3 = ttd.train.Coordinator()
    th = qr3.create_threads(None, coord=coord3, start=True)
    for t in th:
        t.join(5)
    assert coord3.should_stop() and isinstance(qr3.exceptions_raised[0], ValueError)
    ttd.train.reset_default_graph()


def test_session_manager_prepare_restores_latest_checkpoint(tmp_path):
    ttd.train.reset_default_graph()
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(seed=0, dropout_rate=0.0)
    op = ttd.train.GradientDescentOptimizer(0.1).minimize(model, global_step=gs)
    with ttd.train.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), save_checkpoint_steps=3,
                                            hooks=[ttd.train.StopAtStepHook(last_step=3)]) as s:
        while not s.should_stop():
            s.run(op, feed_dict={"x-input": np.random.rand(8, 784).astype(np.float32),
                                 "y-input": np.random.randint(0, 10, 8)})
    saved = model.params.master.clone()
    model.params.master.zero_()
    gs.assign(0)
    sm = ttd.train.SessionManager()
    sess, restored = sm.recover_session(checkpoint_dir=str(tmp_path))
    assert restored and gs.value() == 3
    assert np.allclose(model.params.master.numpy(), saved.numpy())
    sess.close()
    assert ttd.train.SummaryWriterCache.get(str(tmp_path)) is ttd.train.SummaryWriterCache.get(str(tmp_path))
    ttd.train.reset_default_graph()


def test_token_queue_and_accumulator_views():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cluster = ClusterSpec({"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1"]})
    server = PS.Server(cluster, "ps", 0)
    try:
        client = PS.PSClient(cluster, {"v": 0})
        client.init_vars({"v": np.zeros(3, np.float32)})
        q = PS.TokenQueue(client)
        q.enqueue_many(2, 7)
        assert q.size() == 2 and q.dequeue() == 7 and q.dequeue() == 7 and q.size() == 0
        acc = PS.ConditionalAccumulatorSet(client)
        acc.set_global_step(5)
        acc.apply_grad(4, {"v": np.ones(3, np.float32)})  # stale: dropped
        acc.apply_grad(5, {"v": np.ones(3, np.float32)})
        assert acc.num_dropped() == 1
        got = {}

        def taker():
            got["gs"] = acc.take_apply(2, 0.5, 2)
        t = threading.Thread(target=taker)
        t.start()
        time.sleep(0.2)
        assert t.is_alive()  # waits for the second fresh gradient
        acc.apply_grad(5, {"v": 3 * np.ones(3, np.float32)})
        t.join(10)
        out = {"v": np.zeros(3, np.float32)}
        client.pull(out)
        np.testing.assert_allclose(out["v"], -0.5 * 2.0)  # mean of (1, 3) = 2
        assert q.size() == 2  # tokens_per_step enqueued by the aggregation
        q.close()
        with pytest.raises(errors.OutOfRangeError):
            q.dequeue()
            q.dequeue()
            q.dequeue()
        client.close()
    finally:
        server.stop()
