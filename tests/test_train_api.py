"""tf.train-shaped API on CPU: flags, schedules, MLP parity constants, MonitoredTrainingSession
with hooks, checkpoint/summary output and resume, data pipeline semantics."""
import math
import os

import numpy as np
import pytest
import torch

import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.data import mnist
from tensorflow_train_distributed_amd.utils.flags import FlagValues, DEFINE_string, DEFINE_integer, DEFINE_boolean


@pytest.fixture(autouse=True)
def fresh_graph():
    ttd.train.reset_default_graph()
    yield
    ttd.summary.FileWriterCache.clear()


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("mnist"))
    mnist.write_synthetic(d, n_train=6000, n_test=1000)
    return d


def test_flags_parsing():
    F = FlagValues()
    DEFINE_string("job_name", "worker", "", flag_values=F)
    DEFINE_integer("task_id", 0, "", flag_values=F)
    DEFINE_boolean("sync_replicas", False, "", flag_values=F)
    rest = F(["prog", "--job_name=ps", "--task_id", "3", "--sync_replicas", "extra"])
    assert (F.job_name, F.task_id, F.sync_replicas) == ("ps", 3, True) and rest == ["prog", "extra"]
    F.reset()
    F(["prog", "--nosync_replicas"])
    assert F.sync_replicas is False


def test_exponential_decay_staircase_reference_values():
    gs = ttd.train.get_or_create_global_step()
    lr = ttd.train.exponential_decay(0.01, gs, int(60000 / 128), 0.96, staircase=True)
    assert lr.decay_steps == 468  # 60000 (not 55000) / 128
    assert lr(467) == pytest.approx(0.01) and lr(468) == pytest.approx(0.0096)
    assert lr(936) == pytest.approx(0.01 * 0.96 ** 2)


def test_mlp_parity_constants():
    m = ttd.models.mnist_mlp()
    n = sum(int(np.prod(s.shape)) for s in m.params.specs)
    assert n == 183685
    assert m.creation_order()[:3] == ["hidden1/kernel", "hidden1/bias", "hidden2/kernel"]
    w = m.params.var["hidden1/kernel"]
    sigma = math.sqrt(1.3 * 2 / 784)
    assert float(w.abs().max()) <= 2 * sigma + 1e-6
    assert abs(float(w.std()) - sigma * 0.8796) < 0.003  # std of a +-2-sigma truncated normal
    assert float(m.params.var["hidden1/bias"].abs().sum()) == 0


def test_next_batch_epoch_semantics():
    x = np.arange(10, dtype=np.float32)[:, None].repeat(3, 1)
    y = np.arange(10, dtype=np.uint8)
    ds = mnist.DataSet(x, y, reshape=False, seed=1)
    seen = []
    for _ in range(3):
        bx, by = ds.next_batch(4)
        seen.append(by)
        assert bx.shape == (4, 3)
    first_epoch = np.concatenate(seen)[:10]
    assert sorted(first_epoch.tolist()) == list(range(10))  # boundary batch = tail + head of new perm
    assert ds.epochs_completed == 1
    pf = mnist.DataSet(x, y, reshape=False, seed=1, native_prefetch=True)
    got = np.concatenate([pf.next_batch(5)[1] for _ in range(4)])
    assert sorted(got[:10].tolist()) == list(range(10)) and sorted(got[10:].tolist()) == list(range(10))


def _train_local(ckdir, mnist_dir, steps, hooks=(), save_steps=25):
    data = mnist.read_data_sets(mnist_dir, seed=0)
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(seed=0)
    lr = ttd.train.exponential_decay(0.02, gs, 468, 0.96, staircase=True)
    op = ttd.train.MomentumOptimizer(lr, 0.9).minimize(model, global_step=gs)
    ttd.summary.scalar("loss_0", op.loss)
    ttd.summary.scalar("accuracy_0", op.accuracy)
    x = ttd.placeholder(torch.float32, [None, 784], "x-input")
    y = ttd.placeholder(torch.int64, [None], "y-input")
    logs = []
    with ttd.train.MonitoredTrainingSession(checkpoint_dir=ckdir, hooks=[ttd.train.StopAtStepHook(last_step=steps)]
                                            + list(hooks), save_checkpoint_steps=save_steps,
                                            save_summaries_steps=10) as sess:
        while not sess.should_stop():
            bx, by = data.train.next_batch(64)
            _, l, a, g = sess.run([op, op.loss, op.accuracy, gs], feed_dict={x: bx, y: by})
            logs.append((g, l, a))
    return logs, model, op


def test_monitored_training_session_local(tmp_path, mnist_dir):
    ck = str(tmp_path / "ck")
    logs, model, op = _train_local(ck, mnist_dir, 120)
    assert logs[-1][0] == 120 and len(logs) == 120
    assert np.mean([l for _, l, _ in logs[-20:]]) < np.mean([l for _, l, _ in logs[:20]]) - 0.3
    latest = ttd.train.latest_checkpoint(ck)
    assert latest.endswith("model.ckpt-120")
    keys = dict(ttd.train.list_variables(latest))
    assert keys["hidden1/kernel"] == (784, 200) and "global_step" in keys
    assert "hidden1/kernel/Momentum" in keys
    ev = [f for f in os.listdir(ck) if f.startswith("events.out.tfevents")]
    assert ev
    events = ttd.summary.read_events(os.path.join(ck, ev[0]))
    tags = {t for e in events for t, _ in e.get("summary", [])}
    assert {"loss_0", "accuracy_0", "global_step/sec"} <= tags
    # relaunch resumes from the checkpoint (stable checkpoint_dir)
    ttd.train.reset_default_graph()
    logs2, model2, _ = _train_local(ck, mnist_dir, 150)
    assert logs2[0][0] == 121 and logs2[-1][0] == 150
    assert len(logs2) == 30


def test_hooks_logging_nan_and_final_ops(tmp_path, mnist_dir):
    data = mnist.read_data_sets(mnist_dir, seed=0)
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(seed=1)
    op = ttd.train.GradientDescentOptimizer(0.05).minimize(model, global_step=gs)
    lh = ttd.train.LoggingTensorHook({"loss": op.loss, "step": gs}, every_n_iter=5)
    nh = ttd.train.NanTensorHook(op.loss)
    fh = ttd.train.FinalOpsHook({"gs": gs})
    feed = ttd.train.FeedFnHook(lambda: dict(zip(["x-input", "y-input"], data.train.next_batch(32))))
    with ttd.train.MonitoredTrainingSession(hooks=[ttd.train.StopAtStepHook(num_steps=12), lh, nh, fh, feed]) as s:
        while not s.should_stop():
            s.run(op)
    assert [d["step"] for d in lh.logged] == [1, 6, 11]
    assert fh.final_ops_values == {"gs": 12}


def test_object_checkpoint_of_model_and_optimizer(tmp_path):
    model = ttd.models.mnist_mlp(seed=2)
    opt = ttd.train.AdamOptimizer(0.01)
    op = opt.minimize(model)
    ck = ttd.train.Checkpoint(model=model, optimizer=opt.flat)
    mgr = ttd.train.CheckpointManager(ck, str(tmp_path), max_to_keep=3)
    path = mgr.save()
    keys = dict(ttd.train.list_variables(path))
    assert "model/output/kernel/.ATTRIBUTES/VARIABLE_VALUE" in keys
    assert "model/output/kernel/.OPTIMIZER_SLOT/optimizer/v/.ATTRIBUTES/VARIABLE_VALUE" in keys


def test_run_config_layers_file_env_and_flags(tmp_path):
    """Typed RunConfig: defaults <- file <- TTD_RUN_* env <- flags; the
    reference's constants (distribute_training.py:10-36) as a preset; invalid values raise."""
    import argparse
    import json
    from tensorflow_train_distributed_amd.utils.run_config import RunConfig
    ref = RunConfig.reference_mnist()
    assert (ref.per_replica_batch, ref.learning_rate, ref.decay_steps, ref.decay_rate, ref.train_steps,
            ref.save_checkpoints_secs, ref.save_summary_steps) == (128, 0.01, 500, 0.96, 10000, 60.0, 100)
    f = tmp_path / "rc.json"
    f.write_text(json.dumps({"model": "bert", "bucket_mb": 64, "hipgraph": "true", "my_note": "x"}))
    ap = RunConfig.add_arguments(argparse.ArgumentParser())
    args = ap.parse_args(["--run-config", str(f), "--train-steps", "7", "--compress-bf16"])
    import os
    os.environ["TTD_RUN_WARMUP_STEPS"] = "2"
    try:
        rc = RunConfig.from_args(args)
    finally:
        del os.environ["TTD_RUN_WARMUP_STEPS"]
    assert (rc.model, rc.bucket_mb, rc.hipgraph, rc.train_steps, rc.warmup_steps, rc.compress_bf16) == \
        ("bert", 64.0, True, 7, 2, True)
    assert rc.extra == {"my_note": "x"} and rc.to_dict()["extra"] == {"my_note": "x"}
    with pytest.raises(ValueError):
        rc.replace(optimizer="adagrad")
    with pytest.raises(ValueError):
        RunConfig(bucket_mb=0)


def test_checkpoint_timer_agreement_is_not_per_step(tmp_path):
    """Under an all-reduce strategy the seconds-based checkpoint timer is agreed across replicas
    (a broadcast + host sync): only on every agree_every-th global step, never per step."""
    from types import SimpleNamespace
    from tensorflow_train_distributed_amd.train.hooks import CheckpointSaverHook

    calls = []
    saves = []

    class Sess:
        def agree(self, flag):
            calls.append(flag)
            return flag

        def save_checkpoint(self, saver, base, step):
            saves.append(step)
            return "%s-%d" % (base, step)

    h = CheckpointSaverHook(str(tmp_path), save_secs=0.0, saver=object())
    h.agree_every = 50
    h._timer.update_last_triggered_step(0)
    ctx = SimpleNamespace(session=Sess(), request_stop=lambda: None)
    for step in range(1, 201):
        h.after_run(ctx, SimpleNamespace(results=step))
    assert len(calls) == 4  # steps 50, 100, 150, 200
    assert saves == [50, 100, 150, 200]
