"""Coordinated checkpointing and recovery for the all-reduce strategies (2 replicas, gloo):

* MonitoredTrainingSession under MirroredStrategy with a seconds-based checkpoint timer:
  replica 0's clock decides when to save (broadcast), every replica averages its SyncOnRead
  variables, replica 0 alone writes; killed and relaunched, both replicas resume at the saved
  global step with identical weights (reference behaviour: chief-only checkpointing and
  restore on session creation, /root/reference/distribute_training.py:204-215);
* a replica whose communicator fails mid-training (its process group torn down, the peer's
  all-reduce errors) is recovered in-process: the session rebuilds the process group (next
  generation), replica 0 restores the latest checkpoint and broadcasts it.
"""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, json, time
import torch
import torch.distributed as dist
import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.train.hooks import CheckpointSaverHook
from tensorflow_train_distributed_amd.parallel.fault import FaultInjectionHook
from tensorflow_train_distributed_amd.utils import errors
torch.set_num_threads(1)
ckdir, out, last_step, mode = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
strategy = ttd.distribute.MirroredStrategy()
rank = strategy.replica_id
with strategy.scope():
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(seed=7 + rank, dropout_rate=0.0)
    op = ttd.train.MomentumOptimizer(0.05, 0.9).minimize(model, global_step=gs)
g = torch.Generator().manual_seed(rank)
hooks = [ttd.train.StopAtStepHook(last_step=last_step)]
kw = dict(save_checkpoint_secs=0.3)
if mode == "fault":
    kw = dict(save_checkpoint_steps=10)
    if rank == 1:
        def lose_communicator():
            dist.destroy_process_group()
        hooks.append(FaultInjectionHook(at_step=25, error=errors.UnavailableError, action=lose_communicator))
steps = []
with ttd.train.MonitoredTrainingSession(is_chief=(rank == 0), checkpoint_dir=ckdir, hooks=hooks,
                                        save_summaries_steps=None, log_step_count_steps=None, **kw) as sess:
    while not sess.should_stop():
        x = torch.rand((16, 784), generator=g)
        y = torch.randint(0, 10, (16,), generator=g)
        _, s = sess.run([op, gs], feed_dict={"x-input": x, "y-input": y})
        steps.append(int(s))
        print("step", s, flush=True)
        time.sleep(0.02)
    saved = [p for h in sess._hooks if isinstance(h, CheckpointSaverHook) for p in h.saved_paths]
    recoveries = sess.recoveries
w = model.params.master.clone()
ws = strategy.gather(w[None], axis=0)
m = op.flat.mom.clone()
ms = strategy.gather(m[None], axis=0)
json.dump({"rank": rank, "steps": steps, "saved": saved, "recoveries": recoveries,
           "wdiff": float((ws - ws[0]).abs().max()), "mdiff": float((ms - ms[0]).abs().max())},
          open(out + "/r%d.json" % rank, "w"))
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(tmp_path, ckdir, last_step, mode):
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": "2", "LOCAL_RANK": str(r), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "CUDA_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "1",
                    "PYTHONPATH": REPO + os.pathsep + env.get("PYTHONPATH", "")})
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        procs.append(subprocess.Popen([sys.executable, str(tmp_path / "run.py"), ckdir, str(tmp_path), str(last_step),
                                       mode], env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    return procs


def _results(tmp_path):
    return [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(2)]


@pytest.mark.slow
def test_mirrored_checkpoint_kill_and_resume(tmp_path):
    from tensorflow_train_distributed_amd.train import checkpoint as C
    (tmp_path / "run.py").write_text(SCRIPT)
    ckdir = str(tmp_path / "ck")
    procs = _launch(tmp_path, ckdir, 100000, "secs")
    try:
        deadline = time.time() + 120
        saved = None
        while time.time() < deadline:
            lc = C.latest_checkpoint(ckdir)
            if lc and int(lc.rsplit("-", 1)[1]) >= 15:
                saved = lc
                break
            assert all(p.poll() is None for p in procs), procs[0].stdout.read()[-2000:]
            time.sleep(0.05)
        assert saved is not None
    finally:
        for p in procs:
            p.send_signal(signal.SIGKILL)
            p.wait()
    S = int(C.latest_checkpoint(ckdir).rsplit("-", 1)[1])
    procs = _launch(tmp_path, ckdir, S + 10, "secs")
    for p in procs:
        out, _ = p.communicate(timeout=180)
        assert p.returncode == 0, out[-3000:]
    r0, r1 = _results(tmp_path)
    # resumed at the saved step on both replicas, in lockstep, with identical state
    assert r0["steps"][0] == S + 1 and r1["steps"] == r0["steps"] and r0["steps"][-1] == S + 10
    assert r0["wdiff"] == 0.0 and r0["mdiff"] == 0.0
    # one writer: replica 1 never wrote a checkpoint
    assert r0["saved"] and not r1["saved"]
    assert int(C.load_variable(C.latest_checkpoint(ckdir), "global_step")) == S + 10


@pytest.mark.slow
def test_mirrored_collective_failure_recovers_from_checkpoint(tmp_path):
    (tmp_path / "run.py").write_text(SCRIPT)
    ckdir = str(tmp_path / "ck")
    procs = _launch(tmp_path, ckdir, 40, "fault")
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out[-3000:]
    r0, r1 = _results(tmp_path)
    assert r0["recoveries"] >= 1 and r1["recoveries"] >= 1
    assert r0["steps"][-1] == 40 and r1["steps"][-1] == 40
    # after the failure at step 25 both replicas went back to the step-20 checkpoint
    i = next(i for i in range(1, len(r1["steps"])) if r1["steps"][i] <= r1["steps"][i - 1])
    assert r1["steps"][i] == 21
    assert r0["wdiff"] == 0.0 and r0["mdiff"] == 0.0
