"""The reference workload itself on the MI355X (SURVEY.md §7.3 "minimum slice B"): the
784-200-100-50-25-10 ELU/dropout MLP of /root/reference/distribute_training.py:39-110 run by
the HIP kernels (MFMA GEMMs, fused bias+ELU+dropout, fused xent+in_top_k, flat SGD):

* GPU step == fp32 CPU reference step (dropout off so both see the same function);
* the reference training loop (global step, staircase exponential decay, GradientDescent,
  MonitoredTrainingSession with StopAtStepHook + checkpoints) trains on the GPU engine;
* the whole step (forward, backward, optimizer) replays from one hipGraph bit-identically;
* the bucketed gradient all-reduce runs through RCCL (single-rank communicator).
"""
import os

import numpy as np
import pytest
import torch

import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd.data import mnist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("mnist_gpu"))
    mnist.write_synthetic(d, n_train=8000, n_test=200)
    return d


def _batch(seed, B=128):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((B, 784), generator=g)
    y = torch.randint(0, 10, (B,), generator=g)
    return x, y


def test_reference_mlp_gpu_step_matches_cpu():
    """fp32 engine (the reference's dtype): exact-fp32 MFMA GEMMs -> every gradient within 1e-4
    relative of the CPU fp32 autograd step."""
    cpu = ttd.models.mnist_mlp(device="cpu", seed=5, dropout_rate=0.0)
    gpu = ttd.models.mnist_mlp(device="cuda", seed=5, dropout_rate=0.0)
    torch.testing.assert_close(gpu.params.master.cpu(), cpu.params.master)
    x, y = _batch(0)
    rc = cpu.forward_backward({"x-input": x, "y-input": y})
    rg = gpu.forward_backward({"x-input": x, "y-input": y})
    torch.cuda.synchronize()
    assert abs(float(rg["loss"]) - float(rc["loss"])) < 1e-5 * max(1.0, float(rc["loss"]))
    assert float(rg["accuracy"]) == float(rc["accuracy"])
    for n in cpu.params.names():
        a, b = gpu.params.g[n].float().cpu(), cpu.params.g[n]
        rel = float((a - b).norm() / (b.norm() + 1e-12))
        assert rel < 1e-4, (n, rel)


def test_reference_mlp_bf16_engine_step_close_to_cpu():
    cpu = ttd.models.mnist_mlp(device="cpu", seed=5, dropout_rate=0.0)
    gpu = ttd.models.mnist_mlp(device="cuda", seed=5, dropout_rate=0.0, dtype="bfloat16")
    x, y = _batch(0)
    rc = cpu.forward_backward({"x-input": x, "y-input": y})
    rg = gpu.forward_backward({"x-input": x, "y-input": y})
    torch.cuda.synchronize()
    assert abs(float(rg["loss"]) - float(rc["loss"])) < 2e-2 * max(1.0, float(rc["loss"]))
    for n in cpu.params.names():
        a, b = gpu.params.g[n].float().cpu(), cpu.params.g[n]
        rel = float((a - b).norm() / (b.norm() + 1e-12))
        assert rel < 3e-2, (n, rel)


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_f32_matches_fp32_reference(ta, tb):
    from tensorflow_train_distributed_amd.ops import gemm as G
    g = torch.Generator().manual_seed(3)
    M, N, K = 133, 77, 201
    a = torch.randn((K, M) if ta else (M, K), generator=g)
    b = torch.randn((N, K) if tb else (K, N), generator=g)
    bias = torch.randn(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    ref = (a.t() if ta else a).double() @ (b.t() if tb else b).double() + bias.double() + c0.double()
    out = c0.cuda()
    G.gemm_f32(a.cuda(), b.cuda(), trans_a=ta, trans_b=tb, bias=bias.cuda(), out=out, beta=1)
    torch.cuda.synchronize()
    err = float((out.cpu().double() - ref).abs().max() / ref.abs().max())
    assert err < 2e-6, err


def test_reference_training_loop_on_gpu(tmp_path, mnist_dir):
    data = mnist.read_data_sets(mnist_dir, seed=0)
    ttd.train.reset_default_graph()
    gs = ttd.train.get_or_create_global_step()
    model = ttd.models.mnist_mlp(device="cuda", seed=0)
    lr = ttd.train.exponential_decay(0.05, gs, 468, 0.96, staircase=True)
    op = ttd.train.GradientDescentOptimizer(lr).minimize(model, global_step=gs)
    x = ttd.placeholder(torch.float32, [None, 784], "x-input")
    y = ttd.placeholder(torch.int64, [None], "y-input")
    losses = []
    ck = str(tmp_path / "ck")
    with ttd.train.MonitoredTrainingSession(checkpoint_dir=ck, hooks=[ttd.train.StopAtStepHook(last_step=150)],
                                            save_checkpoint_steps=100, save_summaries_steps=50) as sess:
        while not sess.should_stop():
            bx, by = data.train.next_batch(128)
            _, l, g = sess.run([op, op.loss, gs], feed_dict={x: bx, y: by})
            losses.append(l)
    assert g == 150 and len(losses) == 150
    assert np.mean(losses[-20:]) < np.mean(losses[:20]) - 0.3, (losses[:5], losses[-5:])
    keys = dict(ttd.train.list_variables(ttd.train.latest_checkpoint(ck)))
    assert keys["hidden1/kernel"] == (784, 200) and keys["output/bias"] == (10,)
    ttd.train.reset_default_graph()


def test_reference_mlp_step_hipgraph_replay_is_bit_identical():
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    from tensorflow_train_distributed_amd.utils.graphs import capture

    def make():
        m = ttd.models.mnist_mlp(device="cuda", seed=9, dropout_rate=0.0)
        return m, FlatSGD(m.params, Schedule(kind=0, base_lr=0.05))

    x, y = _batch(1)
    xd, yd = x.cuda(), y.cuda()
    eager, opt_e = make()
    for _ in range(4):
        eager.forward_backward({"x-input": xd, "y-input": yd})
        opt_e.step()
    graphed, opt_g = make()

    def step():
        out = graphed.forward_backward({"x-input": xd, "y-input": yd})
        opt_g.step()
        return out

    cs, _ = capture(step, warmup=1)  # warmup = eager step 1, capture records (does not run) one step
    for _ in range(3):
        cs.replay()
    torch.cuda.synchronize()
    assert torch.equal(graphed.params.master, eager.params.master)


def test_bucketed_allreduce_through_rccl_single_rank(tmp_path):
    """The RCCL launch path of the reducer on a real (1-rank) communicator: buckets are issued
    during backward in order and reduce in place (SUM over one rank leaves the gradient as the
    backward wrote it). Multi-rank averaging is tested in test_collective_multirank.py (gloo)
    and test_two_gpu_ranks_over_gloo_stay_in_sync below."""
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        m = ttd.models.mnist_mlp(device="cuda", seed=4, dropout_rate=0.0)
        x, y = _batch(2)
        feed = {"x-input": x.cuda(), "y-input": y.cuda()}
        m.forward_backward(feed)
        want = m.params.grad.clone()  # the gradient before any collective touched it
        m.params.grad.zero_()
        red = BucketedAllReducer(m.params, bucket_mb=0.25, first_bucket_mb=0.05)
        red.world = 2  # force the collective path on the single-rank communicator
        assert len(red.buckets) >= 3
        red.begin()
        m.forward_backward(feed, grad_hook=red.mark_ready)
        early = list(red.launch_log)
        red.finish()
        torch.cuda.synchronize()
        assert early and early == list(range(len(early)))  # buckets launched during backward, in order
        assert red.launch_log == list(range(len(red.buckets)))
        assert float(want.abs().sum()) > 0
        assert torch.equal(m.params.grad, want)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["mlp", "resnet50"])
def test_two_gpu_ranks_over_gloo_stay_in_sync(model):
    """bench.py --gpus 2 launches its own two ranks; here both share cuda:0 and talk over gloo
    (RCCL needs one GPU per rank): the data-parallel step with bucketed all-reduce keeps the
    replicas bit-identical and reports a 2-rank process group."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["TTD_DIST_BACKEND"] = "gloo"
    extra = ["--batch", "16", "--image-size", "64"] if model == "resnet50" else []
    p = subprocess.run([sys.executable, "bench.py", "--model", model, "--gpus", "2", "--steps", "2", "--warmup", "1"]
                       + extra, cwd=repo, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["dist"]["world_size"] == 2 and r["dist"]["replicas_in_sync"] is True


def test_restore_refreshes_bf16_compute_copy(tmp_path):
    """A restored model computes with the restored weights: the GPU engine runs on the bf16
    compute copy, which Saver/Checkpoint restores refresh from the restored fp32 masters."""
    x, y = _batch(3)
    feed = {"x-input": x.cuda(), "y-input": y.cuda()}
    a = ttd.models.mnist_mlp(device="cuda", seed=1, dropout_rate=0.0, dtype="bfloat16")
    opt = ttd.train.GradientDescentOptimizer(0.1).build(a.params)
    for _ in range(2):
        a.forward_backward(feed)
        opt.step()
    want = float(a.forward_backward(feed)["loss"])
    p1 = ttd.train.Saver(a.params).save(None, str(tmp_path / "s" / "model.ckpt"), global_step=2)
    p2 = ttd.train.Checkpoint(model=a.params).save(str(tmp_path / "c" / "ckpt"))
    for restore in (lambda m: ttd.train.Saver(m.params).restore(None, p1),
                    lambda m: ttd.train.Checkpoint(model=m.params).restore(p2)):
        b = ttd.models.mnist_mlp(device="cuda", seed=2, dropout_rate=0.0, dtype="bfloat16")
        restore(b)
        assert torch.equal(b.params.compute, a.params.compute)
        assert float(b.forward_backward(feed)["loss"]) == want
