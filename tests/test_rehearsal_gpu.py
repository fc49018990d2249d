"""Rehearsal of the N > 1 data-parallel step on ONE GPU (two processes sharing the device; RCCL
refuses that, so the gradient buckets all go through the direct IPC all-reduce kernels —
BucketedAllReducer(engine="ipc") — with gloo as the control plane).

What the driver's multi-GPU run does over RCCL, checked here end to end with real ranks:
* eager two-rank step: after the bucketed all-reduce every rank holds bit-identical gradients
  (replicas in sync), equal to the mean of the per-shard gradients computed in one process
  (BatchNorm statistics are per replica, as in tf.distribute.MirroredStrategy, so the reference is
  the per-replica average, not a big-batch BN);
* the same step captured as per-stream hipGraph segments (utils/graphs.capture_segmented: main,
  weight-gradient and communicator streams, event nodes at every fork / join) and replayed:
  replay == eager, bit for bit;
* a whole training loop (step + fused SGD) replayed: the replicas' weights stay identical.
Reference: the synchronous data-parallel hot loop, /root/reference/distribute_training.py:223-226
(SyncReplicasOptimizer aggregation at :142-148)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

STAGES = ((64, 1, 1), (128, 1, 2))


def _model(dev):
    from tensorflow_train_distributed_amd.models.resnet import ResNet
    return ResNet(STAGES, num_classes=10, device=dev, seed=3)


def _shard(rank, B=8):
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    x = torch.randn((B, 32, 32, 3), generator=g).bfloat16()
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    return x, y


def _worker(rank, world, port, q):
    try:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
        from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
        from tensorflow_train_distributed_amd.utils import graphs
        m = _model(dev)
        # small buckets: one-shot (<= 1 MB) and two-shot buckets in every step
        red = BucketedAllReducer(m.params, bucket_mb=1.25, first_bucket_mb=0.25, engine="ipc")
        x, y = _shard(rank)
        x, y = x.to(dev), y.to(dev)
        B = x.shape[0]

        def step():
            red.begin()
            s = m.forward_backward(x, y, grad_scale=1.0 / (B * world), grad_hook=red.mark_ready)
            red.finish()
            return s

        res = {"engine": red.engine, "paths": sorted(set(red.bucket_paths)), "buckets": len(red.buckets)}
        main = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
        with torch.cuda.stream(main):
            step()
        torch.cuda.synchronize()
        g_eager = m.params.grad.clone()
        parts = [torch.zeros_like(g_eager.cpu()) for _ in range(world)]
        dist.all_gather(parts, g_eager.cpu())
        res["replicas_equal"] = all(torch.equal(parts[0], p) for p in parts[1:])
        dist.barrier()
        seg = graphs.capture_segmented(step, main=main, warmup=1)
        res["graph_streams"] = seg.info.get("streams")
        seg.replay()
        torch.cuda.synchronize()
        res["replay_bitwise"] = bool(torch.equal(m.params.grad, g_eager))
        res["replay_maxdiff"] = float((m.params.grad - g_eager).abs().max())
        red.check()
        if rank == 0:
            torch.save(g_eager.cpu(), os.environ["TTD_REHEARSAL_OUT"])
        # a replayed training loop: step + SGD; replicas must stay bit-identical
        opt = FlatSGD(m.params, Schedule(kind=0, base_lr=0.05), momentum=0.9)

        def train():
            s = step()
            opt.step()
            return s

        from tensorflow_train_distributed_amd.parallel.collective import sync_on_read_mean_

        def diverged():
            # BN moving statistics are per replica (TF SyncOnRead): averaged as a checkpoint save
            # would; then every variable must be bit-identical across the ranks
            sync_on_read_mean_(m.params)
            P = m.params
            names = [n for n in P.names()]
            w = torch.stack([P.var[n].double().sum() for n in names]).cpu()
            ws = [torch.zeros_like(w) for _ in range(world)]
            dist.all_gather(ws, w)
            return [n for i, n in enumerate(names) if any(v[i] != ws[0][i] for v in ws[1:])]

        # eager training steps first (collectives on the direct kernels, no graph)
        with torch.cuda.stream(main):
            for _ in range(2):
                train()
        torch.cuda.synchronize()
        red.check()
        res["eager_diverged"] = diverged()
        seg2 = graphs.capture_segmented(train, main=main, warmup=1)
        for _ in range(3):
            seg2.replay()
        torch.cuda.synchronize()
        red.check()
        res["replay_diverged"] = diverged()
        res["weights_in_sync"] = not res["eager_diverged"] and not res["replay_diverged"]
        red.ipc.destroy()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001 - reported to the test
        import traceback
        q.put((rank, "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc())))


def test_two_rank_step_on_one_gpu_eager_replay_and_shard_mean(tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out_path = str(tmp_path / "g_eager.pt")
    os.environ["TTD_REHEARSAL_OUT"] = out_path
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            rank, res = q.get(timeout=110)
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(2):
        res = out[rank]
        assert isinstance(res, dict), res
        assert res["engine"] == "ipc-rehearsal"
        assert res["buckets"] >= 2 and {"ipc_oneshot", "ipc_twoshot"} <= set(res["paths"]), res
        assert res["replicas_equal"], res
        assert res["replay_bitwise"], res
        assert res["weights_in_sync"], res
        assert res["graph_streams"] >= 3, res  # main, weight-gradient, communicator
    # the two-rank gradient == mean of the per-shard gradients computed in this process
    g_dp = torch.load(out_path, weights_only=True).cuda()
    dev = torch.device("cuda", 0)
    m = _model(dev)
    acc = torch.zeros_like(m.params.grad)
    for r in range(2):
        x, y = _shard(r)
        m.forward_backward(x.to(dev), y.to(dev), grad_scale=1.0 / (x.shape[0] * 2))
        acc += m.params.grad
    torch.cuda.synchronize()
    rel = float((g_dp - acc).norm() / acc.norm())
    assert rel < 1e-5, rel


def test_segmented_capture_launches_fork_sources_first():
    """A stream that began its segment early (forked from main) and later waits on a fork from a
    stream that began after it must be launched after that stream's segment: the record node
    precedes the wait at replay (the ordering bug the two-rank rehearsal exposed: the
    communicator stream, forked from main for the first bucket, waited on the weight-gradient
    stream for the next one and read its gradients before they were written)."""
    from tensorflow_train_distributed_amd.utils import graphs
    dev = torch.device("cuda", 0)
    main = torch.cuda.Stream(device=dev)
    a = torch.cuda.Stream(device=dev)  # "communicator": forked from main first
    b = torch.cuda.Stream(device=dev)  # "weight gradients": forked from main later
    x = torch.zeros(1 << 20, device=dev)
    y = torch.zeros(1 << 20, device=dev)
    w = torch.zeros(1 << 20, device=dev)
    z = torch.zeros(1 << 20, device=dev)

    def step():
        x.add_(1.0)
        graphs.fork(torch.cuda.current_stream(), a)
        with torch.cuda.stream(a):
            y.copy_(x)
        graphs.fork(torch.cuda.current_stream(), b)
        with torch.cuda.stream(b):
            w.copy_(x)
            for _ in range(20):  # a slow producer: a race would show as a stale z
                w.mul_(1.0)
            w.add_(1.0)
            graphs.fork(b, a)
        with torch.cuda.stream(a):
            z.copy_(w)
        graphs.join(torch.cuda.current_stream(), a)
        graphs.join(torch.cuda.current_stream(), b)

    seg = graphs.capture_segmented(step, main=main, warmup=1)
    order = [s.cuda_stream for s, _ in seg.cap.segments]
    assert order.index(b.cuda_stream) < order.index(a.cuda_stream), order
    for _ in range(5):
        seg.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 6.0 and float(y[0]) == 6.0 and float(z[0]) == 7.0 and float(w[0]) == 7.0
