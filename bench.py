#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 v1.5 bf16 training throughput (images/sec, whole node),
MirroredStrategy-style data parallelism, one process per MI355X (BASELINE.json).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python bench.py --gpus 8 --steps 20 --warmup 5          # self-launches 8 ranks
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Each timed step is a full training step: forward, fused softmax-xent, backward, bucketed
RCCL all-reduce of all gradients (overlapped with backward), in-graph LR schedule and the
fused optimizer update (+ bf16 weight refresh). Weak scaling: per-GPU batch fixed.
Data: one synthetic batch resident on each GPU; weights random-init.

Launch: with --gpus N > 1 and no WORLD_SIZE in the environment, this process starts N rank
processes itself (torch.distributed.run on 127.0.0.1, before it touches any GPU), relays their
output and exits non-zero unless rank 0 reports an N-rank process group whose replicas stayed
bit-identical. Under an external launcher (WORLD_SIZE set) every rank runs the step directly.

--model bert runs BASELINE config 4 instead (BERT-Large seq 512 pre-training, MLM+NSP,
dropout on, LAMB; sequences/sec). --model mlp runs the reference's own workload (the
784-200-100-50-25-10 MNIST MLP of /root/reference/distribute_training.py:39-110, batch 128
per replica, GradientDescent + staircase exponential decay, :136-152); with --device cpu the
ranks talk over gloo (BASELINE config 1, the CPU plumbing run).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _reducer_engine():
    """TTD_REDUCER_ENGINE=ipc: the multi-rank rehearsal on fewer GPUs (ranks share a device over
    gloo, every gradient bucket on the direct IPC kernels, so the N > 1 step — collectives
    included — can be graph-captured and replayed as it would be over RCCL)."""
    return os.environ.get("TTD_REDUCER_ENGINE", "auto")


def build_resnet(args, dev, rank, world):
    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer, broadcast_flat_
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, FlatSGD, Schedule

    # per-GPU batch sized for 288 GB of HBM3E: 1024 images use ~67 GB and run ~4 % more images/s
    # than 512 (bigger GEMM grids, fixed per-step costs amortised, half the all-reduces per image)
    B = args.batch or 1024
    model = resnet50(device=dev, seed=1234, precision=args.precision)
    broadcast_flat_(model.params)
    if args.optimizer == "lamb":  # large-batch recipe (BASELINE config 5)
        opt = FlatLAMB(model.params, Schedule(kind=2, base_lr=0.01 * (B * world / 1024) ** 0.5, warmup_steps=5,
                                              end_lr=0.0, power=2.0, total_steps=10000), weight_decay=5e-5)
    else:
        opt = FlatSGD(model.params, Schedule(kind=2, base_lr=0.1 * B * world / 256, warmup_steps=5, end_lr=0.0,
                                             power=2.0, total_steps=10000), momentum=0.9, weight_decay=5e-5)
    # the backward window the collectives hide under is measured on a warm-up step (main) and
    # fed to the native engine's CTA-budget choice (BucketedAllReducer.retune)
    reducer = BucketedAllReducer(model.params, bucket_mb=args.bucket_mb, compress_bf16=args.compress_bf16,
                                 engine=_reducer_engine())
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    S = args.image_size
    images = torch.randn((B, S, S, 3), generator=g, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 1000, (B,), generator=g, device=dev, dtype=torch.int32)
    grad_scale = 1.0 / (B * world)

    def step():
        reducer.begin()
        sums = model.forward_backward(images, labels, grad_scale=grad_scale, grad_hook=reducer.mark_ready)
        reducer.finish()
        opt.step()
        return sums
    step.params = model.params
    step.reducer = reducer

    info = {
        # BASELINE.json's headline metric string, verbatim
        "metric": "images/sec (whole node) ResNet-50 %s MirroredStrategy at 1/2/4/8 MI355X" % args.precision,
        "unit": "images/sec",
        "data": "synthetic (random NHWC images + labels resident on GPU; random-init weights)",
        "config": {"model": "ResNet-50 v1.5", "global_batch": B * world, "per_gpu_batch": B, "image_size": S,
                   "seq_len": None, "parallelism": "dp%d" % world,
                   "optimizer": ("LAMB wd 5e-5" if args.optimizer == "lamb" else "momentum-SGD 0.9, wd 5e-5")
                   + ", fp32 master",
                   "precision": ("fp8: e4m3 forward of the 3x3 and 1x1 convs with >= 128 channels in and out, "
                                 "e5m2 x e4m3 unit-stride data gradients and e5m2 x e4m3 weight gradients "
                                 "(delayed scaling); stem, strided data gradients, BN and FC in bf16")
                   if args.precision == "fp8" else "bf16"},
    }
    return step, B, info


def build_bert(args, dev, rank, world):
    from tensorflow_train_distributed_amd.models.bert import BertConfig, BertPretraining, synthetic_batch
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer, broadcast_flat_
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, Schedule

    # 128 sequences of 512 tokens per GPU (~56 GB of HBM3E): 631 seq/s vs 553 at 32 — the LAMB
    # step, embedding/heads and launch costs are per step, and the GEMM grids grow 4x
    B = args.batch or 128
    S = args.seq_len
    cfg = BertConfig.large(max_position_embeddings=max(512, S))
    model = BertPretraining(cfg, device=dev, seed=1234)
    model.rng.t[0] = 1234 + 1000003 * rank  # distinct dropout masks per replica
    broadcast_flat_(model.params)
    opt = FlatLAMB(model.params, Schedule(kind=2, base_lr=4e-3, warmup_steps=100, end_lr=0.0, power=1.0,
                                          total_steps=10000), weight_decay=0.01, max_grad_norm=1.0)
    # (overlap window: measured on a warm-up step, see main)
    reducer = BucketedAllReducer(model.params, bucket_mb=args.bucket_mb, compress_bf16=args.compress_bf16,
                                 engine=_reducer_engine())
    batch = synthetic_batch(cfg, B, S, max_predictions=80 if S >= 512 else 20, device=dev, seed=rank)

    def step():
        reducer.begin()
        sums = model.forward_backward(batch, loss_scale=1.0 / world, grad_hook=reducer.mark_ready)
        reducer.finish()
        opt.step()
        return sums
    step.params = model.params
    step.reducer = reducer

    info = {
        "metric": "sequences/sec (whole node) BERT-Large seq%d bf16 MirroredStrategy" % S,
        "unit": "sequences/sec",
        "data": "synthetic (random token ids, 80 masked positions/seq, NSP labels; random-init weights)",
        "config": {"model": "BERT-Large (24x1024x16, MLM+NSP heads)", "global_batch": B * world,
                   "per_gpu_batch": B, "seq_len": S, "parallelism": "dp%d" % world,
                   "optimizer": "LAMB wd 0.01, clip 1.0, fp32 master", "dropout": "0.1 hidden / 0.1 attention"},
    }
    return step, B, info


def build_mlp(args, dev, rank, world):
    """The reference workload (distribute_training.py:39-152) as a MirroredStrategy job."""
    from tensorflow_train_distributed_amd.models.mlp import mnist_mlp
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer, broadcast_flat_
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule

    B = args.batch or 128  # BATCH_SIZE (:10), per replica
    model = mnist_mlp(device=dev, seed=1234 + rank)  # different init per rank: the broadcast must fix it
    broadcast_flat_(model.params)
    opt = FlatSGD(model.params, Schedule(kind=1, base_lr=0.01, decay_steps=468, decay_rate=0.96, staircase=True))
    reducer = BucketedAllReducer(model.params, bucket_mb=args.bucket_mb, first_bucket_mb=0.25,
                                 compress_bf16=args.compress_bf16)
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    feed = {"x-input": torch.rand((B, 784), generator=g, device=dev),
            "y-input": torch.randint(0, 10, (B,), generator=g, device=dev)}

    def step():
        reducer.begin()
        out = model.forward_backward(feed, grad_scale=1.0 / (B * world), grad_hook=reducer.mark_ready)
        reducer.finish()
        opt.step()
        return torch.stack([torch.as_tensor(out["loss"]).float().reshape(()),
                            torch.as_tensor(out["accuracy"]).float().reshape(())])
    step.params = model.params
    step.reducer = reducer
    info = {
        "metric": "examples/sec (whole job) MNIST MLP MirroredStrategy",
        "unit": "examples/sec",
        "data": "synthetic (uniform [0,1) 784-pixel images + labels; random-init weights)",
        "config": {"model": "MNIST MLP 784-200-100-50-25-10 (ELU, dropout 0.01)", "global_batch": B * world,
                   "per_gpu_batch": B, "seq_len": None, "parallelism": "dp%d" % world,
                   "optimizer": "GradientDescent, exponential_decay(0.01, 468, 0.96, staircase)"},
    }
    return step, B, info


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(args) -> int:
    """Start args.gpus rank processes (one per GPU) and relay their output. Runs before this
    process touches a GPU; returns the exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    result = None
    for line in proc.stdout:  # relay (the JSON line is printed by rank 0 only)
        sys.stdout.write(line)
        sys.stdout.flush()
        if line.startswith("{"):
            try:
                result = json.loads(line)
            except ValueError:
                pass
    rc = proc.wait()
    if rc != 0:
        return rc
    if result is None:
        print("bench: no result line from rank 0", file=sys.stderr)
        return 3
    d = result.get("dist") or {}
    if result.get("n_gpus") != args.gpus or d.get("world_size") != args.gpus:
        print("bench: asked for %d ranks, the process group had %s" % (args.gpus, d.get("world_size")),
              file=sys.stderr)
        return 4
    if d.get("replicas_in_sync") is False:
        print("bench: replicas diverged", file=sys.stderr)
        return 5
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert", "mlp"])
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="cpu: gloo ranks on the host (the CPU plumbing config; --model mlp)")
    ap.add_argument("--batch", type=int, default=0,
                    help="per-GPU batch (0 = model default: 1024 images / 128 sequences / 128 examples)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--graph", type=int, default=-1, help="hipGraph-capture the step (1/0, -1 = auto)")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--compress-bf16", action="store_true", help="all-reduce gradients in bf16")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8"], help="ResNet conv forward precision")
    ap.add_argument("--optimizer", default="momentum", choices=["momentum", "lamb"], help="ResNet optimizer")
    ap.add_argument("--run-config", default=None,
                    help="JSON/YAML RunConfig file (utils/run_config.py); its fields override the flags above")
    args = ap.parse_args()
    if args.run_config:
        from tensorflow_train_distributed_amd.utils.run_config import RunConfig
        rc = RunConfig.from_file(args.run_config).with_env()
        args.model, args.steps, args.warmup = rc.model, rc.train_steps, rc.warmup_steps
        args.batch, args.image_size, args.seq_len = rc.per_replica_batch, rc.image_size, rc.seq_len
        args.precision, args.bucket_mb, args.compress_bf16 = rc.precision, rc.bucket_mb, rc.compress_bf16
        args.graph = 1 if rc.hipgraph else 0
        if rc.optimizer in ("momentum", "lamb"):
            args.optimizer = rc.optimizer
        if rc.collective_engine != "auto":
            os.environ["TTD_COLLECTIVE"] = "native" if rc.collective_engine == "native" else "torch"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    on_cpu = args.device == "cpu" or (args.device == "auto" and not torch.cuda.is_available())
    if on_cpu and args.model != "mlp":
        print("bench: --device cpu runs --model mlp only", file=sys.stderr)
        sys.exit(2)
    # one process per GPU over RCCL ("nccl"); gloo on the CPU. TTD_DIST_BACKEND=gloo rehearses
    # several GPU ranks on fewer GPUs (ranks share devices round-robin)
    backend = "gloo" if on_cpu else os.environ.get("TTD_DIST_BACKEND", "nccl")
    if on_cpu:
        dev = torch.device("cpu")
    else:
        ndev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank % ndev)
        dev = torch.device("cuda", local_rank % ndev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    sync = (lambda: None) if on_cpu else torch.cuda.synchronize

    build = {"resnet50": build_resnet, "bert": build_bert, "mlp": build_mlp}[args.model]
    step, B, info = build(args, dev, rank, world)

    # hipGraph: the step is captured (segmented per stream, utils/graphs.py) and replayed — one
    # set of graph launches per step instead of ~600 kernel launches from Python. Same-box A/B
    # at ResNet-50 b1024: eager 68.30 / 68.26 ms, replay 68.43 / 68.27 ms (round 4): parity, so
    # auto = on (the host, 8.5 ms of issue per 68 ms step, is free for input / hooks work).
    # Auto = on at N = 1 only: replay of RCCL bucket launches captured on the communicator
    # stream has been exercised on one-rank communicators but never across real ranks (no
    # multi-GPU box is reachable from the build loop), so N > 1 stays eager until a two-rank
    # replay has been checked against eager; --graph 1 / TTD_BENCH_GRAPH=1 opt in.
    red_m = getattr(step, "reducer", None)
    window_ms = None
    if world > 1 and not on_cpu and getattr(red_m, "comm", None) is not None:
        # the overlap window the collectives hide under, MEASURED on one eager warm-up step (the
        # backward after the first bucket is ready, max over ranks), re-decides the engine's CTA
        # budget from its start-up probe table (rccl.retune) instead of a per-model constant
        red_m.measure_window()
        step()
        sync()
        w = red_m.window_ms()
        wt = torch.tensor([w if w is not None else -1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(wt, op=dist.ReduceOp.MAX)
        window_ms = float(wt.item())
        if window_ms > 0:
            red_m.retune(window_ms)
    auto_graph = 1 if world == 1 else int(os.environ.get("TTD_BENCH_GRAPH", "0"))
    use_graph = args.graph if args.graph >= 0 else auto_graph
    red0 = getattr(step, "reducer", None)
    if on_cpu or (world > 1 and getattr(red0, "comm", None) is None and getattr(red0, "ipc_stream", None) is None):
        # torch process-group collectives are issued eagerly; the native RCCL engine's bucket
        # launches (and the ipc rehearsal engine's kernels) are stream-ordered and capture into
        # the step's hipGraph
        use_graph = 0
    graph = None
    out = None
    # The step (its main chain; the weight gradients stay on the engine's normal-priority side
    # stream) on a high-priority HIP stream: the main chain's small BN/reduce kernels are
    # dispatched ahead of the side stream's GEMM workgroups as CUs free up. A/B on one box:
    # ResNet-50 b1024 82.1 -> 81.4 ms (3 pairs); BERT 190.9 -> 191.8 ms, so auto = ResNet only.
    main_prio = os.environ.get("TTD_MAIN_PRIO", "auto")
    main_prio = (args.model == "resnet50") if main_prio == "auto" else main_prio != "0"
    prio = None
    if main_prio and not on_cpu:
        prio = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
        prio.wait_stream(torch.cuda.current_stream())
    graph_info = None
    if use_graph:
        from tensorflow_train_distributed_amd.utils import graphs
        mode = os.environ.get("TTD_GRAPH_MODE", "segmented")
        if mode == "segmented":
            # per-stream linear graph segments replayed on the eager step's own streams (main
            # high priority, weight gradients normal priority, the native RCCL engine's
            # communicator stream); cross-stream edges — bucket forks and the final join
            # included — are event nodes (utils/graphs.py, parallel/collective.py)
            main_s = prio if prio is not None else torch.cuda.Stream(device=dev)
            err = None
            try:
                graph = graphs.capture_segmented(step, main=main_s, warmup=2)
            except Exception as e:  # noqa: BLE001 - every rank falls back together below
                graph, err = None, "%s: %s" % (type(e).__name__, e)
            if world > 1:
                # a replayed graph holds collectives: either every rank replays or none does (no
                # captured collective has run yet, so falling back here leaves the ranks in step)
                flag = torch.tensor([0 if graph is None else 1], dtype=torch.int32, device=dev)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                if int(flag.item()) == 0:
                    graph, err = None, err or "capture failed on another rank"
            if graph is None:
                print("bench: hipGraph capture failed (%s); running eagerly" % err, file=sys.stderr)
                use_graph = 0
                graph_info = {"mode": "segmented", "capture_failed": err}
                if world > 1 and getattr(red0, "comm", None) is not None:
                    # the native communicator's sequence may differ across ranks after a partial
                    # capture: the gradients go through the torch process group from here on
                    from tensorflow_train_distributed_amd.parallel import rccl
                    rccl.abort_all()
                    red0.comm = None
                    red0.engine = "torch-nccl"
                sync()
            else:
                out = graph.outputs
                graph_info = dict(graph.info, mode="segmented")
        else:
            for _ in range(2):
                step()
            sync()
            graph, out = graphs.capture(step, stream=prio)
            graph_info = {"mode": "single"}
    if graph is not None:
        run = graph.replay
        comm0 = getattr(red0, "comm", None)
        if comm0 is not None:
            # a captured join arms no watchdog marker: arm it after every replay, so a replayed
            # step whose collectives never finish still trips the no-progress deadline
            replay = run

            def run():
                out_ = replay()
                comm0.arm()
                return out_
    else:
        run = step
    if prio is not None:
        inner = run

        def run():
            with torch.cuda.stream(prio):
                return inner()

    for _ in range(args.warmup):
        run()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    per_rank = [elapsed]
    if world > 1:
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        per_rank = [float(p.item()) for p in parts]
    elapsed = max(per_rank)
    red = getattr(step, "reducer", None)
    comm_stats = None
    if red is not None and world > 1 and red.time_next_step():
        # one extra (untimed, eager) step with the collectives instrumented: busy time on the
        # communicator stream and the part of it the backward did not hide
        if graph is None:
            run()
        elif prio is not None:
            with torch.cuda.stream(prio):
                step()
        else:
            step()
        sync()
        comm_stats = red.comm_stats()
    sums = step() if graph is None else out
    loss = float(sums[0])
    # replicas must hold identical weights after synchronous data-parallel steps
    params = getattr(step, "params", None)
    replicas_in_sync = None
    if world > 1 and params is not None:
        # BN moving statistics are per replica (TF SyncOnRead): average them as a checkpoint
        # save would, then every variable must be bit-identical across ranks
        from tensorflow_train_distributed_amd.parallel.collective import sync_on_read_mean_
        sync_on_read_mean_(params)
        chk = params.master.double().sum().reshape(1)
        lo, hi = chk.clone(), chk.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        replicas_in_sync = bool(lo.item() == hi.item())
        if not replicas_in_sync:
            # which variables differ (diagnostic for the failure line; collective on every rank)
            names = params.names()
            w = torch.stack([params.var[n].double().sum() for n in names])
            wl, wh = w.clone(), w.clone()
            dist.all_reduce(wl, op=dist.ReduceOp.MIN)
            dist.all_reduce(wh, op=dist.ReduceOp.MAX)
            bad = [n for n, a_, b_ in zip(names, wl.tolist(), wh.tolist()) if a_ != b_]
            if rank == 0:
                print("bench: %d of %d variables differ across replicas, e.g. %s" % (len(bad), len(names), bad[:8]),
                      file=sys.stderr)
    # collective evidence for the scaling run: RCCL bus bandwidth of the gradient all-reduce at
    # the bucket sizes the reducer uses and at the whole gradient buffer (after the timed region,
    # on scratch copies: it does not touch the weights)
    probe = None
    red = getattr(step, "reducer", None)
    if world > 1 and red is not None and not on_cpu and backend == "nccl":
        probe = []
        nbytes_all = red.flat.numel * 4
        sizes = sorted({min(nbytes_all, 4 << 20), min(nbytes_all, int(args.bucket_mb * (1 << 20))), nbytes_all})
        for nb in sizes:
            if red.comm is not None:  # the native engine's own communicator and stream
                probe.append(red.comm.probe(nb, iters=5))
                continue
            buf = torch.zeros(nb // 4, dtype=torch.float32, device=dev)
            dist.all_reduce(buf)
            sync()
            reps = 5
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                dist.all_reduce(buf)
            e1.record()
            sync()
            t_ms = e0.elapsed_time(e1) / reps
            probe.append({"bytes": nb, "ms": round(t_ms, 4),
                          "busbw_GBps": round(2.0 * (world - 1) / world * nb / (t_ms * 1e-3) / 1e9, 1)})
            del buf
    ms = elapsed / args.steps * 1e3
    rate = B * world * args.steps / elapsed
    if rank == 0:
        cfg = dict(info["config"])
        cfg["hipgraph"] = bool(use_graph)
        if graph_info is not None:
            cfg["hipgraph_capture"] = graph_info
        if not on_cpu:
            cfg["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
        cfg["final_loss"] = loss
        red = getattr(step, "reducer", None)
        dinfo = {"world_size": dist.get_world_size() if world > 1 else 1, "backend": backend if world > 1 else None,
                 "per_rank_ms": [round(e / args.steps * 1e3, 3) for e in per_rank],
                 "replicas_in_sync": replicas_in_sync}
        if red is not None:
            dinfo["allreduce_bytes_per_step"] = red.bytes_per_step() if world > 1 else 0
            dinfo["buckets"] = len(red.buckets)
            dinfo["allreduce_dtype"] = "bf16" if red.compress else "fp32"
            dinfo["collective_engine"] = red.engine
            if world > 1:
                # per bucket: bytes and the path it took (direct xGMI one-/two-shot or RCCL)
                dinfo["bucket_bytes"] = [(e - s_) * (2 if red.compress else 4) for s_, e in red.buckets]
                dinfo["bucket_paths"] = red.bucket_paths
                if red.ipc is None and red.ipc_reason:
                    dinfo["ipc_allreduce_unavailable"] = red.ipc_reason
                dinfo["overlap_window_ms"] = round(window_ms, 3) if window_ms else None
            if world > 1 and red.comm is None and backend == "nccl":
                from tensorflow_train_distributed_amd.parallel import rccl
                dinfo["native_engine_unavailable"] = rccl.failure_reason() or os.environ.get("TTD_COLLECTIVE")
        if probe is not None:
            dinfo["allreduce_probe"] = probe
        pol = red.policy() if red is not None and world > 1 else None
        if pol is not None:
            dinfo["cta_budget"] = pol.get("cta_budget")
            dinfo["cta_policy"] = {k: pol.get(k) for k in ("reason", "overlap_ms", "projected_ms", "first_bucket_mb",
                                                         "probe")}
        if comm_stats is not None:
            dinfo["comm_per_step"] = comm_stats
        if backend == "nccl" and world > 1:
            try:
                dinfo["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
            except Exception:  # noqa: BLE001
                pass
        print(json.dumps({
            "metric": info["metric"],
            "value": round(rate, 2),
            "unit": info["unit"],
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp32" if args.model == "mlp" else  # the reference MLP runs fp32 everywhere
                      "fp8+bf16" if args.precision == "fp8" else "bf16"),
            "data": info["data"],
            "config": cfg,
            "dist": dinfo,
        }), flush=True)
    if world > 1:
        if not on_cpu:
            from tensorflow_train_distributed_amd.parallel import rccl
            rccl.shutdown()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
