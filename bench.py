#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 v1.5 bf16 training throughput (images/sec, whole node),
MirroredStrategy-style data parallelism, one process per MI355X (BASELINE.json).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Each timed step is a full training step: forward, fused softmax-xent, backward, bucketed
RCCL all-reduce of all gradients (overlapped with backward), in-graph LR schedule and the
fused momentum-SGD update (+ bf16 weight refresh). Weak scaling: per-GPU batch fixed.
Data: one synthetic ImageNet-shaped batch resident on each GPU (random NHWC bf16 images,
random labels); weights random-init.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--graph", type=int, default=-1, help="hipGraph-capture the step (1/0, -1 = auto)")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world), file=sys.stderr)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer, broadcast_flat_
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule

    model = resnet50(device=dev, seed=1234)
    broadcast_flat_(model.params)
    B = args.batch
    opt = FlatSGD(model.params, Schedule(kind=2, base_lr=0.1 * B * world / 256, warmup_steps=5, end_lr=0.0,
                                         power=2.0, total_steps=10000), momentum=0.9, weight_decay=5e-5)
    reducer = BucketedAllReducer(model.params, bucket_mb=args.bucket_mb)
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

    use_graph = args.graph if args.graph >= 0 else 0
    graph = None
    if use_graph:
        from tensorflow_train_distributed_amd.utils.graphs import capture
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        graph, out = capture(step)
        run = graph.replay
    else:
        run = step

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    sums = step() if graph is None else out
    loss = float(sums[0])
    ms = elapsed / args.steps * 1e3
    ips = B * world * args.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet-50 bf16 MirroredStrategy",
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random NHWC images + labels resident on GPU; random-init weights)",
            "config": {"model": "ResNet-50 v1.5", "global_batch": B * world, "per_gpu_batch": B,
                       "image_size": S, "seq_len": None, "parallelism": "dp%d" % world,
                       "optimizer": "momentum-SGD 0.9, wd 5e-5, fp32 master", "hipgraph": bool(use_graph),
                       "final_loss": loss},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
