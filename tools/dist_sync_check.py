#!/usr/bin/env python3
"""Data-parallel consistency check (run under torch.distributed.run, any backend): after each
phase of a training step, compare a checksum of the flat buffers across ranks.
usage: TTD_DIST_BACKEND=gloo torchrun --nproc-per-node 2 tools/dist_sync_check.py [resnet|bert]"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def same(t, what):
    c = t.double().sum().reshape(1)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if dist.get_rank() == 0:
        print("%-28s %s  (%.10g vs %.10g)" % (what, "OK" if lo.item() == hi.item() else "DIFFERS", lo.item(), hi.item()),
              flush=True)


def main():
    rank, world, lr = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
    dev = torch.device("cuda", lr % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    backend = os.environ.get("TTD_DIST_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer, broadcast_flat_
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, FlatSGD, Schedule
    which = sys.argv[1] if len(sys.argv) > 1 else "resnet"
    if which == "bert":
        from tensorflow_train_distributed_amd.models.bert import BertConfig, BertPretraining, synthetic_batch
        cfg = BertConfig.large(num_hidden_layers=2, max_position_embeddings=512)
        m = BertPretraining(cfg, device=dev, seed=rank + 5)
        m.rng.t[0] = 77 + rank
        opt = FlatLAMB(m.params, Schedule(kind=0, base_lr=1e-3), weight_decay=0.01, max_grad_norm=1.0)
        batch = synthetic_batch(cfg, 2, 128, max_predictions=20, device=dev, seed=rank)

        def fb(hook):
            return m.forward_backward(batch, loss_scale=1.0 / world, grad_hook=hook)
    else:
        from tensorflow_train_distributed_amd.models.resnet import ResNet
        m = ResNet(((64, 1, 1), (128, 1, 2)), device=dev, seed=rank + 5)  # different init per rank on purpose
        opt = FlatSGD(m.params, Schedule(kind=0, base_lr=0.05), momentum=0.9)
        g = torch.Generator(device=dev).manual_seed(rank)
        x = torch.randn((8, 64, 64, 3), generator=g, device=dev).bfloat16()
        y = torch.randint(0, 1000, (8,), generator=g, device=dev, dtype=torch.int32)

        def fb(hook):
            return m.forward_backward(x, y, grad_scale=1.0 / (8 * world), grad_hook=hook)
    broadcast_flat_(m.params)
    torch.cuda.synchronize()
    same(m.params.master, "master after broadcast")
    red = BucketedAllReducer(m.params, bucket_mb=0.5, first_bucket_mb=0.1)
    for it in range(2):
        red.begin()
        fb(red.mark_ready)
        red.finish()
        torch.cuda.synchronize()
        same(m.params.grad * m.params.valid_mask(), "grads (trainable) step %d" % it)
        opt.step()
        torch.cuda.synchronize()
        trainable = m.params.master * m.params.valid_mask()
        same(trainable, "trainable weights step %d" % it)
        from tensorflow_train_distributed_amd.parallel.collective import sync_on_read_mean_
        sync_on_read_mean_(m.params)
        same(m.params.master, "all after SyncOnRead mean %d" % it)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
