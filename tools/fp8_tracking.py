#!/usr/bin/env python3
"""Loss tracking of the fp8 ResNet-50 path against bf16 (BASELINE config 5 quality check).

Trains ResNet-50 v1.5 at the bench's shape (b1024, 224^2, LAMB large-batch recipe as bench.py
--optimizer lamb) for --steps steps in bf16 and in --precision fp8 from the same initial weights,
cycling over --batches distinct synthetic batches (default 8: the model has to fit 8192 images,
not memorise one batch), and reports both loss curves and the relative gap of the mean loss over
the second half of the run (the acceptance line: within 10 %; windowed means reported).

    python tools/fp8_tracking.py --steps 200 --out gpurun_out/fp8_tracking.json
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(precision, steps, B, S, log_every, nbatches=8):
    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, Schedule
    dev = torch.device("cuda", 0)
    model = resnet50(device=dev, seed=1234, precision=precision)
    opt = FlatLAMB(model.params, Schedule(kind=2, base_lr=0.01 * (B / 1024) ** 0.5, warmup_steps=5, end_lr=0.0,
                                          power=2.0, total_steps=10000), weight_decay=5e-5)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    data = []
    for _ in range(nbatches):
        data.append((torch.randn((B, S, S, 3), generator=g, device=dev).to(torch.bfloat16),
                     torch.randint(0, 1000, (B,), generator=g, device=dev, dtype=torch.int32)))
    losses = []
    t0 = time.time()
    for i in range(steps):
        images, labels = data[i % nbatches]
        sums = model.forward_backward(images, labels, grad_scale=1.0 / B)
        opt.step()
        losses.append(sums[0:1].clone())
        if log_every and (i + 1) % log_every == 0:
            print("%s step %d loss %.4f (%.1f s)" % (precision, i + 1, float(losses[-1]), time.time() - t0), flush=True)
    torch.cuda.synchronize()
    return [round(float(x), 5) for x in torch.cat(losses).cpu()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/fp8_tracking.json")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    res = {"steps": a.steps, "batch": a.batch, "distinct_batches": a.batches,
           "optimizer": "LAMB (bench.py --optimizer lamb)"}
    for p in ("bf16", "fp8"):
        res[p] = run(p, a.steps, a.batch, a.image_size, log_every=25, nbatches=a.batches)
        torch.cuda.empty_cache()
    k = min(10, a.steps)
    mb = sum(res["bf16"][-k:]) / k
    m8 = sum(res["fp8"][-k:]) / k
    res["mean_last10"] = {"bf16": round(mb, 5), "fp8": round(m8, 5)}
    # per-step losses differ batch to batch, so a 10-step mean is noise-dominated: the acceptance
    # line compares the mean over the second half of the run (within 10 %) and the windowed means
    # are reported
    h = a.steps // 2
    hb = sum(res["bf16"][h:]) / (a.steps - h)
    h8 = sum(res["fp8"][h:]) / (a.steps - h)
    res["mean_second_half"] = {"bf16": round(hb, 5), "fp8": round(h8, 5)}
    res["windows"] = {"%d-%d" % (w0, w1): {"bf16": round(sum(res["bf16"][w0:w1]) / (w1 - w0), 5),
                                          "fp8": round(sum(res["fp8"][w0:w1]) / (w1 - w0), 5)}
                      for w0, w1 in ((0, a.steps // 4), (a.steps // 4, h), (h, a.steps)) if w1 > w0}
    res["rel_gap"] = round((h8 - hb) / hb, 4)
    res["within_10pct"] = abs(h8 - hb) <= 0.10 * abs(hb)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f)
    print(json.dumps({k2: res[k2] for k2 in ("mean_last10", "mean_second_half", "windows", "rel_gap", "within_10pct")}),
          flush=True)


if __name__ == "__main__":
    main()
