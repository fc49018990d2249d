#!/usr/bin/env python3
"""Fused (streaming pointwise kernel) vs unfused ResNet engine: one forward+backward each with
the same weights/data, per-variable gradient differences, per fusion switch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_train_distributed_amd.models.resnet import ResNet  # noqa: E402


def run(parts, fuse=True, seed=5):
    torch.manual_seed(0)
    stages = ((64, 3, 1), (128, 2, 2), (256, 1, 2), (512, 1, 2))
    x = torch.randn(8, 96, 96, 3, device="cuda").bfloat16()
    y = torch.randint(0, 100, (8,), device="cuda")
    m = ResNet(stages, num_classes=100, device="cuda", seed=seed)
    m.fuse_pw = fuse
    m.pw_parts = dict(parts)
    s = m.forward_backward(x, y)
    torch.cuda.synchronize()
    return float(s[0]), m.params.grad.clone(), m


def reference(m, seed=5):
    torch.manual_seed(0)
    x = torch.randn(8, 96, 96, 3, device="cuda").bfloat16()
    y = torch.randint(0, 100, (8,), device="cuda")
    leaves = {n: m.params.c[n].float().detach().clone().requires_grad_(m.params.spec(n).trainable)
              for n in m.params.names()}
    loss, _, _ = m.reference_loss(x.float(), y, leaves, bf16_activations=True)
    loss.backward()
    names = [n for n in m.params.names() if m.params.spec(n).trainable]
    return float(loss), names, {n: leaves[n].grad.flatten() for n in names}


def cos_vs_ref(g, m, names, ref):
    a = torch.cat([g[m.params.offsets[n]:m.params.offsets[n] + ref[n].numel()] for n in names])
    b = torch.cat([ref[n] for n in names])
    return float(torch.dot(a, b) / (a.norm() * b.norm()))


def main():
    base_l, base_g, m = run({}, fuse=False)
    rl, names, ref = reference(m)
    print("fp32 reference loss %.6f; unfused engine cos vs reference %.6f" % (rl, cos_vs_ref(base_g, m, names, ref)))
    rep_l, rep_g, _ = run({}, fuse=False)
    print("unfused repeat: loss %.6f vs %.6f, max|dg| %.3g" % (base_l, rep_l, float((base_g - rep_g).abs().max())))
    all_off = {"plain": False, "c23": False, "c31": False, "dgrad": False}
    for part in ["plain", "c23", "c31", "dgrad", "all"]:
        parts = dict(all_off)
        if part == "all":
            parts = {k: True for k in parts}
        else:
            parts[part] = True
        l, g, _ = run(parts)
        cos = float(torch.dot(g, base_g) / (g.norm() * base_g.norm()))
        print("== %-6s loss %.6f (unfused %.6f) cos %.6f, cos vs fp32 reference %.6f" % (
            part, l, base_l, cos, cos_vs_ref(g, m, names, ref)))
        worst = []
        for s in m.params.specs:
            if not s.trainable:
                continue
            o = m.params.offsets[s.name]
            n = 1
            for d in s.shape:
                n *= d
            a, b = g[o:o + n], base_g[o:o + n]
            worst.append((float((a - b).norm() / (b.norm() + 1e-20)), s.name))
        worst.sort(reverse=True)
        print("   worst:", ", ".join("%s %.3f" % (nm, r) for r, nm in worst[:6]))


if __name__ == "__main__":
    main()
