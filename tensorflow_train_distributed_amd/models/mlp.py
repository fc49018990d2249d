"""The reference's MNIST model: a 5-layer dense MLP 784 -> 200 -> 100 -> 50 -> 25 -> 10.

Parity with /root/reference/distribute_training.py:39-110:
* hidden layers `hidden{i}`: Dense (He / variance-scaling truncated-normal init,
  sigma = sqrt(1.3 * 2 / fan_in)), ELU, dropout(rate=0.01, training=True — dropout stays on
  even for the reported accuracy);
* output layer `output`: Dense without activation/regularizer;
* loss = mean sparse softmax cross-entropy; the L1 regularizer (scale 0.01) is built but NOT
  added to the loss (Q1) unless apply_regularization=True;
* accuracy = mean(in_top_k(logits, labels, 1)).
Variables keep TF names/layouts (kernel [in, out]) so checkpoints match the reference's keys.

GPU path (dtype="float32", the default — the reference trains in fp32): exact-fp32 MFMA GEMMs
(gemm_f32.hip, v_mfma_f32_32x32x2_f32) on the fp32 master weights, fused bias+ELU+Philox-dropout
and the fused xent/in_top_k kernel in fp32, gradients written straight into the flat fp32
gradient buffer; a GPU step matches the CPU fp32 step to ~1e-6 relative. dtype="bfloat16" runs
the bf16 MFMA GEMMs (gemm_conv.hip) on a bf16 compute copy instead. CPU path: fp32 PyTorch
autograd (the plumbing config).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..train.flat import FlatParams, ParamSpec


def variance_scaling_init(fan_in, factor=2.0):
    std = math.sqrt(1.3 * factor / fan_in)

    def init(t, gen):
        t.normal_(0.0, std, generator=gen)
        bad = t.abs() > 2 * std
        while bool(bad.any()):  # resample outside +-2 sigma (tf.truncated_normal)
            t[bad] = torch.empty(int(bad.sum())).normal_(0.0, std, generator=gen)
            bad = t.abs() > 2 * std
    init.stddev = std
    return init


def zeros_init(t, gen):
    t.zero_()


class MLP:
    input_names = ("x-input", "y-input")

    def __init__(self, layer_hidden_nums: Sequence[int] = (200, 100, 50, 25, 10), input_dim: int = 784,
                 dropout_rate: float = 0.01, regularizer_scale: float = 0.01, apply_regularization: bool = False,
                 training: bool = True, device="cpu", seed: int = 0, activation: str = "elu",
                 dtype: str = "float32"):
        self.device = torch.device(device)
        if dtype not in ("float32", "bfloat16"):
            raise ValueError("MLP dtype must be float32 or bfloat16, got %r" % (dtype,))
        self.bf16 = dtype == "bfloat16" and self.device.type == "cuda"
        self.sizes = [input_dim] + list(layer_hidden_nums)
        self.names = ["hidden%d" % (i + 1) for i in range(len(layer_hidden_nums) - 1)] + ["output"]
        self.dropout_rate = float(dropout_rate)
        self.regularizer_scale = float(regularizer_scale)
        self.apply_regularization = apply_regularization
        self.training = training
        self.activation = activation
        specs = []
        for i in reversed(range(len(self.names))):  # backward-completion order
            n, fi, fo = self.names[i], self.sizes[i], self.sizes[i + 1]
            specs.append(ParamSpec(n + "/kernel", (fi, fo), variance_scaling_init(fi), True))
            specs.append(ParamSpec(n + "/bias", (fo,), zeros_init, False))
        self.params = FlatParams(specs, self.device, seed=seed,
                                 compute_dtype=torch.bfloat16 if self.bf16 else None)
        self._seed = int(seed) * 7919 + 17
        self._offset = 0

    def creation_order(self):
        """Variable creation order of the TF1 graph (forward order), used by
        replica_device_setter's round-robin placement."""
        return [n + suf for n in self.names for suf in ("/kernel", "/bias")]

    # ------------------------------------------------------------------ feeds
    def _inputs(self, feed: Dict):
        x = feed.get("x-input", feed.get("x"))
        y = feed.get("y-input", feed.get("y"))
        x = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x)
        y = torch.as_tensor(np.asarray(y) if not isinstance(y, torch.Tensor) else y)
        return x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)

    # ------------------------------------------------------------------ reference math (CPU)
    def reference_loss(self, x, y, P=None, rng: Optional[torch.Generator] = None):
        P = P if P is not None else {n: self.params.var[n] for n in self.params.names()}
        a = x.float()
        reg = 0.0
        for i, n in enumerate(self.names):
            z = a @ P[n + "/kernel"] + P[n + "/bias"]
            if i == len(self.names) - 1:
                a = z
                break
            a = F.elu(z) if self.activation == "elu" else F.relu(z)
            if self.training and self.dropout_rate > 0:
                keep = (torch.rand(a.shape, generator=rng, device=a.device) >= self.dropout_rate).float()
                a = a * keep / (1.0 - self.dropout_rate)
            reg = reg + self.regularizer_scale * P[n + "/kernel"].abs().sum()
        logits = a
        loss = F.cross_entropy(logits, y.long())
        tgt = logits.gather(1, y.long()[:, None])
        acc = ((logits > tgt).sum(1) < 1).float().mean()
        total = loss + reg if self.apply_regularization else loss
        return total, loss, acc, logits

    def _cpu_step(self, x, y, grad_scale):
        P = self.params
        leaves = {n: P.var[n].detach().clone().requires_grad_(True) for n in P.names()}
        gen = torch.Generator().manual_seed(self._seed + self._offset)
        self._offset += 1
        total, loss, acc, _ = self.reference_loss(x, y, leaves, gen)
        scale = 1.0 if grad_scale is None else grad_scale * x.shape[0]
        (total * scale).backward()
        with torch.no_grad():
            for n, t in leaves.items():
                P.g[n].copy_(t.grad)
        return {"loss": loss.detach(), "accuracy": acc.detach(), "total_loss": total.detach()}

    # ------------------------------------------------------------------ GPU engine
    def _gpu_step(self, x, y, grad_scale, grad_hook):
        from ..ops import gemm as G
        from ..ops import kernels as K
        P = self.params
        B = x.shape[0]
        if grad_scale is None:
            grad_scale = 1.0 / B
        x = x.float().contiguous()
        if self.bf16:
            a = K.f32_to_bf16(x)
            W = P.c
            mm = G.gemm
        else:
            a = x
            W = P.var
            mm = G.gemm_f32
        act = K.ACT_ELU if self.activation == "elu" else K.ACT_RELU
        rate = self.dropout_rate if self.training else 0.0
        seed = self._seed
        offs = []
        acts, pres = [a], []
        L = len(self.names)
        for i, n in enumerate(self.names):
            if i == L - 1:
                logits = mm(acts[-1], W[n + "/kernel"], bias=P.var[n + "/bias"])
                break
            z = mm(acts[-1], W[n + "/kernel"])
            off = self._offset
            self._offset += 1
            a = K.bias_act_dropout(z, P.var[n + "/bias"], act, rate, seed, off)
            pres.append(z)
            offs.append(off)
            acts.append(a)
        sums, dl, _, _ = K.sparse_xent(logits, y, grad_scale)
        d = dl
        for i in reversed(range(L)):
            n = self.names[i]
            a_in = acts[i]
            if i < L - 1:
                d = K.bias_act_dropout_bwd(d, pres[i], P.var[n + "/bias"], act, rate, seed, offs[i])
            mm(a_in, d, trans_a=True, out=P.g[n + "/kernel"])
            K.colsum(d, out=P.g[n + "/bias"])
            if self.apply_regularization and i < L - 1:
                P.g[n + "/kernel"].add_(self.regularizer_scale * grad_scale * B * torch.sign(P.var[n + "/kernel"]))
            if grad_hook is not None:
                grad_hook(n + "/bias")
            if i > 0:
                d = mm(d, W[n + "/kernel"], trans_b=True)
        return {"loss": sums[0], "accuracy": sums[1]}

    def forward_backward(self, feed: Dict, grad_scale: Optional[float] = None, grad_hook=None):
        x, y = self._inputs(feed)
        if self.device.type == "cuda":
            return self._gpu_step(x, y, grad_scale, grad_hook)
        out = self._cpu_step(x, y, grad_scale)
        if grad_hook is not None:
            grad_hook(self.params.specs[-1].name)
        return out

    def evaluate(self, feed: Dict, training: Optional[bool] = None) -> Dict[str, float]:
        """Forward only (no gradients): loss and accuracy on a batch."""
        x, y = self._inputs(feed)
        saved = self.training
        if training is not None:
            self.training = training
        try:
            with torch.no_grad():
                P = {n: self.params.var[n].float() for n in self.params.names()}
                gen = torch.Generator(device=x.device).manual_seed(self._seed)
                _, loss, acc, _ = self.reference_loss(x.float(), y, P, gen)
        finally:
            self.training = saved
        return {"loss": float(loss), "accuracy": float(acc)}


def mnist_mlp(device="cpu", **kw) -> MLP:
    return MLP(device=device, **kw)
