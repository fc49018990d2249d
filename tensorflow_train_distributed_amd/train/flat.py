"""Flat parameter store + fused flat optimizers.

MI355X-first memory layout: every trainable variable of a model is a *view* into one
contiguous fp32 master buffer, its gradient a view into one contiguous fp32 gradient buffer
and its compute copy a view into one bf16 buffer. Consequences:

* the optimizer step is ONE kernel launch over a chunk table (optim.hip);
* the gradient all-reduce buckets are contiguous slices of the gradient buffer, so the
  collective engine reduces in place (no pack/unpack copies), in the order the backward
  pass finishes them (variables are laid out in backward-completion order);
* kernels write weight gradients straight into their slice (no autograd accumulation);
* 288 GB of HBM makes the fp32 master + bf16 copy + optimizer state trivially resident.

Reference parity: the reference's ten MLP variables (hidden{1..4}/{kernel,bias},
output/{kernel,bias}) updated by ApplyGradientDescent (distribute_training.py:150-152)
are exactly such a flat set; GradientDescent/Momentum/Adam/LAMB all run on it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

ALIGN = 64  # elements (256 B of fp32): every variable starts 16-B aligned for vector loads
CHUNK = 16384

HYPER_SIZE = 8
# hyper slots (must match optim.hip)
H_LR, H_MU, H_BETA2, H_EPS, H_BC1, H_BC2, H_MAXNORM, H_GRADSCALE = range(8)


@dataclass
class ParamSpec:
    name: str
    shape: Sequence[int]
    init: Optional[Callable[[torch.Tensor], None]] = None
    weight_decay: bool = True
    trainable: bool = True
    meta: dict = field(default_factory=dict)


class FlatParams:
    def __init__(self, specs: List[ParamSpec], device, compute_dtype=torch.bfloat16, seed: int = 0,
                 device_init: bool = False):
        self.device = torch.device(device)
        self.specs = list(specs)
        self.offsets: Dict[str, int] = {}
        off = 0
        for s in self.specs:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            self.offsets[s.name] = off
            off += int(np.prod(s.shape)) if len(s.shape) else 1
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.compute_dtype = compute_dtype
        self.compute = (torch.zeros(self.numel, dtype=compute_dtype, device=self.device)
                        if compute_dtype is not None and compute_dtype != torch.float32 else None)
        self.var: Dict[str, torch.Tensor] = {}
        self.g: Dict[str, torch.Tensor] = {}
        self.c: Dict[str, torch.Tensor] = {}
        for s in self.specs:
            o, n = self.offsets[s.name], int(np.prod(s.shape)) if len(s.shape) else 1
            shape = tuple(s.shape)
            self.var[s.name] = self.master[o:o + n].view(shape)
            self.g[s.name] = self.grad[o:o + n].view(shape)
            if self.compute is not None:
                self.c[s.name] = self.compute[o:o + n].view(shape)
        gen = torch.Generator(device="cpu")
        gen.manual_seed(seed)
        # device_init: initialisers that describe their distribution (`init.dev` = (dist, a, b),
        # see models/resnet.py) run as the Philox init kernel on the GPU (init.hip), keyed by
        # (seed, variable index) — no host RNG or host->device copy of the whole model
        on_dev = device_init and self.device.type == "cuda"
        with torch.no_grad():
            for i, s in enumerate(self.specs):
                dev = getattr(s.init, "dev", None) if on_dev else None
                if dev is not None:
                    from ..ops import kernels as K
                    K.init_random_(self.var[s.name], dev[0], dev[1], dev[2], seed=seed, offset=i)
                    rows = getattr(s.init, "dev_zero_rows", None)
                    if rows is not None:
                        self.var[s.name][rows:].zero_()
                elif s.init is not None:
                    t = torch.empty(tuple(s.shape), dtype=torch.float32)
                    s.init(t, gen)
                    self.var[s.name].copy_(t)
        self.refresh_compute()
        self._chunks = None
        self._seg_wd = None

    # -- helpers ---------------------------------------------------------------------
    def names(self):
        return [s.name for s in self.specs]

    def spec(self, name) -> ParamSpec:
        for s in self.specs:
            if s.name == name:
                return s
        raise KeyError(name)

    def refresh_compute(self):
        if self.compute is not None:
            with torch.no_grad():
                if self.device.type == "cuda":
                    from ..ops import kernels as K
                    K.f32_to_bf16(self.master, self.compute)
                else:
                    self.compute.copy_(self.master)

    def zero_grad(self):
        if self.grad.is_cuda:
            from ..ops import kernels as K
            K.zero_(self.grad)  # hipMemsetAsync, no framework kernel
        else:
            self.grad.zero_()

    def valid_mask(self):
        """1.0 on trainable variable elements, 0.0 on alignment padding / non-trainables."""
        m = getattr(self, "_valid", None)
        if m is None:
            m = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            for s in self.specs:
                if s.trainable:
                    o = self.offsets[s.name]
                    m[o:o + (int(np.prod(s.shape)) if len(s.shape) else 1)] = 1.0
            self._valid = m
        return m

    def chunk_table(self):
        """Device tensors (chunks, seg_wd_mask) for the optim.hip kernels."""
        if self._chunks is None:
            rows = []
            for seg, s in enumerate(self.specs):
                o, n = self.offsets[s.name], int(np.prod(s.shape)) if len(s.shape) else 1
                if not s.trainable:
                    continue
                for st in range(0, n, CHUNK):
                    rows.append((o + st, min(CHUNK, n - st), seg))
            arr = np.zeros(len(rows), dtype=np.dtype([("start", "<i8"), ("len", "<i4"), ("seg", "<i4")]))
            for i, r in enumerate(rows):
                arr[i] = r
            self._chunks = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)
            self._n_chunks = len(rows)
            self._decay_mask = torch.tensor([1.0 if s.weight_decay else 0.0 for s in self.specs],
                                            dtype=torch.float32, device=self.device)
        return self._chunks, self._n_chunks, self._decay_mask

    def state_dict(self):
        return {n: self.var[n].detach().cpu().clone() for n in self.names()}

    def load_state_dict(self, sd, strict=True):
        with torch.no_grad():
            for n in self.names():
                if n in sd:
                    self.var[n].copy_(torch.as_tensor(sd[n]).reshape(self.var[n].shape))
                elif strict:
                    raise KeyError("missing variable %s" % n)
        self.refresh_compute()


# ---------------------------------------------------------------------- LR schedules
@dataclass
class Schedule:
    """Device-evaluable learning-rate schedule (mirrors optim.hip lr_schedule_kernel).

    kind 0 constant, 1 exponential decay (tf.train.exponential_decay), 2 polynomial decay with
    linear warmup, 3 warmup + cosine.
    """
    kind: int = 0
    base_lr: float = 0.01
    decay_steps: float = 1.0
    decay_rate: float = 1.0
    staircase: bool = False
    warmup_steps: float = 0.0
    end_lr: float = 0.0
    power: float = 1.0
    total_steps: float = 1.0

    def params(self):
        return [self.base_lr, self.decay_steps, self.decay_rate, 1.0 if self.staircase else 0.0,
                self.warmup_steps, self.end_lr, self.power, self.total_steps]

    def value(self, step: int) -> float:
        s = float(step)
        if self.kind == 1:
            p = s / self.decay_steps
            if self.staircase:
                p = math.floor(p)
            return self.base_lr * self.decay_rate ** p
        if self.kind == 2:
            if self.warmup_steps > 0 and s < self.warmup_steps:
                return self.base_lr * (s + 1) / self.warmup_steps
            t = min(s, self.total_steps)
            return (self.base_lr - self.end_lr) * (1 - t / self.total_steps) ** self.power + self.end_lr
        if self.kind == 3:
            if self.warmup_steps > 0 and s < self.warmup_steps:
                return self.base_lr * (s + 1) / self.warmup_steps
            frac = min(1.0, (s - self.warmup_steps) / max(1.0, self.total_steps - self.warmup_steps))
            return self.end_lr + 0.5 * (self.base_lr - self.end_lr) * (1 + math.cos(math.pi * frac))
        return self.base_lr


# ---------------------------------------------------------------------- optimizers
class FlatOptimizer:
    """Base class: owns optimizer state for a FlatParams and the device hyper array.

    step() reads the gradient buffer, updates master weights (+ bf16 compute copy) in one
    fused launch (GPU) or with torch ops (CPU). With `device_schedule=True` the LR and Adam
    bias corrections are computed on device from a device-resident global step, so the call
    can live inside a captured hipGraph.
    """

    kind_name = "sgd"

    def __init__(self, params: FlatParams, schedule: Schedule, weight_decay=0.0, max_grad_norm=0.0,
                 beta1=0.9, beta2=0.999, eps=1e-8):
        self.p = params
        self.schedule = schedule
        self.weight_decay = float(weight_decay)
        self.max_grad_norm = float(max_grad_norm)
        self.beta1, self.beta2, self.eps = float(beta1), float(beta2), float(eps)
        dev = params.device
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)  # device global step
        self.hyper = torch.zeros(HYPER_SIZE, dtype=torch.float32, device=dev)
        self.sched_t = torch.tensor(schedule.params(), dtype=torch.float32, device=dev)
        self.hyper[H_MU] = self.beta1
        self.hyper[H_BETA2] = self.beta2
        self.hyper[H_EPS] = self.eps
        self.hyper[H_MAXNORM] = self.max_grad_norm
        self.hyper[H_GRADSCALE] = 1.0
        self.hyper[H_LR] = schedule.value(0)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._host_step = 0

    @property
    def is_cuda(self):
        return self.p.device.type == "cuda"

    def seg_wd(self):
        """Per-segment weight decay (cached: computed once, not per step)."""
        c = getattr(self, "_seg_wd", None)
        if c is None or c[0] != self.weight_decay:
            _, _, mask = self.p.chunk_table()
            c = (self.weight_decay, mask * self.weight_decay)
            self._seg_wd = c
        return c[1]

    def set_step(self, step: int):
        self.step_t.fill_(int(step))
        self._host_step = int(step)

    def current_lr(self):
        return self.schedule.value(self._host_step)

    def _prologue(self, increment=True):
        """Evaluate the schedule for the current step (device) and advance the step."""
        from ..ops import _lib
        if self.is_cuda:
            _lib.call("ttdk_lr_schedule", self.step_t.data_ptr(), self.sched_t.data_ptr(), self.schedule.kind,
                      self.hyper.data_ptr(), self.beta1, self.beta2, int(increment), _lib.stream())
            if self.max_grad_norm > 0:
                from ..ops import kernels as K
                K.sumsq(self.p.grad, out=self._sumsq)
        else:
            s = self._host_step
            self.hyper[H_LR] = self.schedule.value(s)
            self.hyper[H_BC1] = 1 - self.beta1 ** (s + 1)
            self.hyper[H_BC2] = 1 - self.beta2 ** (s + 1)
            if increment:
                self.step_t += 1
        if increment:
            self._host_step += 1

    def _masked_grad(self):
        return self.p.grad * self.p.valid_mask()

    def _clip_scale_cpu(self):
        gs = float(self.hyper[H_GRADSCALE])
        if self.max_grad_norm > 0:
            n = float(self._masked_grad().norm()) * gs
            if n > self.max_grad_norm:
                gs *= self.max_grad_norm / n
        return gs

    def step(self):
        raise NotImplementedError


class FlatSGD(FlatOptimizer):
    """GradientDescent (momentum=0) / Momentum / Nesterov momentum (TF MomentumOptimizer:
    accum = mu*accum + g; w -= lr*accum)."""

    def __init__(self, params, schedule, momentum=0.0, nesterov=False, **kw):
        super().__init__(params, schedule, beta1=momentum, **kw)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)
        self.mom = torch.zeros_like(params.master) if momentum > 0 else None

    def step(self):
        self._prologue()
        kind = 0 if self.mom is None else (2 if self.nesterov else 1)
        if self.is_cuda:
            from ..ops import _lib
            chunks, n, _ = self.p.chunk_table()
            _lib.call("ttdk_opt_sgd", self.p.master.data_ptr(), self.p.grad.data_ptr(),
                      self.mom.data_ptr() if self.mom is not None else None,
                      self.p.compute.data_ptr() if self.p.compute is not None else None, chunks.data_ptr(), n,
                      self.seg_wd().data_ptr(), self.hyper.data_ptr(),
                      self._sumsq.data_ptr() if self.max_grad_norm > 0 else None, kind, _lib.stream())
            return
        with torch.no_grad():
            lr = float(self.hyper[H_LR])
            g = self._masked_grad() * self._clip_scale_cpu()
            if self.weight_decay:
                g = g + self._wd_vector() * self.p.master
            if self.mom is None:
                self.p.master.sub_(lr * g)
            else:
                self.mom.mul_(self.momentum).add_(g)
                upd = g + self.momentum * self.mom if self.nesterov else self.mom
                self.p.master.sub_(lr * upd)
            self.p.refresh_compute()

    def _wd_vector(self):
        v = torch.zeros_like(self.p.master)
        for s in self.p.specs:
            if s.weight_decay and s.trainable:
                o = self.p.offsets[s.name]
                v[o:o + int(np.prod(s.shape))] = self.weight_decay
        return v


class FlatAdam(FlatOptimizer):
    """TF AdamOptimizer semantics (lr_t = lr*sqrt(1-b2^t)/(1-b1^t)); decoupled=True gives AdamW."""

    def __init__(self, params, schedule, beta1=0.9, beta2=0.999, eps=1e-8, decoupled=False, **kw):
        super().__init__(params, schedule, beta1=beta1, beta2=beta2, eps=eps, **kw)
        self.decoupled = bool(decoupled)
        self.m = torch.zeros_like(params.master)
        self.v = torch.zeros_like(params.master)

    def step(self):
        self._prologue()
        if self.is_cuda:
            from ..ops import _lib
            chunks, n, _ = self.p.chunk_table()
            _lib.call("ttdk_opt_adam", self.p.master.data_ptr(), self.p.grad.data_ptr(), self.m.data_ptr(),
                      self.v.data_ptr(), self.p.compute.data_ptr() if self.p.compute is not None else None,
                      chunks.data_ptr(), n, self.seg_wd().data_ptr(), self.hyper.data_ptr(),
                      self._sumsq.data_ptr() if self.max_grad_norm > 0 else None, int(self.decoupled),
                      _lib.stream())
            return
        with torch.no_grad():
            lr = float(self.hyper[H_LR])
            bc1, bc2 = float(self.hyper[H_BC1]), float(self.hyper[H_BC2])
            g = self._masked_grad() * self._clip_scale_cpu()
            wdv = FlatSGD._wd_vector(self) if self.weight_decay else None
            if wdv is not None and not self.decoupled:
                g = g + wdv * self.p.master
            self.m.mul_(self.beta1).add_((1 - self.beta1) * g)
            self.v.mul_(self.beta2).add_((1 - self.beta2) * g * g)
            step = lr * math.sqrt(bc2) / bc1
            w_old = self.p.master.clone()
            self.p.master.sub_(step * self.m / (self.v.sqrt() + self.eps))
            if wdv is not None and self.decoupled:
                self.p.master.sub_(lr * wdv * w_old)
            self.p.refresh_compute()


class FlatLAMB(FlatOptimizer):
    """LAMB (You et al. 2019): Adam direction + decoupled wd, scaled per variable by the
    trust ratio ||w|| / ||u||."""

    def __init__(self, params, schedule, beta1=0.9, beta2=0.999, eps=1e-6, **kw):
        super().__init__(params, schedule, beta1=beta1, beta2=beta2, eps=eps, **kw)
        self.m = torch.zeros_like(params.master)
        self.v = torch.zeros_like(params.master)
        self.u = torch.zeros_like(params.master)
        self.seg_norms = torch.zeros(2 * len(params.specs), dtype=torch.float32, device=params.device)

    def step(self):
        self._prologue()
        if self.is_cuda:
            from ..ops import _lib
            chunks, n, _ = self.p.chunk_table()
            if getattr(self, "_chunk_norms", None) is None or self._chunk_norms.numel() < 2 * n:
                self._chunk_norms = torch.empty(2 * max(1, n), dtype=torch.float32, device=self.p.device)
            _lib.call("ttdk_opt_lamb", self.p.master.data_ptr(), self.p.grad.data_ptr(), self.m.data_ptr(),
                      self.v.data_ptr(), self.u.data_ptr(),
                      self.p.compute.data_ptr() if self.p.compute is not None else None, chunks.data_ptr(), n,
                      len(self.p.specs), self.seg_wd().data_ptr(), self.hyper.data_ptr(),
                      self._sumsq.data_ptr() if self.max_grad_norm > 0 else None, self.seg_norms.data_ptr(),
                      self._chunk_norms.data_ptr(), _lib.stream())
            return
        with torch.no_grad():
            lr = float(self.hyper[H_LR])
            bc1, bc2 = float(self.hyper[H_BC1]), float(self.hyper[H_BC2])
            g = self._masked_grad() * self._clip_scale_cpu()
            self.m.mul_(self.beta1).add_((1 - self.beta1) * g)
            self.v.mul_(self.beta2).add_((1 - self.beta2) * g * g)
            u = (self.m / bc1) / ((self.v / bc2).sqrt() + self.eps)
            if self.weight_decay:
                u = u + FlatSGD._wd_vector(self) * self.p.master
            for s in self.p.specs:
                if not s.trainable:
                    continue
                o, k = self.p.offsets[s.name], int(np.prod(s.shape))
                w = self.p.master[o:o + k]
                uu = u[o:o + k]
                wn, un = float(w.norm()), float(uu.norm())
                trust = wn / un if wn > 0 and un > 0 else 1.0
                w.sub_(lr * trust * uu)
            self.p.refresh_compute()
