"""GradientTape + Optimizer.apply_gradients for user-defined models under a strategy.

Reference behaviour: `opt.minimize(loss, global_step)` computes the gradients of the replica's
loss and applies them, aggregated across replicas when synchronous
(/root/reference/distribute_training.py:142-152); tf.distribute's custom-training-loop form is
`tape.gradient` + `optimizer.apply_gradients` inside `strategy.run`, where apply_gradients
all-reduces (SUM) the replicas' gradients before the update.

MI355X-first execution:
* a `ttd.layers` model built inside `strategy.scope()` keeps its variables as views of ONE
  FlatParams store (fp32 master, flat fp32 gradient buffer laid out in backward-completion
  order), so autograd accumulates every gradient straight into a contiguous bucket slice;
* `tape.gradient` runs the backward with post-accumulate-grad hooks that advance a "ready"
  watermark over the flat layout and launch each all-reduce bucket as soon as it is complete
  (BucketedAllReducer), i.e. the RCCL collectives overlap the rest of the backward; the
  returned gradients are the replica-summed flat views (TF's aggregated gradients);
* `apply_gradients` then runs the fused flat optimizer (one launch for all variables). Gradients
  the caller replaced (clipping, custom grads) are copied into the flat buffer and all-reduced
  in one collective before the update.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from ..utils import errors


def flat_of(var):
    """(FlatParams, TF name) a variable is a view of, or (None, None)."""
    return getattr(var, "_ttd_flat", None), getattr(var, "_ttd_name", None)


def _replica_strategy():
    from ..parallel.strategy import get_strategy
    st = get_strategy(allow_default=True)
    if st is not None and st.num_replicas_in_sync > 1:
        return st
    return None


class _ReadyTracker:
    """Turns per-variable "gradient accumulated" events (any order) into the in-order
    watermark BucketedAllReducer.mark_ready expects."""

    def __init__(self, flat, reducer):
        self.names = [s.name for s in flat.specs]
        self.index = {n: i for i, n in enumerate(self.names)}
        self.trainable = [s.trainable for s in flat.specs]
        self.reducer = reducer
        self.ready = [False] * len(self.names)
        self.next = 0

    def _advance(self):
        j = self.next
        while j < len(self.names) and (self.ready[j] or not self.trainable[j]):
            j += 1
        if j > self.next:
            self.next = j
            self.reducer.mark_ready(self.names[j - 1])

    def hit(self, name):
        i = self.index.get(name)
        if i is not None and not self.ready[i]:
            self.ready[i] = True
            if i == self.next or (i > self.next and all(self.ready[k] or not self.trainable[k]
                                                        for k in range(self.next, i))):
                self._advance()


def _reducer_for(strategy, flat):
    red = getattr(flat, "_ttd_reducer", None)
    if red is None or getattr(flat, "_ttd_reducer_group", None) is not strategy.group \
            or red.world != strategy.num_replicas_in_sync:
        red = strategy.make_reducer(flat)  # broadcasts replica 0's weights once
        flat._ttd_reducer = red
        flat._ttd_reducer_group = strategy.group
    return red


def _arm_hooks(flat):
    """Post-accumulate-grad hooks on every trainable flat variable (installed once).

    While a tape runs the backward, the variables' .grad is None, so autograd's AccumulateGrad
    hands over the freshly computed gradient without an accumulate kernel; the hook moves it
    into the variable's slice of the flat gradient buffer (a same-dtype device copy) and then
    advances the all-reduce watermark."""
    if getattr(flat, "_ttd_hooks", None):
        return
    handles = []
    for name, p in getattr(flat, "_ttd_vars", {}).items():
        if p.requires_grad:
            def hook(param, name=name, flat=flat):
                if getattr(flat, "_ttd_steal", False) and param.grad is not None:
                    dst = flat.g[name]
                    if param.grad.data_ptr() != dst.data_ptr():
                        dst.copy_(param.grad)
                    param.grad = None
                tr = getattr(flat, "_ttd_tracker", None)
                if tr is not None:
                    tr.hit(name)
            handles.append(p.register_post_accumulate_grad_hook(hook))
    flat._ttd_hooks = handles


_ONES = {}


def _seed_grad(target):
    """d(target)/d(target) = 1 for a scalar target, cached per (dtype, device) so a steady-state
    step launches no fill kernel for it."""
    if target.numel() != 1:
        return None
    key = (target.dtype, target.device, tuple(target.shape))
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(target.shape, dtype=target.dtype, device=target.device)
    return t


class GradientTape:
    """tf.GradientTape over torch autograd. Record the forward under the tape, then
    `gradient(loss, variables)`. persistent=True allows several gradient() calls."""

    def __init__(self, persistent: bool = False, watch_accessed_variables: bool = True):
        self.persistent = persistent
        self._used = False

    def __enter__(self):
        self._grad_mode = torch.is_grad_enabled()
        torch.set_grad_enabled(True)
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._grad_mode)
        return False

    def watch(self, tensor):
        if isinstance(tensor, torch.Tensor) and not tensor.requires_grad:
            tensor.requires_grad_(True)

    def gradient(self, target, sources, output_gradients=None, unconnected_gradients="none"):
        if self._used and not self.persistent:
            raise RuntimeError("a non-persistent GradientTape can compute gradients once")
        self._used = True
        single = isinstance(sources, torch.Tensor)
        srcs = [sources] if single else list(sources)
        flats: Dict[int, object] = {}
        for v in srcs:
            fp, _ = flat_of(v)
            if fp is not None:
                flats[id(fp)] = fp
        plain = [v for v in srcs if flat_of(v)[0] is None]
        if plain:
            grads = torch.autograd.grad(target, plain, grad_outputs=output_gradients,
                                        retain_graph=self.persistent, allow_unused=True)
            got = dict(zip(map(id, plain), grads))
            if not flats:
                out = [got.get(id(v)) for v in srcs]
                if unconnected_gradients == "zero":
                    out = [torch.zeros_like(v) if g is None else g for g, v in zip(out, srcs)]
                return out[0] if single else out
        else:
            got = {}
        st = _replica_strategy()
        reducers = []
        for fp in flats.values():
            fp.zero_grad()
            fp._ttd_aggregated = False
            _arm_hooks(fp)
            fp._ttd_steal = True
            for p in getattr(fp, "_ttd_vars", {}).values():
                p.grad = None
            if st is not None:
                red = _reducer_for(st, fp)
                red.begin()
                fp._ttd_tracker = _ReadyTracker(fp, red)
                reducers.append((fp, red))
        seed = output_gradients if output_gradients is not None else _seed_grad(target)
        try:
            target.backward(gradient=seed, retain_graph=self.persistent)
        finally:
            for fp in flats.values():
                fp._ttd_steal = False
                fp._ttd_tracker = None
                for name, p in getattr(fp, "_ttd_vars", {}).items():
                    if p.grad is not None and p.grad.data_ptr() != fp.g[name].data_ptr():
                        fp.g[name].copy_(p.grad)  # a variable without the hook (not trainable)
                    p.grad = fp.g[name]
        for fp, red in reducers:
            red.finish()  # buckets not yet launched (unused variables) go now; waits for all
            fp._ttd_aggregated = True
        out = []
        for v in srcs:
            fp, name = flat_of(v)
            if fp is not None:
                out.append(fp.g[name])
            else:
                g = got.get(id(v))
                out.append(torch.zeros_like(v) if g is None and unconnected_gradients == "zero" else g)
        return out[0] if single else out


def clip_by_global_norm(t_list, clip_norm, use_norm=None):
    """tf.clip_by_global_norm: scale every tensor by clip_norm / max(global_norm, clip_norm).
    Returns (clipped list, global_norm). None entries pass through. One fused norm over the
    list (torch._foreach_norm), no host sync. `use_norm` may be a tensor or a Python number.

    Divergence from TF MirroredStrategy (documented, parity unpinned: the reference has no
    clipping): inside a replica context `GradientTape.gradient` here returns the gradients
    already all-reduced across replicas (the bucketed all-reduce overlaps the backward, tape.py),
    so clipping between `gradient()` and `apply_gradients` clips the replica-SUMMED gradient —
    the same as clipping the big-batch gradient of a single replica. TF clips each replica's
    local gradient there and aggregates afterwards, so its clip triggers at different norms.
    For per-replica clipping, clip inside the loss (or scale the per-replica loss)."""
    ts = [t for t in t_list if t is not None]
    if use_norm is not None and not isinstance(use_norm, torch.Tensor):
        dev = ts[0].device if ts else None
        use_norm = torch.as_tensor(float(use_norm), dtype=torch.float32, device=dev)
    if use_norm is None:
        if ts:
            norms = torch._foreach_norm([t.float() for t in ts])
            use_norm = torch.linalg.vector_norm(torch.stack(norms))
        else:
            use_norm = torch.zeros(())
    scale = clip_norm / torch.maximum(use_norm, torch.as_tensor(clip_norm, dtype=use_norm.dtype,
                                                                    device=use_norm.device))
    out = [None if t is None else t * scale.to(t.dtype) for t in t_list]
    return out, use_norm


def apply_gradients(optimizer, grads_and_vars, global_step=None, name=None,
                    experimental_aggregate_gradients: bool = True):
    """Optimizer.apply_gradients for flat-backed variables (see module docstring)."""
    pairs = [(g, v) for g, v in grads_and_vars]
    if not pairs:
        raise errors.InvalidArgumentError("apply_gradients: no (gradient, variable) pairs")
    fps = {id(flat_of(v)[0]): flat_of(v)[0] for _, v in pairs}
    if None in fps.values() or len(fps) != 1:
        raise errors.InvalidArgumentError(
            "apply_gradients: every variable must belong to one model built under strategy.scope() "
            "(or converted with model.to_flat())")
    fp = next(iter(fps.values()))
    passed = set()
    copied = False
    with torch.no_grad():
        for g, v in pairs:
            _, vname = flat_of(v)
            passed.add(vname)
            dst = fp.g[vname]
            if g is None:
                dst.zero_()
                copied = True
            elif g.data_ptr() != dst.data_ptr():
                dst.copy_(g.reshape(dst.shape))
                copied = True
        for s in fp.specs:  # variables not passed are not updated by their gradient
            if s.trainable and s.name not in passed:
                fp.g[s.name].zero_()
    st = _replica_strategy()
    # One aggregation point: gradients from tape.gradient are already replica-summed (the bucket
    # all-reduce overlapped the backward). Whatever the caller did to them afterwards (clipping,
    # scaling) ran on identical values on every replica, so reducing again would multiply every
    # gradient by the world size. Only gradients that did not come from an aggregating tape
    # (e.g. torch.autograd.grad) are all-reduced here. `copied` only says the flat buffer was
    # refreshed from the caller's tensors.
    del copied
    if st is not None and experimental_aggregate_gradients and not getattr(fp, "_ttd_aggregated", False):
        import torch.distributed as dist
        dist.all_reduce(fp.grad, op=dist.ReduceOp.SUM, group=st.group)
    fp._ttd_aggregated = False
    flat_opt = optimizer.build(fp)
    if global_step is not None and getattr(global_step, "_ttd_bound_to", None) is not flat_opt:
        global_step.bind(lambda: flat_opt._host_step, flat_opt.set_step)
        global_step._ttd_bound_to = flat_opt
    flat_opt.step()
    return flat_opt
