"""TF1-style optimizers, learning-rate schedules and the TrainOp that executes a step.

Reference surface (/root/reference/distribute_training.py:114-165):
* `tf.train.exponential_decay(0.01, global_step, 468, 0.96, staircase=True)` (:136-140);
* `tf.train.GradientDescentOptimizer(lr)` (:145,150), `opt.minimize(loss, global_step)` (:152);
* `tf.train.SyncReplicasOptimizer(opt, replicas_to_aggregate=n, total_num_replicas=n)` +
  `make_session_run_hook(is_chief)` (:144-148).
Plus the north-star optimizers (Momentum, Adam/AdamW, LAMB) on fused flat kernels.

`minimize(model, global_step)` returns a TrainOp. Executing it (MonitoredTrainingSession.run
or strategy.run) performs one complete step in the mode chosen at construction:
  local        forward/backward -> fused optimizer launch
  mirrored     forward/backward with bucketed RCCL all-reduce overlapped -> optimizer
  ps-async     pull -> forward/backward -> Hogwild ApplyGD on the PS (global_step += 1)
  ps-sync      pull -> forward/backward -> accumulator push -> token dequeue (the chief's
               queue-runner thread takes the mean of N fresh gradients and applies it).
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Union

import numpy as np
import torch

from ..utils import errors
from . import graph as G
from .flat import FlatAdam, FlatLAMB, FlatOptimizer, FlatParams, FlatSGD, Schedule


# ------------------------------------------------------------------ learning-rate schedules
class LearningRateSchedule(Schedule):
    """A Schedule bound to a global step: calling it (no args) evaluates at the current step."""

    def __init__(self, global_step: Optional[G.GlobalStep] = None, **kw):
        super().__init__(**kw)
        self.global_step = global_step

    def __call__(self, step=None):
        if step is None:
            step = self.global_step.value() if self.global_step is not None else 0
        return self.value(int(step))

    def __float__(self):
        return float(self())


def exponential_decay(learning_rate, global_step, decay_steps, decay_rate, staircase=False, name=None):
    """lr * decay_rate ^ (global_step / decay_steps) (floored when staircase)."""
    return LearningRateSchedule(global_step, kind=1, base_lr=float(learning_rate), decay_steps=float(decay_steps),
                                decay_rate=float(decay_rate), staircase=bool(staircase))


def polynomial_decay(learning_rate, global_step, decay_steps, end_learning_rate=0.0001, power=1.0, cycle=False,
                     warmup_steps=0, name=None):
    return LearningRateSchedule(global_step, kind=2, base_lr=float(learning_rate), end_lr=float(end_learning_rate),
                                power=float(power), total_steps=float(decay_steps), warmup_steps=float(warmup_steps))


def cosine_decay(learning_rate, global_step, decay_steps, alpha=0.0, warmup_steps=0, name=None):
    return LearningRateSchedule(global_step, kind=3, base_lr=float(learning_rate),
                                end_lr=float(learning_rate) * alpha, total_steps=float(decay_steps),
                                warmup_steps=float(warmup_steps))


def _as_schedule(lr) -> Schedule:
    if isinstance(lr, Schedule):
        return lr
    return Schedule(kind=0, base_lr=float(lr))


# ------------------------------------------------------------------ optimizers
class Optimizer:
    flat_cls = FlatSGD
    supports_ps = False

    def __init__(self, learning_rate, use_locking=False, name="Optimizer", weight_decay=0.0, max_grad_norm=0.0):
        self.learning_rate = learning_rate
        self.schedule = _as_schedule(learning_rate)
        self.use_locking = use_locking
        self.name = name
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.flat: Optional[FlatOptimizer] = None

    def _make_flat(self, params: FlatParams) -> FlatOptimizer:
        return FlatSGD(params, self.schedule, weight_decay=self.weight_decay, max_grad_norm=self.max_grad_norm)

    def build(self, params: FlatParams) -> FlatOptimizer:
        if self.flat is None or self.flat.p is not params:
            self.flat = self._make_flat(params)
        return self.flat

    def minimize(self, model, global_step: Optional[G.GlobalStep] = None, var_list=None, name=None,
                 strategy=None) -> "TrainOp":
        """`model` with forward_backward (the framework's engines): returns a TrainOp to run
        in a session / strategy.run. A loss tensor or zero-argument loss callable with
        var_list (user-defined ttd.layers models, TF2 style): computes and applies the
        gradients now."""
        if var_list is not None and (callable(model) and not hasattr(model, "forward_backward")
                                     or isinstance(model, torch.Tensor)):
            return self.apply_gradients(self.compute_gradients(model, var_list), global_step=global_step)
        return TrainOp(model, self, global_step, strategy=strategy, name=name or "train_op")

    def compute_gradients(self, loss, var_list=None, **kw):
        """tf.train.Optimizer.compute_gradients: [(gradient, variable)] of a scalar loss tensor
        (or a zero-argument callable returning it) w.r.t. var_list (flat-backed model
        variables: aggregated across replicas, see train/tape.py)."""
        from .tape import GradientTape
        if var_list is None:
            raise errors.InvalidArgumentError("compute_gradients needs var_list (e.g. model.trainable_variables)")
        var_list = list(var_list)
        with GradientTape() as tape:
            value = loss() if callable(loss) else loss
        return list(zip(tape.gradient(value, var_list), var_list))

    def apply_gradients(self, grads_and_vars, global_step=None, name=None, experimental_aggregate_gradients=True):
        """Apply (gradient, variable) pairs with the fused flat optimizer; under a multi-replica
        strategy the gradients are all-reduced (SUM) first unless GradientTape already did it."""
        from .tape import apply_gradients
        return apply_gradients(self, grads_and_vars, global_step=global_step,
                               experimental_aggregate_gradients=experimental_aggregate_gradients)

    def variables(self):
        return [] if self.flat is None else [t for t in (getattr(self.flat, k, None) for k in ("mom", "m", "v"))
                                             if isinstance(t, torch.Tensor)]


class GradientDescentOptimizer(Optimizer):
    supports_ps = True

    def __init__(self, learning_rate, use_locking=False, name="GradientDescent", **kw):
        super().__init__(learning_rate, use_locking, name, **kw)


class MomentumOptimizer(Optimizer):
    def __init__(self, learning_rate, momentum, use_locking=False, name="Momentum", use_nesterov=False, **kw):
        super().__init__(learning_rate, use_locking, name, **kw)
        self.momentum = momentum
        self.use_nesterov = use_nesterov

    def _make_flat(self, params):
        return FlatSGD(params, self.schedule, momentum=self.momentum, nesterov=self.use_nesterov,
                       weight_decay=self.weight_decay, max_grad_norm=self.max_grad_norm)


class AdamOptimizer(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, use_locking=False, name="Adam",
                 decoupled_weight_decay=False, **kw):
        super().__init__(learning_rate, use_locking, name, **kw)
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon
        self.decoupled = decoupled_weight_decay

    def _make_flat(self, params):
        return FlatAdam(params, self.schedule, beta1=self.beta1, beta2=self.beta2, eps=self.epsilon,
                        decoupled=self.decoupled, weight_decay=self.weight_decay, max_grad_norm=self.max_grad_norm)


class AdamWOptimizer(AdamOptimizer):
    def __init__(self, learning_rate=0.001, weight_decay=0.01, **kw):
        super().__init__(learning_rate, decoupled_weight_decay=True, weight_decay=weight_decay, name="AdamW", **kw)


class LAMBOptimizer(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-6, weight_decay=0.01, name="LAMB",
                 **kw):
        super().__init__(learning_rate, False, name, weight_decay=weight_decay, **kw)
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon

    def _make_flat(self, params):
        return FlatLAMB(params, self.schedule, beta1=self.beta1, beta2=self.beta2, eps=self.epsilon,
                        weight_decay=self.weight_decay, max_grad_norm=self.max_grad_norm)


class SyncReplicasOptimizer(Optimizer):
    """Synchronous aggregation: a step applies the MEAN of `replicas_to_aggregate` fresh
    gradients; gradients computed against an older global step are dropped."""

    def __init__(self, opt: Optimizer, replicas_to_aggregate: int, total_num_replicas: Optional[int] = None,
                 variable_averages=None, variables_to_average=None, use_locking=False, name="sync_replicas"):
        super().__init__(opt.learning_rate, use_locking, name)
        self.opt = opt
        self.schedule = opt.schedule
        self.replicas_to_aggregate = int(replicas_to_aggregate)
        self.total_num_replicas = int(total_num_replicas if total_num_replicas is not None else replicas_to_aggregate)
        self.tokens_per_step = max(self.total_num_replicas, self.replicas_to_aggregate)
        self.variable_averages = variable_averages
        self._train_op: Optional["TrainOp"] = None

    def _make_flat(self, params):
        return self.opt._make_flat(params)

    def minimize(self, model, global_step=None, var_list=None, name=None, strategy=None):
        op = TrainOp(model, self, global_step, strategy=strategy, name=name or "train_op", sync=True)
        self._train_op = op
        return op

    def make_session_run_hook(self, is_chief: bool, num_tokens: int = -1):
        from .hooks import SyncReplicasOptimizerHook
        return SyncReplicasOptimizerHook(self, is_chief, num_tokens)


# ------------------------------------------------------------------ TrainOp
class TrainOp:
    """One executable training step (what `opt.minimize()` returns)."""

    def __init__(self, model, optimizer: Optimizer, global_step: Optional[G.GlobalStep] = None, strategy=None,
                 name="train_op", sync=False):
        from ..parallel.ps import current_device_setter
        from ..parallel.strategy import get_strategy
        self.model = model
        self.optimizer = optimizer
        self.name = name
        self.sync = sync
        self.global_step = global_step if global_step is not None else G.get_or_create_global_step()
        self.strategy = strategy if strategy is not None else get_strategy(allow_default=True)
        self.setter = current_device_setter()
        self.params: FlatParams = model.params
        self.mode = "ps" if (self.setter is not None and self.setter.ps_tasks > 0) else \
            ("mirrored" if self.strategy is not None and self.strategy.num_replicas_in_sync > 1 else "local")
        if self.mode == "ps":
            if not (optimizer.supports_ps or (sync and optimizer.opt.supports_ps)):
                raise errors.InvalidArgumentError("parameter-server mode applies GradientDescent on the PS; "
                                                  "use GradientDescentOptimizer (optionally in SyncReplicasOptimizer)")
            # TF round-robin: the global step (created first) and then every variable in
            # creation (forward) order.
            self.setter.assign(self.global_step.name)
            for n in getattr(model, "creation_order", lambda: [s.name for s in self.params.specs])():
                self.setter.assign(n, int(np.prod(self.params.spec(n).shape)) * 4)
            self.placement = {s.name: self.setter.placement[s.name] for s in self.params.specs}
        self.flat = optimizer.build(self.params) if self.mode != "ps" else None
        self.reducer = None
        self.outputs: Dict[str, object] = {}
        self.client = None           # PSClient, set by the session
        self.local_step = 0          # SyncReplicas local step (token value)
        self._host_params = None
        self._host_grads = None
        if self.mode in ("local", "mirrored") and self.flat is not None:
            # the optimizer's step counter is the global step (identical on every replica)
            self.global_step.bind(lambda: self.flat._host_step, self._set_step_local)
        g = G.get_default_graph()
        g.add_to_collection(G.TRAIN_OP, self)

    # handles for session.run fetches
    def __getitem__(self, key) -> G.Fetch:
        return G.Fetch(self, key)

    @property
    def loss(self) -> G.Fetch:
        return G.Fetch(self, "loss")

    @property
    def accuracy(self) -> G.Fetch:
        return G.Fetch(self, "accuracy")

    def _set_step_local(self, v):
        if self.flat is not None:
            self.flat.set_step(v)

    # -- PS wiring (called by the session on creation / re-creation)
    def attach_ps(self, client):
        self.client = client
        self.global_step.bind(client.global_step, client.set_global_step)
        P = self.params
        if P.device.type == "cpu":
            base = P.master.numpy()
            gbase = P.grad.numpy()
        else:
            self._pin_m = torch.empty(P.numel, dtype=torch.float32, pin_memory=True)
            self._pin_g = torch.empty(P.numel, dtype=torch.float32, pin_memory=True)
            base = self._pin_m.numpy()
            gbase = self._pin_g.numpy()
        self._host_params, self._host_grads = {}, {}
        for s in P.specs:
            o, n = P.offsets[s.name], int(np.prod(s.shape))
            self._host_params[s.name] = base[o:o + n].reshape(s.shape)
            self._host_grads[s.name] = gbase[o:o + n].reshape(s.shape)

    def initial_values(self) -> Dict[str, np.ndarray]:
        return {s.name: self.params.var[s.name].detach().float().cpu().numpy() for s in self.params.specs}

    def _pull(self):
        self.client.pull(self._host_params)
        P = self.params
        if P.device.type != "cpu":
            P.master.copy_(self._pin_m, non_blocking=True)
        P.refresh_compute()

    def _grads_to_host(self):
        P = self.params
        if P.device.type != "cpu":
            self._pin_g.copy_(P.grad)
        return {s.name: self._host_grads[s.name] for s in P.specs if s.trainable}

    # -- execution
    def run(self, feed: Dict) -> Dict[str, object]:
        m = self.model
        if self.mode == "local":
            out = m.forward_backward(feed)
            self.flat.step()
        elif self.mode == "mirrored":
            st = self.strategy
            if self.reducer is None:
                self.reducer = st.make_reducer(self.params)
            self.reducer.begin()
            out = m.forward_backward(feed, grad_scale=st.grad_scale(feed), grad_hook=self.reducer.mark_ready)
            self.reducer.finish()
            self.flat.step()
        else:
            if self.client is None:
                raise errors.FailedPreconditionError("parameter-server TrainOp used outside a session")
            self._pull()
            if not self.sync:
                gs = self.client.global_step()
                lr = self.optimizer.schedule.value(gs)
                out = m.forward_backward(feed)
                grads = self._grads_to_host()
                self.client.apply_gd(lr, grads)
            else:
                out = m.forward_backward(feed)
                grads = self._grads_to_host()
                self.client.accum_apply(self.local_step, grads)
                self.local_step = self.client.dequeue_token()
        self.outputs = out
        return out

    def __call__(self, feed: Dict):
        return self.run(feed)
