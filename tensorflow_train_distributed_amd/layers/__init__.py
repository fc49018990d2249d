"""`ttd.layers` — tf.layers / Keras-style layers over `ttd.nn`.

Layers create their variables on first call (Keras `build`) with TF names
(`dense/kernel`, `dense_1/bias`, `conv2d/kernel` [R, S, C, K], ...), so `ttd.train.Saver`
/ `Checkpoint` write TF-compatible keys. Compute dispatches through `ttd.nn` (HIP kernels
for GPU tensors, fp32 PyTorch on CPU).

    x = ttd.layers.dense(x, 200, activation=ttd.nn.elu, kernel_initializer=..., name="hidden1")
    model = ttd.layers.Sequential([ttd.layers.Dense(200, "elu"), ttd.layers.Dropout(0.01),
                                   ttd.layers.Dense(10)])
    flat = model.to_flat(device)   # one FlatParams for the fused optimizers / all-reduce

Regularizer outputs go to `layer.losses` and the REGULARIZATION_LOSSES collection; like
tf.layers they are NOT part of any loss unless the caller adds them (reference quirk Q1).
"""
from __future__ import annotations

import collections
from typing import Callable, Dict, List, Optional, Sequence, Union

import torch

from .. import initializers as I
from .. import nn as N

_name_uid: Dict[str, int] = collections.defaultdict(int)
_depth = [0]  # nesting depth of Layer calls (the outermost call owns the model)
_generator = torch.Generator(device="cpu")
_generator.manual_seed(0)


def reset_naming(seed: Optional[int] = None):
    _name_uid.clear()
    if seed is not None:
        _generator.manual_seed(seed)


def _unique(base: str) -> str:
    n = _name_uid[base]
    _name_uid[base] += 1
    return base if n == 0 else "%s_%d" % (base, n)


def _child_layers(mod):
    """Direct Layer descendants of `mod`, looking through plain containers (ModuleList)."""
    for m in mod.children():
        if isinstance(m, Layer):
            yield m
        else:
            yield from _child_layers(m)


def _act(a):
    if a is None or callable(a):
        return a
    return {"linear": None, "relu": N.relu, "elu": N.elu, "gelu": N.gelu, "tanh": N.tanh}[a]


class Layer(torch.nn.Module):
    _default_name = "layer"

    def __init__(self, name: Optional[str] = None, trainable: bool = True):
        super().__init__()
        self.layer_name = name or _unique(self._default_name)
        self.trainable = trainable
        self.built = False
        self._var_names: List[str] = []
        self._regularizers = []

    # TF-style variable creation
    def add_weight(self, name, shape, initializer="zeros", regularizer=None, trainable=True, attr=None):
        """Create variable `<layer name>/<name>`, registered as attribute `attr` (default: name
        with '/' -> '_'); always read it back through that attribute (to_flat re-homes it)."""
        init = I.get(initializer)
        value = init(tuple(shape), _generator)
        p = torch.nn.Parameter(value, requires_grad=trainable and self.trainable)
        key = attr or name.replace("/", "_")
        self.register_parameter(key, p)
        self._var_names.append((self.layer_name + "/" + name, key))
        if regularizer is not None:
            self._regularizers.append((regularizer, key))
        return p

    def build(self, input_shape):
        self.built = True

    def call(self, x, **kw):
        raise NotImplementedError

    def forward(self, x, **kw):
        if not self.built:
            self.build(tuple(x.shape))
            self.built = True
            if x.is_cuda:
                self.to(x.device)
        top = _depth[0] == 0
        _depth[0] += 1
        try:
            out = self.call(x, **kw)
        finally:
            _depth[0] -= 1
        if top and getattr(self, "params", None) is None and self._var_names_all():
            from ..parallel.strategy import get_strategy, has_strategy
            if has_strategy():
                # built inside strategy.scope(): the model's variables become one flat store
                # (fused optimizer, bucketed all-reduce overlapped with the backward), mirrored
                # from replica 0 like tf.distribute's variable creation; the building call is
                # then re-run on the flat variables so its autograd graph feeds them
                fp = self.to_flat(x.device)
                st = get_strategy()
                if st is not None and st.num_replicas_in_sync > 1:
                    from ..parallel.collective import broadcast_flat_
                    broadcast_flat_(fp, group=st.group)
                _depth[0] += 1
                try:
                    out = self.call(x, **kw)
                finally:
                    _depth[0] -= 1
        return out

    def _var_names_all(self):
        return bool(self._var_names) or any(m._var_names for m in self.modules() if isinstance(m, Layer))

    @property
    def losses(self):
        out = [r(getattr(self, key)) for r, key in self._regularizers]
        for m in _child_layers(self):
            out += m.losses
        return out

    def named_variables(self):
        """(TF variable name, tensor) for this layer and its sub-layers."""
        out = [(full, getattr(self, key)) for full, key in self._var_names]
        for m in _child_layers(self):
            out += m.named_variables()
        return out

    @property
    def variables(self):
        return [t for _, t in self.named_variables()]

    @property
    def trainable_variables(self):
        return [t for _, t in self.named_variables() if t.requires_grad]

    def to_flat(self, device=None, compute_dtype=torch.bfloat16):
        """Re-home every variable into one FlatParams store (fp32 master + grad views) for the
        fused flat optimizers and the bucketed all-reduce; returns the FlatParams."""
        from ..train.flat import FlatParams, ParamSpec
        named = self.named_variables()
        dev = torch.device(device) if device is not None else (named[0][1].device if named else "cpu")
        specs = []
        for name, t in reversed(named):  # backward-completion order
            specs.append(ParamSpec(name, tuple(t.shape), None, weight_decay=t.dim() > 1, trainable=t.requires_grad))
        fp = FlatParams(specs, dev, compute_dtype=compute_dtype if dev.type == "cuda" else None)
        with torch.no_grad():
            for name, t in named:
                fp.var[name].copy_(t.detach().to(dev))
        fp.refresh_compute()
        # point the module parameters at the flat views (fp32 master; grads land in the flat buffer)
        fp._ttd_vars = {}
        for m in self.modules():
            if isinstance(m, Layer):
                for full, key in m._var_names:
                    p = torch.nn.Parameter(fp.var[full], requires_grad=getattr(m, key).requires_grad)
                    p.grad = fp.g[full]
                    p._ttd_flat, p._ttd_name = fp, full  # GradientTape / apply_gradients routing
                    fp._ttd_vars[full] = p
                    setattr(m, key, p)
        self.params = fp
        return fp


class Dense(Layer):
    """tf.layers.Dense: kernel [in, units] (default glorot_uniform), bias zeros."""
    _default_name = "dense"

    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None, name=None, trainable=True):
        super().__init__(name, trainable)
        self.units = int(units)
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer, self.bias_initializer = kernel_initializer, bias_initializer
        self.kernel_regularizer, self.bias_regularizer = kernel_regularizer, bias_regularizer

    def build(self, input_shape):
        self.add_weight("kernel", (input_shape[-1], self.units), self.kernel_initializer, self.kernel_regularizer)
        if self.use_bias:
            self.add_weight("bias", (self.units,), self.bias_initializer, self.bias_regularizer)
        else:
            self.bias = None
        super().build(input_shape)

    def call(self, x, **kw):
        act = self.activation
        if isinstance(act, str) and act in ("relu", "gelu", "tanh", "elu", "linear"):
            return N.dense(x, self.kernel, self.bias, activation=None if act == "linear" else act)
        y = N.dense(x, self.kernel, self.bias)
        f = _act(act)
        return f(y) if f is not None else y


class Dropout(Layer):
    _default_name = "dropout"

    def __init__(self, rate=0.5, name=None):
        super().__init__(name)
        self.rate = float(rate)

    def call(self, x, training=True, **kw):
        return N.dropout(x, self.rate, training=training)


class Activation(Layer):
    _default_name = "activation"

    def __init__(self, activation, name=None):
        super().__init__(name)
        self.fn = _act(activation)

    def call(self, x, **kw):
        return self.fn(x) if self.fn is not None else x


class Flatten(Layer):
    _default_name = "flatten"

    def call(self, x, **kw):
        return x.reshape(x.shape[0], -1)


class Conv2D(Layer):
    """NHWC conv; kernel [R, S, C, K] (TF layout)."""
    _default_name = "conv2d"

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="same", activation=None, use_bias=True,
                 kernel_initializer="glorot_uniform", bias_initializer="zeros", kernel_regularizer=None, name=None):
        super().__init__(name)
        ks = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.filters, self.kernel_size = int(filters), ks
        self.strides = (strides, strides) if isinstance(strides, int) else tuple(strides)
        self.padding = padding.upper()
        self.activation = _act(activation)
        self.use_bias = use_bias
        self.kernel_initializer, self.bias_initializer = kernel_initializer, bias_initializer
        self.kernel_regularizer = kernel_regularizer

    def build(self, input_shape):
        self.add_weight("kernel", self.kernel_size + (input_shape[-1], self.filters), self.kernel_initializer,
                        self.kernel_regularizer)
        if self.use_bias:
            self.add_weight("bias", (self.filters,), self.bias_initializer)
        else:
            self.bias = None
        super().build(input_shape)

    def call(self, x, **kw):
        y = N.conv2d(x, self.kernel, self.strides, self.padding)
        if self.bias is not None:
            y = N.bias_add(y, self.bias)
        return self.activation(y) if self.activation is not None else y


class BatchNormalization(Layer):
    """Over the last (channel) axis; gamma/beta trainable, moving_mean/variance not."""
    _default_name = "batch_normalization"

    def __init__(self, momentum=0.99, epsilon=1e-3, name=None):
        super().__init__(name)
        self.momentum, self.epsilon = float(momentum), float(epsilon)

    def build(self, input_shape):
        C = input_shape[-1]
        self.add_weight("gamma", (C,), "ones")
        self.add_weight("beta", (C,), "zeros")
        self.add_weight("moving_mean", (C,), "zeros", trainable=False)
        self.add_weight("moving_variance", (C,), "ones", trainable=False)
        super().build(input_shape)

    def call(self, x, training=True, **kw):
        return N.batch_norm(x, self.gamma, self.beta, self.moving_mean, self.moving_variance, training,
                            self.momentum, self.epsilon)


class LayerNormalization(Layer):
    _default_name = "layer_normalization"

    def __init__(self, epsilon=1e-12, name=None):
        super().__init__(name)
        self.epsilon = float(epsilon)

    def build(self, input_shape):
        self.add_weight("gamma", (input_shape[-1],), "ones")
        self.add_weight("beta", (input_shape[-1],), "zeros")
        super().build(input_shape)

    def call(self, x, **kw):
        return N.layer_norm(x, self.gamma, self.beta, self.epsilon)


class Embedding(Layer):
    _default_name = "embedding"

    def __init__(self, input_dim, output_dim, embeddings_initializer=None, name=None):
        super().__init__(name)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)
        self.init = embeddings_initializer or I.TruncatedNormal(stddev=0.02)

    def build(self, input_shape):
        self.add_weight("embeddings", (self.input_dim, self.output_dim), self.init)
        super().build(input_shape)

    def call(self, ids, **kw):
        return N.embedding_lookup(self.embeddings, ids)


class MultiHeadAttention(Layer):
    """Self-attention with fused QKV projection (head size 64 on the GPU flash kernels)."""
    _default_name = "multi_head_attention"

    def __init__(self, num_heads, key_dim=64, dropout=0.0, name=None):
        super().__init__(name)
        self.num_heads, self.key_dim, self.dropout = int(num_heads), int(key_dim), float(dropout)

    def build(self, input_shape):
        D = input_shape[-1]
        inner = self.num_heads * self.key_dim
        init = I.TruncatedNormal(stddev=0.02)
        self.add_weight("qkv/kernel", (D, 3 * inner), init, attr="qkv_kernel")
        self.add_weight("qkv/bias", (3 * inner,), "zeros", attr="qkv_bias")
        self.add_weight("output/kernel", (inner, D), init, attr="out_kernel")
        self.add_weight("output/bias", (D,), "zeros", attr="out_bias")
        super().build(input_shape)

    def call(self, x, seqlen=None, training=True, **kw):
        inner = self.num_heads * self.key_dim
        qkv = N.dense(x, self.qkv_kernel, self.qkv_bias)
        q, k, v = qkv[..., :inner], qkv[..., inner:2 * inner], qkv[..., 2 * inner:]
        a = N.attention(q.contiguous(), k.contiguous(), v.contiguous(), self.num_heads,
                        self.dropout if training else 0.0, seqlen=seqlen)
        return N.dense(a, self.out_kernel, self.out_bias)


class MaxPooling2D(Layer):
    _default_name = "max_pooling2d"

    def __init__(self, pool_size=3, strides=2, padding=1, name=None):
        super().__init__(name)
        self.k, self.s, self.p = pool_size, strides, padding

    def call(self, x, **kw):
        return N.max_pool2d(x, self.k, self.s, self.p)


class GlobalAveragePooling2D(Layer):
    _default_name = "global_average_pooling2d"

    def call(self, x, **kw):
        return N.global_avg_pool(x)


class Sequential(Layer):
    _default_name = "sequential"

    def __init__(self, layers: Sequence[Layer] = (), name=None):
        super().__init__(name)
        self.layer_list = torch.nn.ModuleList(list(layers))

    def add(self, layer: Layer):
        self.layer_list.append(layer)

    def call(self, x, training=True, **kw):
        for l in self.layer_list:
            x = l(x, training=training) if isinstance(l, (Dropout, BatchNormalization, Sequential)) else l(x)
        return x


# ------------------------------------------------------------------ tf.layers functional API
def dense(inputs, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
          bias_initializer="zeros", kernel_regularizer=None, name=None, trainable=True):
    """tf.layers.dense: builds a Dense layer, registers its variables / regularization
    losses in the default graph's collections and applies it."""
    from ..train import graph as Gr
    layer = Dense(units, activation, use_bias, kernel_initializer, bias_initializer, kernel_regularizer, name=name,
                  trainable=trainable)
    y = layer(inputs)
    for full, t in layer.named_variables():
        Gr.add_to_collection("variables", (full, t))
        if t.requires_grad:
            Gr.add_to_collection("trainable_variables", (full, t))
    for l in layer.losses:
        Gr.add_to_collection("regularization_losses", l)
    Gr.add_to_collection("layers", layer)
    return y


def dropout(inputs, rate=0.5, training=False, name=None):
    return N.dropout(inputs, rate, training=training)


def batch_normalization(inputs, training=False, momentum=0.99, epsilon=1e-3, name=None):
    layer = BatchNormalization(momentum, epsilon, name=name)
    return layer(inputs, training=training)
