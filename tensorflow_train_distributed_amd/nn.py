"""`ttd.nn` — functional ops with autograd (tf.nn-shaped), SURVEY.md §2.2 T22-T25/T30 and
§7.5 ("mitrain.nn.*").

Every op runs a hand-written gfx950 kernel when its inputs live on the GPU (a
torch.autograd.Function whose backward is also a HIP kernel) and a plain fp32 PyTorch
implementation on CPU tensors (the "soft placement" CPU fallback of
ConfigProto(allow_soft_placement=True), reference distribute_training.py:201-202). There is no
silent GPU fallback to torch compute: a GPU input the kernels cannot take (dtype other than
fp32/bf16, an unsupported attention head size) raises InvalidArgumentError.

GPU precision: fp32 inputs stay fp32 for dense/matmul (exact-fp32 MFMA, gemm_f32.hip),
normalisation, pooling, embeddings, activations and losses (nn_generic.hip / elementwise.hip /
xent.hip); bf16 inputs use the bf16 MFMA engines. conv2d and attention compute in bf16 (fp32
accumulation) for either input dtype.

    ttd.nn.elu(x); ttd.nn.dropout(x, rate=0.01)
    ttd.nn.sparse_softmax_cross_entropy_with_logits(labels=y, logits=z)
    ttd.nn.in_top_k(z, y, 1); ttd.nn.layer_norm(x, gamma, beta)
    ttd.nn.dense(x, kernel, bias, activation="relu")      # kernel [in, out] (TF layout)
    ttd.nn.conv2d(x, kernel, strides, padding)            # NHWC, kernel [R, S, C, K]
    ttd.nn.attention(q, k, v, num_heads, dropout_rate)    # [B, S, H*64] token-major
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from .utils.errors import InvalidArgumentError

_ACT_CODES = {None: 0, "linear": 0, "relu": 1, "gelu": 2, "tanh": 3}  # GEMM epilogue codes
_EW_ACT = {None: 0, "linear": 0, "relu": 1, "gelu": 2, "elu": 3}       # elementwise kernel codes


def _on_gpu(*ts):
    if not (all(t is None or t.is_cuda for t in ts) and any(t is not None for t in ts)):
        return False
    for t in ts:
        if t is not None and t.is_floating_point() and t.dtype not in (torch.float32, torch.bfloat16):
            raise InvalidArgumentError("ttd.nn GPU kernels take float32/bfloat16 tensors, got %s" % t.dtype)
    return True


def _f32(t):
    """fp32 contiguous view/copy of a (small) parameter vector, or None."""
    return None if t is None else t.float().contiguous()


class _Rng:
    """Host-side Philox (seed, offset) stream for eager-mode dropout."""
    seed = 0x5EED
    offset = 0

    @classmethod
    def next(cls, n):
        off = cls.offset
        cls.offset += (n + 3) // 4 + 1
        return cls.seed, off


def set_random_seed(seed: int):
    _Rng.seed = int(seed)
    _Rng.offset = 0
    torch.manual_seed(seed)


# ------------------------------------------------------------------ activations
def _act_ref(x, act):
    if act in (None, "linear"):
        return x
    if act == "relu":
        return F.relu(x)
    if act == "elu":
        return F.elu(x)
    if act == "gelu":
        return F.gelu(x, approximate="tanh")
    if act == "tanh":
        return torch.tanh(x)
    raise ValueError("unknown activation %r" % act)


class _BiasActDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act, rate):
        from .ops import kernels as K
        xb = x.contiguous()
        seed, off = _Rng.next(xb.numel()) if rate > 0 else (0, 0)
        code = _EW_ACT[act]
        b = bias.float().contiguous() if bias is not None else None
        y = K.bias_act_dropout(xb, b, act=code, rate=rate, seed=seed, offset=off)
        ctx.save_for_backward(xb, b)
        ctx.cfg = (code, rate, seed, off, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        xb, b = ctx.saved_tensors
        code, rate, seed, off, has_b = ctx.cfg
        dz = K.bias_act_dropout_bwd(dy.contiguous().to(xb.dtype), xb, b, act=code, rate=rate, seed=seed, offset=off)
        db = None
        if has_b:
            db = K.colsum(dz.reshape(-1, dz.shape[-1]))
        return dz, db, None, None


def _bias_act_dropout(x, bias, act, rate):
    if _on_gpu(x) and x.dtype in (torch.float32, torch.bfloat16) and (act in _EW_ACT):
        return _BiasActDropout.apply(x, bias, act, float(rate))
    y = x + bias if bias is not None else x
    y = _act_ref(y, act)
    if rate > 0:
        y = F.dropout(y, rate, training=True)
    return y


def elu(x):
    return _bias_act_dropout(x, None, "elu", 0.0)


def relu(x):
    return _bias_act_dropout(x, None, "relu", 0.0)


def gelu(x):
    return _bias_act_dropout(x, None, "gelu", 0.0)


class _Unary(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, op):
        from .ops import kernels as K
        y = K.unary(x.contiguous(), op)
        ctx.save_for_backward(y)
        ctx.op = op
        return y

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        (y,) = ctx.saved_tensors
        return K.unary_bwd(dy.contiguous().to(y.dtype), y, ctx.op), None


def tanh(x):
    if _on_gpu(x):
        return _Unary.apply(x, 0)
    return torch.tanh(x)


def sigmoid(x):
    if _on_gpu(x):
        return _Unary.apply(x, 1)
    return torch.sigmoid(x)


def bias_add(x, bias):
    return _bias_act_dropout(x, bias, None, 0.0)


def dropout(x, rate: float = 0.5, training: bool = True):
    """tf.nn.dropout / tf.layers.dropout: keep with probability 1-rate, scale by 1/(1-rate)."""
    if not training or rate <= 0:
        return x
    return _bias_act_dropout(x, None, None, rate)


# ------------------------------------------------------------------ dense (GEMM + epilogue)
class _Dense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, bias, act):
        from .ops import gemm as G
        shp = x.shape
        xb = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        wb = kernel.to(torch.bfloat16).contiguous()          # [in, out]
        b = bias.float().contiguous() if bias is not None else None
        code = _ACT_CODES.get(act, None)
        pre = None
        if act in ("gelu", "tanh", "relu"):
            pre = torch.empty((xb.shape[0], wb.shape[1]), dtype=torch.bfloat16, device=x.device)
        y = G.gemm(xb, wb, bias=b, act=code or 0, aux=pre)
        if act == "elu":
            from .ops import kernels as K
            pre = y
            y = K.bias_act_dropout(y, None, act=_EW_ACT["elu"])
        ctx.save_for_backward(xb, wb, pre, y if act == "tanh" else None)
        ctx.cfg = (act, bias is not None, shp, x.dtype, kernel.dtype)
        return y.reshape(*shp[:-1], wb.shape[1]).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        from .ops import gemm as G
        from .ops import kernels as K
        from .ops import transformer as T
        xb, wb, pre, y = ctx.saved_tensors
        act, has_b, shp, xdt, wdt = ctx.cfg
        d = dy.reshape(-1, wb.shape[1]).to(torch.bfloat16).contiguous()
        if act == "gelu":
            d = T.dact(d, pre, 0)
        elif act == "tanh":
            d = T.dact(d, y, 1)
        elif act in ("relu", "elu"):
            d = K.bias_act_dropout_bwd(d, pre, None, act=_EW_ACT[act])
        dw = torch.empty(wb.shape, dtype=torch.float32, device=d.device)
        G.gemm(xb, d, trans_a=True, out=dw, splits=G.gemm_wgrad_splits(wb.shape[0], wb.shape[1], xb.shape[0]))
        db = K.colsum(d) if has_b else None
        dx = G.gemm(d, wb, trans_b=True) if ctx.needs_input_grad[0] else None
        return (dx.reshape(shp).to(xdt) if dx is not None else None), dw.to(wdt), db, None


class _DenseF32(torch.autograd.Function):
    """Exact-fp32 dense layer: f32-MFMA GEMMs (gemm_f32.hip) + fp32 element-wise kernels."""

    @staticmethod
    def forward(ctx, x, kernel, bias, act):
        from .ops import gemm as G
        from .ops import kernels as K
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        w = kernel.contiguous()
        y = G.gemm_f32(x2, w, bias=_f32(bias))
        pre = None
        if act in ("relu", "gelu", "elu"):
            pre = y
            y = K.bias_act_dropout(y, None, act=_EW_ACT[act])
        elif act == "tanh":
            y = K.unary(y, K.UNARY_TANH)
        elif act not in (None, "linear"):
            raise InvalidArgumentError("unknown dense activation %r" % (act,))
        ctx.save_for_backward(x2, w, pre, y if act == "tanh" else None)
        ctx.cfg = (act, bias is not None, shp)
        return y.reshape(*shp[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        from .ops import gemm as G
        from .ops import kernels as K
        x2, w, pre, y = ctx.saved_tensors
        act, has_b, shp = ctx.cfg
        d = dy.reshape(-1, w.shape[1]).contiguous()
        if act in ("relu", "gelu", "elu"):
            d = K.bias_act_dropout_bwd(d, pre, None, act=_EW_ACT[act])
        elif act == "tanh":
            d = K.unary_bwd(d, y, K.UNARY_TANH)
        dw = G.gemm_f32(x2, d, trans_a=True) if ctx.needs_input_grad[1] else None
        db = K.colsum(d) if has_b and ctx.needs_input_grad[2] else None
        dx = G.gemm_f32(d, w, trans_b=True).reshape(shp) if ctx.needs_input_grad[0] else None
        return dx, dw, db, None


def dense(x, kernel, bias=None, activation=None):
    """y = activation(x @ kernel + bias); kernel [in, out] (tf.layers.dense layout)."""
    if _on_gpu(x, kernel):
        if x.dtype == torch.float32 and kernel.dtype == torch.float32:
            return _DenseF32.apply(x, kernel, bias, activation)
        return _Dense.apply(x, kernel, bias, activation)
    y = x @ kernel
    if bias is not None:
        y = y + bias
    return _act_ref(y, activation)


class _MatMul(torch.autograd.Function):
    """[..., M, K] @ [..., K, N] with identical leading (batch) shapes: ONE strided-batched GEMM
    launch per product (ops.gemm.gemm_batched: batch index on the grid), forward and backward.
    fp32 operands stay exact fp32 (f32 MFMA); otherwise bf16 operands with fp32 accumulation."""

    @staticmethod
    def _bmm(a, b, ta=False, tb=False):
        from .ops import gemm as G
        if a.dtype == torch.float32 and b.dtype == torch.float32:
            return G.gemm_batched(a, b, trans_a=ta, trans_b=tb)
        return G.gemm_batched(a.to(torch.bfloat16), b.to(torch.bfloat16), trans_a=ta, trans_b=tb,
                              out_dtype=torch.float32)

    @staticmethod
    def forward(ctx, a, b):
        a3 = a.reshape(-1, a.shape[-2], a.shape[-1]).contiguous()
        b3 = b.reshape(-1, b.shape[-2], b.shape[-1]).contiguous()
        out = _MatMul._bmm(a3, b3)
        ctx.save_for_backward(a3, b3)
        ctx.shapes = (a.shape, b.shape, a.dtype, b.dtype)
        return out.reshape(*a.shape[:-1], b.shape[-1]).to(a.dtype)

    @staticmethod
    def backward(ctx, dy):
        a3, b3 = ctx.saved_tensors
        sa, sb, da_t, db_t = ctx.shapes
        d3 = dy.reshape(a3.shape[0], a3.shape[1], b3.shape[2]).contiguous()
        if d3.dtype != a3.dtype and a3.dtype == torch.float32:
            d3 = d3.float()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _MatMul._bmm(d3, b3, tb=True).reshape(sa).to(da_t)
        if ctx.needs_input_grad[1]:
            db = _MatMul._bmm(a3, d3, ta=True).reshape(sb).to(db_t)
        return da, db


def matmul(a, b, transpose_a=False, transpose_b=False):
    a2 = a.transpose(-1, -2) if transpose_a else a
    b2 = b.transpose(-1, -2) if transpose_b else b
    if _on_gpu(a, b):
        if a2.dim() == 2 and b2.dim() == 2:
            return dense(a2.contiguous(), b2.contiguous())
        if a2.shape[:-2] != b2.shape[:-2]:
            raise InvalidArgumentError("ttd.nn.matmul on GPU needs equal batch shapes, got %s and %s"
                                       % (tuple(a2.shape), tuple(b2.shape)))
        return _MatMul.apply(a2, b2)
    return a2 @ b2


# ------------------------------------------------------------------ losses / metrics
class _SparseXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        from .ops import kernels as K
        z = logits.contiguous()
        if z.dtype not in (torch.float32, torch.bfloat16):
            z = z.float()
        _, dl, rows, _ = K.sparse_xent(z, labels.contiguous(), grad_scale=1.0, want_rows=True)
        ctx.save_for_backward(dl)
        ctx.dt = logits.dtype
        return rows

    @staticmethod
    def backward(ctx, g):
        from .ops import kernels as K
        (dl,) = ctx.saved_tensors
        d = K.row_scale(dl, g.float().contiguous())
        return (d if d.dtype == ctx.dt else d.to(ctx.dt)), None


def sparse_softmax_cross_entropy_with_logits(labels=None, logits=None):
    """Per-example loss [N] (tf.nn.sparse_softmax_cross_entropy_with_logits)."""
    if _on_gpu(logits) and logits.dim() == 2:
        return _SparseXent.apply(logits, labels)
    return F.cross_entropy(logits.float(), labels.long(), reduction="none")


def in_top_k(predictions, targets, k: int = 1):
    """TF semantics: correct iff fewer than k classes have a STRICTLY greater logit than the
    target's; a non-finite target logit is never correct."""
    if _on_gpu(predictions) and predictions.dim() == 2:
        from .ops import kernels as K
        t = targets if targets.dtype in (torch.int32, torch.int64) else targets.long()
        return K.in_top_k(predictions.contiguous(), t.contiguous(), int(k)).bool()
    z = predictions.float()
    t = targets.long()
    zt = z.gather(1, t[:, None])
    greater = (z > zt).sum(1)
    return (greater < k) & torch.isfinite(zt[:, 0])


class _Mean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        from .ops import kernels as K
        xc = x.contiguous()
        ctx.shape, ctx.dt = x.shape, x.dtype
        return K.sum_all(xc, 1.0 / max(1, xc.numel()))

    @staticmethod
    def backward(ctx, g):
        from .ops import kernels as K
        n = 1
        for d in ctx.shape:
            n *= d
        return K.fill_scaled(ctx.shape, g.to(ctx.dt).contiguous(), 1.0 / max(1, n), ctx.dt)


def reduce_mean(x):
    """tf.reduce_mean over all elements (0-d result)."""
    if _on_gpu(x):
        return _Mean.apply(x)
    return x.mean()


def l1_loss(w):
    return w.abs().sum()


def l2_loss(w):
    return 0.5 * (w * w).sum()


# ------------------------------------------------------------------ normalisation
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        from .ops import transformer as T
        shp = x.shape
        xb = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        g, b = gamma.float().contiguous(), beta.float().contiguous()
        y, s, mean, rstd = T.layernorm_fwd(xb, g, b, eps=eps)
        ctx.save_for_backward(s, mean, rstd, g)
        ctx.cfg = (shp, x.dtype, gamma.dtype)
        return y.reshape(shp).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        from .ops import transformer as T
        s, mean, rstd, g = ctx.saved_tensors
        shp, xdt, gdt = ctx.cfg
        H = shp[-1]
        dg = torch.empty(H, dtype=torch.float32, device=dy.device)
        db = torch.empty(H, dtype=torch.float32, device=dy.device)
        ds, _ = T.layernorm_bwd(dy.reshape(-1, H).to(torch.bfloat16).contiguous(), s, mean, rstd, g, dg, db)
        return ds.reshape(shp).to(xdt), dg.to(gdt), db.to(gdt), None


class _LayerNormGeneric(torch.autograd.Function):
    """Any width, fp32 or bf16 (nn_generic.hip): wave-per-row statistics, deterministic
    column-partial dgamma/dbeta."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        from .ops import kernels as K
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        g, b = _f32(gamma), _f32(beta)
        y, mean, rstd = K.ln_generic_fwd(x2, g, b, eps)
        ctx.save_for_backward(x2, g, mean, rstd)
        ctx.cfg = (shp, gamma.dtype, beta.dtype)
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        x2, g, mean, rstd = ctx.saved_tensors
        shp, gdt, bdt = ctx.cfg
        H = shp[-1]
        dg = torch.empty(H, dtype=torch.float32, device=dy.device)
        db = torch.empty(H, dtype=torch.float32, device=dy.device)
        d2 = dy.reshape(-1, H).contiguous().to(x2.dtype)
        dx = K.ln_generic_bwd(d2, x2, g, mean, rstd, dg, db, want_dx=ctx.needs_input_grad[0])
        return (dx.reshape(shp) if dx is not None else None), dg.to(gdt), db.to(bdt), None


_LN_FAST_WIDTHS = (512, 1024, 1536, 2048, 4096)


def layer_norm(x, gamma, beta, eps: float = 1e-12):
    if _on_gpu(x):
        if x.dtype == torch.bfloat16 and x.shape[-1] in _LN_FAST_WIDTHS:
            return _LayerNorm.apply(x, gamma, beta, float(eps))   # vectorised BERT kernel
        return _LayerNormGeneric.apply(x, gamma, beta, float(eps))
    return F.layer_norm(x, (x.shape[-1],), gamma, beta, eps)


class _BatchNorm(torch.autograd.Function):
    """NHWC BatchNorm over all but the channel axis on the GPU: column statistics
    (nn_generic.hip) folded by the ResNet engine's finalize kernel (batchnorm.hip: mean/rstd,
    scale/shift, TF moving-average update with the unbiased variance), one affine pass; the
    backward is (sum g, sum g*x) -> dgamma/dbeta + coefficients -> one affine pass."""

    @staticmethod
    def forward(ctx, x, gamma, beta, moving_mean, moving_variance, training, momentum, eps):
        from .ops import kernels as K
        C = x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        M = x2.shape[0]
        g, b = _f32(gamma), _f32(beta)
        if training:
            part, T = K.col_stats(x2, mode=0)
            st = K.BNState(C, x.device)
            for t in (moving_mean, moving_variance):
                if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda):
                    raise InvalidArgumentError("batch_norm moving statistics must be contiguous fp32 GPU tensors")
            K.bn_fwd_stats(part, T, M, g, b, eps, momentum, moving_mean, moving_variance, st)
            y = K.col_affine(x2, st.scale, c2=st.shift)
            ctx.save_for_backward(x2, g, st.mean, st.rstd, None)
        else:
            if moving_mean is None or moving_variance is None:
                raise InvalidArgumentError("batch_norm(training=False) needs moving_mean/moving_variance")
            mm = moving_mean.float().contiguous()
            scale, shift, rstd = K.bn_infer_coef(mm, moving_variance.float().contiguous(), g, b, eps)
            y = K.col_affine(x2, scale, c2=shift)
            ctx.save_for_backward(x2, g, mm, rstd, scale)
        ctx.cfg = (training, x.shape, None if gamma is None else gamma.dtype, None if beta is None else beta.dtype)
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        x2, g, mean, rstd, scale = ctx.saved_tensors
        training, shp, gdt, bdt = ctx.cfg
        M, C = x2.shape
        d2 = dy.reshape(-1, C).contiguous().to(x2.dtype)
        dgamma = torch.empty(C, dtype=torch.float32, device=dy.device)
        dbeta = torch.empty(C, dtype=torch.float32, device=dy.device)
        part, T = K.col_stats(d2, x2, mode=1)
        if training:
            st = K.BNState(C, dy.device)
            st.mean, st.rstd = mean, rstd
            coef = K.bn_backward_coef(M, C, g, st, dgamma, dbeta, part, T, device=dy.device)
            dx = K.col_affine(d2, coef[0], b=x2, c1=coef[1], c2=coef[2])
        else:
            K.bn_infer_bwd(part, T, mean, rstd, dgamma, dbeta)
            dx = K.col_affine(d2, scale)
        dg = dgamma.to(gdt) if gdt is not None else None
        db = dbeta.to(bdt) if bdt is not None else None
        return dx.reshape(shp), dg, db, None, None, None, None, None


def batch_norm(x, gamma, beta, moving_mean=None, moving_variance=None, training=True, momentum=0.99,
               eps=1e-3):
    """NHWC batch normalisation over all but the last axis (tf.layers.batch_normalization);
    updates the moving statistics in place when training."""
    if _on_gpu(x):
        return _BatchNorm.apply(x, gamma, beta, moving_mean, moving_variance, bool(training), float(momentum),
                                float(eps))
    C = x.shape[-1]
    x2 = x.reshape(-1, C)
    if training:
        mean = x2.float().mean(0)
        var = x2.float().var(0, unbiased=False)
        if moving_mean is not None:
            with torch.no_grad():
                n = x2.shape[0]
                moving_mean.mul_(momentum).add_((1 - momentum) * mean.detach())
                moving_variance.mul_(momentum).add_((1 - momentum) * var.detach() * n / max(1, n - 1))
    else:
        mean, var = moving_mean, moving_variance
    y = (x2.float() - mean) * torch.rsqrt(var + eps)
    if gamma is not None:
        y = y * gamma
    if beta is not None:
        y = y + beta
    return y.reshape(x.shape).to(x.dtype)


# ------------------------------------------------------------------ convolution
class _Conv2D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, stride, padding):
        from .ops import gemm as G
        xb = x.to(torch.bfloat16).contiguous()
        wk = kernel.permute(3, 0, 1, 2).to(torch.bfloat16).contiguous()  # [R,S,C,K] -> [K,R,S,C]
        y = G.conv_fwd(xb, wk, stride, padding)
        ctx.save_for_backward(xb, wk)
        ctx.cfg = (stride, padding, x.dtype, kernel.dtype)
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        from .ops import gemm as G
        from .ops import kernels as K
        xb, wk = ctx.saved_tensors
        stride, padding, xdt, wdt = ctx.cfg
        d = dy.to(torch.bfloat16).contiguous()
        dw = G.conv_wgrad(xb, d, tuple(wk.shape), stride, padding)  # [K,R,S,C] fp32
        dx = None
        if ctx.needs_input_grad[0]:
            dx = G.conv_dgrad(d, K.krsc_to_crsk(wk), xb.shape, stride, padding).to(xdt)
        return dx, dw.permute(1, 2, 3, 0).to(wdt), None, None


def _same_pad(size, k, s):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def conv2d(x, kernel, strides=(1, 1), padding="SAME"):
    """NHWC conv; kernel [R, S, C, K] (TF layout). padding 'SAME' | 'VALID' | (ph, pw)."""
    if isinstance(strides, int):
        strides = (strides, strides)
    R, S = kernel.shape[0], kernel.shape[1]
    if isinstance(padding, str):
        if padding.upper() == "VALID":
            pads = (0, 0)
            extra = None
        else:
            (ph0, ph1), (pw0, pw1) = _same_pad(x.shape[1], R, strides[0]), _same_pad(x.shape[2], S, strides[1])
            pads = (ph0, pw0)
            extra = (ph1 - ph0, pw1 - pw0)
            if extra != (0, 0):  # asymmetric SAME padding: pad explicitly (right/bottom)
                x = F.pad(x, (0, 0, 0, pw1 - pw0, 0, ph1 - ph0))
    else:
        pads = tuple(padding)
    if _on_gpu(x):
        C, K = x.shape[-1], kernel.shape[-1]
        Cp, Kp = -(-C // 8) * 8, -(-K // 8) * 8
        if Cp != C or Kp != K:  # the implicit-GEMM kernels want channel counts % 8: zero-pad
            x = F.pad(x, (0, Cp - C))
            kernel = F.pad(kernel, (0, Kp - K, 0, Cp - C))
        y = _Conv2D.apply(x, kernel, tuple(strides), pads)
        return y[..., :K] if Kp != K else y
    y = F.conv2d(x.permute(0, 3, 1, 2), kernel.permute(3, 2, 0, 1), stride=strides, padding=pads)
    return y.permute(0, 2, 3, 1)


def _pair(v):
    if isinstance(v, int):
        return v, v
    v = tuple(v)
    if len(v) == 4:  # TF NHWC [1, kh, kw, 1]
        return v[1], v[2]
    return v[0], v[1]


def _pool_geometry(H, W, k, s, padding):
    """(ph, pw, P, Q): TF 'SAME' / 'VALID' (SAME pads the extra row/column at the bottom/right)
    or explicit symmetric padding (int / pair)."""
    (R, S), (sh, sw) = k, s
    if isinstance(padding, str):
        if padding.upper() == "VALID":
            return 0, 0, (H - R) // sh + 1, (W - S) // sw + 1
        P, Q = -(-H // sh), -(-W // sw)
        return (max((P - 1) * sh + R - H, 0) // 2, max((Q - 1) * sw + S - W, 0) // 2, P, Q)
    ph, pw = _pair(padding)
    return ph, pw, (H + 2 * ph - R) // sh + 1, (W + 2 * pw - S) // sw + 1


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, geo):
        from .ops import kernels as K
        xc = x.contiguous()
        (R, S), (sh, sw) = k, s
        ph, pw, P, Q = geo
        C = x.shape[-1]
        fast = (x.dtype == torch.bfloat16 and C % 8 == 0 and R == S and sh == sw and ph == pw
                and P == K.pool_out(x.shape[1], R, sh, ph) and Q == K.pool_out(x.shape[2], S, sw, pw))
        if fast:
            y, arg = K.maxpool_fwd(xc, R, sh, ph)
        else:
            y, arg = K.maxpool_generic_fwd(xc, R, S, sh, sw, ph, pw, P, Q)
        ctx.save_for_backward(arg)
        ctx.cfg = (fast, tuple(x.shape), k, s, geo)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        (arg,) = ctx.saved_tensors
        fast, xs, (R, S), (sh, sw), (ph, pw, _, _) = ctx.cfg
        d = dy.contiguous()
        if fast:
            return K.maxpool_bwd(d, arg, xs, R, sh, ph), None, None, None
        return K.maxpool_generic_bwd(d, arg, xs, R, S, sh, sw, ph, pw), None, None, None


def max_pool2d(x, ksize=3, strides=2, padding=1):
    """NHWC max pooling; ksize/strides int, pair or TF [1, k, k, 1]; padding 'SAME' | 'VALID'
    | int / pair (explicit, symmetric)."""
    k, s = _pair(ksize), _pair(strides)
    ph, pw, P, Q = _pool_geometry(x.shape[1], x.shape[2], k, s, padding)
    if _on_gpu(x):
        return _MaxPool.apply(x, k, s, (ph, pw, P, Q))
    # explicit -inf padding (covers TF SAME's extra bottom/right row) then an unpadded pool
    eh = max((P - 1) * s[0] + k[0] - x.shape[1] - 2 * ph, 0)
    ew = max((Q - 1) * s[1] + k[1] - x.shape[2] - 2 * pw, 0)
    xp = F.pad(x.permute(0, 3, 1, 2), (pw, pw + ew, ph, ph + eh), value=float("-inf"))
    y = F.max_pool2d(xp, k, s, 0)
    return y[:, :, :P, :Q].permute(0, 2, 3, 1)


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        from .ops import kernels as K
        xc = x.contiguous()
        fast = x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0
        ctx.cfg = (fast, tuple(x.shape))
        return K.avgpool_fwd(xc) if fast else K.gap_fwd(xc)

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        fast, xs = ctx.cfg
        d = dy.contiguous()
        return K.avgpool_bwd(d, xs) if fast else K.gap_bwd(d, xs)


def global_avg_pool(x):
    if _on_gpu(x):
        return _GlobalAvgPool.apply(x)
    return x.mean(dim=(1, 2))


# ------------------------------------------------------------------ attention
class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, num_heads, rate, seqlen, site):
        from .ops import transformer as T
        B, S, D = q.shape
        q2, k2, v2 = [t.reshape(B * S, D).to(torch.bfloat16).contiguous() for t in (q, k, v)]
        o = torch.empty_like(q2)
        lse = torch.empty((B * num_heads, S), dtype=torch.float32, device=q.device)
        rng = None
        if rate > 0:
            rng = T.RngState(_Rng.seed, q.device)
            rng.t[1] = _Rng.offset
            _Rng.offset += 1
        T.attention_fwd(q2, k2, v2, o, lse, B, num_heads, S, seqlen=seqlen, p_drop=rate, rng=rng, site=site)
        ctx.save_for_backward(q2, k2, v2, o, lse, seqlen)
        ctx.cfg = (B, S, D, num_heads, rate, rng, site, q.dtype)
        return o.reshape(B, S, D).to(q.dtype)

    @staticmethod
    def backward(ctx, do):
        from .ops import transformer as T
        q2, k2, v2, o, lse, seqlen = ctx.saved_tensors
        B, S, D, nh, rate, rng, site, dt = ctx.cfg
        d2 = do.reshape(B * S, D).to(torch.bfloat16).contiguous()
        dq, dk, dv = torch.empty_like(q2), torch.empty_like(k2), torch.empty_like(v2)
        T.attention_bwd(q2, k2, v2, o, d2, lse, dq, dk, dv, B, nh, S, seqlen=seqlen, p_drop=rate, rng=rng, site=site)
        return (dq.reshape(B, S, D).to(dt), dk.reshape(B, S, D).to(dt), dv.reshape(B, S, D).to(dt),
                None, None, None, None)


def attention(q, k, v, num_heads: int, dropout_rate: float = 0.0, seqlen=None, site: int = 0):
    """Multi-head scaled dot-product attention, token-major [B, S, num_heads*64] inputs,
    keys >= seqlen[b] masked. GPU: the flash kernels (head_dim 64, S % 128 == 0)."""
    B, S, D = q.shape
    hd = D // num_heads
    if _on_gpu(q, k, v):
        if hd != 64 or S % 128 != 0 or D % num_heads:
            raise InvalidArgumentError(
                "ttd.nn.attention on GPU runs the flash kernels for head_dim 64 and seq_len %% 128 == 0 "
                "(got head_dim %s, seq_len %d); pad the sequence (and mask it with seqlen) or use 64-wide heads"
                % (D / num_heads, S))
        sl = seqlen.to(torch.int32).contiguous() if seqlen is not None else None
        return _Attention.apply(q, k, v, num_heads, float(dropout_rate), sl, int(site))
    qh = q.reshape(B, S, num_heads, hd).transpose(1, 2)
    kh = k.reshape(B, S, num_heads, hd).transpose(1, 2)
    vh = v.reshape(B, S, num_heads, hd).transpose(1, 2)
    sc = qh @ kh.transpose(-1, -2) / math.sqrt(hd)
    if seqlen is not None:
        m = torch.arange(S, device=q.device)[None, :] < seqlen[:, None].long()
        sc = sc.masked_fill(~m[:, None, None, :], float("-inf"))
    p = sc.softmax(-1)
    if dropout_rate > 0:
        p = F.dropout(p, dropout_rate, training=True)
    return (p @ vh).transpose(1, 2).reshape(B, S, D)


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, ids):
        from .ops import kernels as K
        idc = ids.contiguous() if ids.dtype in (torch.int32, torch.int64) else ids.long().contiguous()
        ctx.save_for_backward(idc)
        ctx.cfg = (tuple(params.shape), params.dtype)
        return K.gather_generic(params.contiguous(), idc)

    @staticmethod
    def backward(ctx, dy):
        from .ops import kernels as K
        (idc,) = ctx.saved_tensors
        shp, dt = ctx.cfg
        dtable = K.zeros(shp, dtype=torch.float32, device=dy.device)
        K.scatter_add_generic(dy.reshape(-1, shp[1]).contiguous(), idc, dtable)
        return (dtable if dt == torch.float32 else dtable.to(dt)), None


def embedding_lookup(params, ids):
    """tf.nn.embedding_lookup (single table): rows of params [V, H] for ids of any shape; on GPU
    out-of-range ids give zero rows (tf.gather's GPU behaviour)."""
    if _on_gpu(params):
        return _Embedding.apply(params, ids)
    return F.embedding(ids.long(), params)
