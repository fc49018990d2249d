"""`ttd.nn` — functional ops with autograd (tf.nn-shaped), SURVEY.md §2.2 T22-T25/T30 and
§7.5 ("mitrain.nn.*").

Every op runs the hand-written gfx950 kernel when its inputs live on the GPU (bf16 compute,
fp32 accumulation, a torch.autograd.Function whose backward is also a HIP kernel) and a
plain fp32 PyTorch implementation on CPU tensors (the "soft placement" CPU fallback of
ConfigProto(allow_soft_placement=True), reference distribute_training.py:201-202).

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

_ACT_CODES = {None: 0, "linear": 0, "relu": 1, "gelu": 2, "tanh": 3}  # GEMM epilogue codes
_EW_ACT = {None: 0, "linear": 0, "relu": 1, "gelu": 2, "elu": 3}       # elementwise kernel codes


def _on_gpu(*ts):
    return all(t is None or t.is_cuda for t in ts) and any(t is not None for t in ts)


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


def tanh(x):
    return torch.tanh(x)


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


def dense(x, kernel, bias=None, activation=None):
    """y = activation(x @ kernel + bias); kernel [in, out] (tf.layers.dense layout)."""
    if _on_gpu(x):
        return _Dense.apply(x, kernel, bias, activation)
    y = x @ kernel
    if bias is not None:
        y = y + bias
    return _act_ref(y, activation)


def matmul(a, b, transpose_a=False, transpose_b=False):
    a2 = a.transpose(-1, -2) if transpose_a else a
    b2 = b.transpose(-1, -2) if transpose_b else b
    if _on_gpu(a, b) and a2.dim() == 2 and b2.dim() == 2:
        return dense(a2.contiguous(), b2.contiguous())
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
        (dl,) = ctx.saved_tensors
        return (dl.float() * g[:, None]).to(ctx.dt), None


def sparse_softmax_cross_entropy_with_logits(labels=None, logits=None):
    """Per-example loss [N] (tf.nn.sparse_softmax_cross_entropy_with_logits)."""
    if _on_gpu(logits) and logits.dim() == 2:
        return _SparseXent.apply(logits, labels)
    return F.cross_entropy(logits.float(), labels.long(), reduction="none")


def in_top_k(predictions, targets, k: int = 1):
    """TF semantics: correct iff fewer than k classes have a STRICTLY greater logit than the
    target's; a non-finite target logit is never correct."""
    z = predictions.float()
    t = targets.long()
    zt = z.gather(1, t[:, None])
    greater = (z > zt).sum(1)
    return (greater < k) & torch.isfinite(zt[:, 0])


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


def layer_norm(x, gamma, beta, eps: float = 1e-12):
    if _on_gpu(x) and x.shape[-1] in (512, 1024, 1536, 2048, 4096):
        return _LayerNorm.apply(x, gamma, beta, float(eps))
    return F.layer_norm(x, (x.shape[-1],), gamma, beta, eps)


def batch_norm(x, gamma, beta, moving_mean=None, moving_variance=None, training=True, momentum=0.99,
               eps=1e-3):
    """NHWC batch normalisation over all but the last axis (tf.layers.batch_normalization);
    updates the moving statistics in place when training."""
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
    y = (x2.float() - mean) * torch.rsqrt(var + eps) * gamma + beta
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


def max_pool2d(x, ksize=3, strides=2, padding=1):
    y = F.max_pool2d(x.permute(0, 3, 1, 2), ksize, strides, padding)
    return y.permute(0, 2, 3, 1)


def global_avg_pool(x):
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
    if _on_gpu(q, k, v) and hd == 64 and S % 128 == 0:
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


def embedding_lookup(params, ids):
    return F.embedding(ids.long(), params)
