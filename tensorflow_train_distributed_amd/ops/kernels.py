"""Thin launch wrappers for the non-GEMM gfx950 kernels (BatchNorm, pooling, fused
cross-entropy, element-wise/layout, optimizers, fp8). All tensors are CUDA tensors; every
launch goes to PyTorch's current stream. See the .hip files for the math."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1}

ACT_NONE, ACT_RELU, ACT_GELU, ACT_ELU = 0, 1, 2, 3


def _s():
    return _lib.stream()


def _p(t):
    return None if t is None else t.data_ptr()


# ------------------------------------------------------------------ BatchNorm (NHWC)
def bn_num_partials(M, C):
    return _lib.query("ttdk_bn_num_partials", M, C)


def bn_stats_partial(x2d, partial=None):
    """Per-block partial sums of x and x^2 over rows of x2d [M, C] -> (partial [T,2,C], T)."""
    M, C = x2d.shape
    T = bn_num_partials(M, C)
    if partial is None:
        partial = torch.empty((T, 2, C), dtype=torch.float32, device=x2d.device)
    _lib.call("ttdk_bn_stats_partial", x2d.data_ptr(), M, C, partial.data_ptr(), T, _s())
    return partial, T


def bn_reduce_partials(partial, T, C, sums=None):
    if sums is None:
        sums = torch.empty((2, C), dtype=torch.float32, device=partial.device)
    _lib.call("ttdk_bn_reduce_partials", partial.data_ptr(), T, C, sums.data_ptr(), _s())
    return sums


class BNState:
    """Per-call saved statistics of a training-mode BN forward."""

    __slots__ = ("mean", "rstd", "scale", "shift")

    def __init__(self, C, device):
        buf = torch.empty((4, C), dtype=torch.float32, device=device)
        self.mean, self.rstd, self.scale, self.shift = buf[0], buf[1], buf[2], buf[3]


def _bn_reduce_finalize(partial, T, C, bwd, count, gamma=None, beta=None, eps=0.0, momentum=0.0,
                        running_mean=None, running_var=None, state=None, dgamma=None, dbeta=None, coef=None,
                        accumulate=False):
    S = _lib.query("ttdk_bn_finalize_slices", T)
    slab = torch.empty((S, 2, C), dtype=torch.float32, device=partial.device)
    _lib.call("ttdk_bn_reduce_finalize", partial.data_ptr(), T, C, slab.data_ptr(), int(bwd), float(count), _p(gamma), _p(beta), float(eps),
              float(momentum), _p(running_mean), _p(running_var), state.mean.data_ptr(), state.rstd.data_ptr(),
              state.scale.data_ptr(), state.shift.data_ptr(), _p(dgamma), _p(dbeta), _p(coef), int(accumulate),
              _s())


def bn_fwd_stats(partial, T, count, gamma, beta, eps, momentum, running_mean, running_var, state):
    """Fold the per-tile partial sums [T, 2, C] (conv epilogue or bn_stats_partial) and
    finalize the forward statistics into `state` in one launch."""
    _bn_reduce_finalize(partial, T, partial.shape[-1], False, count, gamma, beta, eps, momentum, running_mean,
                        running_var, state)


def bn_fwd_finalize(sums, count, gamma, beta, eps, momentum, running_mean, running_var, state):
    C = sums.shape[-1]
    _lib.call("ttdk_bn_fwd_finalize", sums.data_ptr(), float(count), C, _p(gamma), _p(beta), float(eps),
              float(momentum), _p(running_mean), _p(running_var), state.mean.data_ptr(), state.rstd.data_ptr(),
              state.scale.data_ptr(), state.shift.data_ptr(), _s())


def bn_apply(y2d, scale, shift, *, residual=None, residual_bn=None, relu=False, out=None, mask=None, q8=None,
             q8_slot=None, store_out=True):
    """out = act(y*scale + shift (+ residual)); `residual_bn` = (rscale, rshift) applies a BN
    affine to the residual first (a raw projection-shortcut conv output); `mask` (uint8
    [M*C/8]) optionally receives the ReLU mask as bits so the backward need not re-read `out`;
    `q8` (uint8 like out) an fp8 e4m3 copy quantised with the delayed scale of `q8_slot`
    (fp32[FP8_SLOT], see fp8.hip). store_out=False (with q8): only the fp8 copy and the mask are
    written (the bf16 output has no consumer); returns None."""
    M, C = y2d.shape
    if not store_out:
        if q8 is None:
            raise ValueError("bn_apply: store_out=False needs the fp8 copy")
        _lib.call("ttdk_bn_apply", y2d.data_ptr(), scale.data_ptr(), shift.data_ptr(), _p(residual),
                  _p(residual_bn[0] if residual_bn else None), _p(residual_bn[1] if residual_bn else None), None,
                  _p(mask), _p(q8), _p(q8_slot), M * C, C, int(relu), _s())
        return None
    if out is None:
        out = torch.empty_like(y2d)
    rs, rh = residual_bn if residual_bn is not None else (None, None)
    _lib.call("ttdk_bn_apply", y2d.data_ptr(), scale.data_ptr(), shift.data_ptr(), _p(residual), _p(rs), _p(rh),
              out.data_ptr(), _p(mask), _p(q8), _p(q8_slot), M * C, C, int(relu), _s())
    return out


FP8_SLOT = 72  # floats per fp8 scaling slot (see fp8.hip)


def fp8_rollover(slots, margin=1.0, fmax=448.0):
    """Delayed scaling step for fp8 slots [n, FP8_SLOT] (see fp8.hip): e4m3 activations (fmax
    448), e5m2 gradients (fmax 57344)."""
    _lib.call("ttdk_fp8_rollover", slots.data_ptr(), slots.shape[0], float(fmax), float(margin), _s())


def fp8_quant_weights(src, dst, table, n_tensors, max_len, slots):
    _lib.call("ttdk_fp8_quant_weights", src.data_ptr(), dst.data_ptr(), table.data_ptr(), n_tensors, max_len,
              slots.data_ptr(), slots.shape[0], _s())


def bn_backward(dout, out_for_relu, y, gamma, state, dgamma, dbeta, *, g_out=None, dz=None, accumulate=False,
                mask=None):
    """dz = BN-backward(relu-mask(dout)). Writes dgamma/dbeta (fp32 [C]) and optionally the
    relu-masked gradient g_out (needed by residual shortcuts). The ReLU mask comes from the
    bit mask written by bn_apply (if given) or from `out_for_relu > 0`."""
    M, C = y.shape
    T = bn_num_partials(M, C)
    partial = torch.empty((T, 2, C), dtype=torch.float32, device=y.device)
    _lib.call("ttdk_bn_bwd_partial", dout.data_ptr(), _p(out_for_relu), _p(mask), y.data_ptr(), M, C,
              partial.data_ptr(), T, _p(g_out), _s())
    coef = torch.empty((3, C), dtype=torch.float32, device=y.device)
    _bn_reduce_finalize(partial, T, C, True, M, gamma, state=state, dgamma=dgamma, dbeta=dbeta, coef=coef,
                        accumulate=accumulate)
    if dz is None:
        dz = torch.empty_like(y)
    _lib.call("ttdk_bn_bwd_apply", dout.data_ptr(), _p(out_for_relu), _p(mask), y.data_ptr(), coef.data_ptr(),
              dz.data_ptr(), M * C, C, _s())
    return dz


def bn_backward_coef(M, C, gamma, state, dgamma, dbeta, partial, T, *, accumulate=False, device=None):
    """BN-backward finalize from per-tile sums (sum g, sum g*y): writes dgamma/dbeta and returns
    coef [3, C] with dz = coef[0]*g + coef[1]*y + coef[2] (for a consumer that applies it)."""
    coef = torch.empty((3, C), dtype=torch.float32, device=device if device is not None else gamma.device)
    _bn_reduce_finalize(partial, T, C, True, M, gamma, state=state, dgamma=dgamma, dbeta=dbeta, coef=coef,
                        accumulate=accumulate)
    return coef


def bn_backward_from_partial(g, y, gamma, state, dgamma, dbeta, partial, T, *, dz=None, accumulate=False, q8=None,
                             q8_slot=None, store_dz=True):
    """BN backward when the producer of the (already ReLU-masked) gradient g also emitted the
    per-tile sums (sum g, sum g*y) — ops.gemm.conv_dgrad(bn_stat=...): finalize + one apply
    pass, no separate statistics pass over g and y. q8 (uint8 like dz): an OCP e5m2 copy of dz
    quantised with the delayed scale of q8_slot (fp32[FP8_SLOT]; its amax lanes collect this
    step's amax). store_dz=False (with q8): only the fp8 copy is written; returns None."""
    M, C = y.shape
    coef = bn_backward_coef(M, C, gamma, state, dgamma, dbeta, partial, T, accumulate=accumulate, device=y.device)
    if not store_dz:
        if q8 is None:
            raise ValueError("bn_backward_from_partial: store_dz=False needs the fp8 copy")
        dz = None
    elif dz is None:
        dz = torch.empty_like(y)
    _lib.call("ttdk_bn_bwd_apply_q8", g.data_ptr(), None, None, y.data_ptr(), coef.data_ptr(), _p(dz),
              _p(q8), _p(q8_slot), M * C, C, _s())
    return dz


# ------------------------------------------------------------------ pooling
def pool_out(H, k, s, p):
    return (H + 2 * p - k) // s + 1


def maxpool_fwd(x, k=3, s=2, p=1):
    N, H, W, C = x.shape
    P, Q = pool_out(H, k, s, p), pool_out(W, k, s, p)
    y = torch.empty((N, P, Q, C), dtype=x.dtype, device=x.device)
    arg = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device)
    _lib.call("ttdk_maxpool_fwd", x.data_ptr(), y.data_ptr(), arg.data_ptr(), N, H, W, C, P, Q, k, k, s, s, p, p, _s())
    return y, arg


def maxpool_bwd(dy, arg, x_shape, k=3, s=2, p=1):
    N, H, W, C = x_shape
    P, Q = dy.shape[1], dy.shape[2]
    dx = torch.empty(tuple(x_shape), dtype=dy.dtype, device=dy.device)
    _lib.call("ttdk_maxpool_bwd", dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, H, W, C, P, Q, k, k, s, s, p, p,
              _s())
    return dx


def stem_pool_fusable(y_shape, k=3, s=2, p=1):
    N, H, W, C = y_shape
    return (k, s, p) == (3, 2, 1) and H % 2 == 0 and W % 2 == 0 and C % 8 == 0 and 256 % (C // 8) == 0


def bn_relu_maxpool(y, scale, shift):
    """pooled = maxpool3x3/s2/p1(relu(y*scale + shift)) without storing the BN+ReLU output;
    returns (pooled, argmax bytes, ReLU bit mask of the activation) — see pool.hip."""
    N, H, W, C = y.shape
    P, Q = H // 2, W // 2
    out = torch.empty((N, P, Q, C), dtype=y.dtype, device=y.device)
    arg = torch.empty((N, P, Q, C), dtype=torch.uint8, device=y.device)
    mask = torch.empty(N * H * W * C // 8, dtype=torch.uint8, device=y.device)
    _lib.call("ttdk_bn_relu_maxpool", y.data_ptr(), scale.data_ptr(), shift.data_ptr(), out.data_ptr(), arg.data_ptr(),
              mask.data_ptr(), N, H, W, C, P, Q, _s())
    return out, arg, mask


def maxpool_bwd_bnstat(dy, arg, mask, y):
    """g = relu_mask * maxpool_bwd(dy) plus the BN-backward partial sums (sum g, sum g*y) of the
    stem BN; returns (g, partial [T, 2, C], T) for bn_backward_from_partial."""
    N, H, W, C = y.shape
    P, Q = dy.shape[1], dy.shape[2]
    T = _lib.query("ttdk_maxpool_bwd_bnstat_blocks", N, P, Q, C)
    g = torch.empty_like(y)
    partial = torch.empty((T, 2, C), dtype=torch.float32, device=y.device)
    _lib.call("ttdk_maxpool_bwd_bnstat", dy.data_ptr(), arg.data_ptr(), mask.data_ptr(), y.data_ptr(), g.data_ptr(),
              partial.data_ptr(), N, H, W, C, P, Q, _s())
    return g, partial, T


def avgpool_fwd(x):
    N, H, W, C = x.shape
    y = torch.empty((N, C), dtype=x.dtype, device=x.device)
    _lib.call("ttdk_avgpool_fwd", x.data_ptr(), y.data_ptr(), None, N, H * W, C, _s())
    return y


def avgpool_bwd(dy, x_shape):
    N, H, W, C = x_shape
    dx = torch.empty(tuple(x_shape), dtype=dy.dtype, device=dy.device)
    _lib.call("ttdk_avgpool_bwd", dy.data_ptr(), dx.data_ptr(), N, H * W, C, _s())
    return dx


# ------------------------------------------------------------------ cross-entropy
def sparse_xent(logits, labels, grad_scale=None, *, want_grad=True, want_rows=False, sums=None):
    """Fused sparse softmax cross-entropy fwd+bwd + in_top_k(1).

    Returns (sums[2] = (mean loss, mean accuracy), dlogits or None, loss_rows or None, correct or None).
    """
    rows, V = logits.shape
    if grad_scale is None:
        grad_scale = 1.0 / rows
    lab = labels if labels.dtype in (torch.int32, torch.int64) else labels.long()
    if sums is None:
        sums = torch.empty(2, dtype=torch.float32, device=logits.device)
    part = torch.empty(2 * rows, dtype=torch.float32, device=logits.device)  # per-row terms (fixed-order sum)
    dl = torch.empty_like(logits) if want_grad else None
    lr = torch.empty(rows, dtype=torch.float32, device=logits.device) if want_rows else None
    corr = torch.empty(rows, dtype=torch.uint8, device=logits.device) if want_rows else None
    _lib.call("ttdk_sparse_xent", logits.data_ptr(), _DT[logits.dtype], lab.data_ptr(),
              0 if lab.dtype == torch.int32 else 1, rows, V, float(grad_scale), _p(lr), _p(dl), _p(corr),
              sums.data_ptr(), part.data_ptr(), _s())
    return sums, dl, lr, corr


# ------------------------------------------------------------------ element-wise / layout
def f32_to_bf16(x, out=None):
    if out is None:
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    _lib.call("ttdk_f32_to_bf16", x.data_ptr(), out.data_ptr(), x.numel(), _s())
    return out


def bf16_round_probe(x):
    """The kernels' three fp32 -> bf16 roundings of fp32 `x` (numel % 8 == 0): (f2bf per element,
    pack_bf16x2 per pair, pack8 per 16-B chunk), each as bf16 bits in an int16 tensor of x's size."""
    x = x.contiguous()
    n = x.numel()
    assert x.dtype == torch.float32 and n % 8 == 0
    one = torch.empty(n, dtype=torch.int16, device=x.device)
    pair = torch.empty(n, dtype=torch.int16, device=x.device)
    eight = torch.empty(n, dtype=torch.int16, device=x.device)
    _lib.call("ttdk_bf16_round_probe", x.data_ptr(), one.data_ptr(), pair.data_ptr(), eight.data_ptr(), n, _s())
    return one, pair, eight


def bf16_to_f32(x, out=None):
    if out is None:
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    _lib.call("ttdk_bf16_to_f32", x.data_ptr(), out.data_ptr(), x.numel(), _s())
    return out


def pad_channels(x, Cp):
    C = x.shape[-1]
    rows = x.numel() // C
    y = torch.empty(x.shape[:-1] + (Cp,), dtype=x.dtype, device=x.device)
    _lib.call("ttdk_pad_channels", x.data_ptr(), y.data_ptr(), rows, C, Cp, _s())
    return y


def krsc_to_crsk(w, out=None):
    """bf16 conv filter [K,R,S,C] -> [C,R,S,K] (the data-gradient operand)."""
    K, R, S, C = w.shape
    if out is None:
        out = torch.empty((C, R, S, K), dtype=w.dtype, device=w.device)
    _lib.call("ttdk_transpose_aca_bf16", w.data_ptr(), out.data_ptr(), K, R * S, C, _s())
    return out


def subpixel_phases(s, pad, R, H):
    """(first tap, tap count) of each non-empty sub-pixel phase along one axis of a stride-s
    data gradient, in ttdk_conv_dgrad_subpixel's order (mirror of conv_dgrad.hip phase_of)."""
    out = []
    for a in range(s):
        r0 = (a + pad) % s
        T = (R - r0 + s - 1) // s if r0 < R else 0
        n = (H - a + s - 1) // s if a < H else 0
        if n:
            out.append((r0, T))
    return out


class TransposeBatch:
    """bf16 [A][C] -> [C][A] for a fixed list of (src, dst) 2-D tensor pairs in ONE launch
    (ttdk_transpose128_batch_bf16; A and C multiples of 128, 16-B aligned, contiguous rows).
    The device table holds raw pointers: run() re-checks them against the tensors and rebuilds
    the table when one moved (never inside a graph capture — there it raises)."""

    _DT = np.dtype([("src", "<u8"), ("dst", "<u8"), ("A", "<i4"), ("C", "<i4"), ("tile_begin", "<i4"),
                    ("pad", "<i4")])

    @staticmethod
    def fits(src, dst):
        A, C = src.shape
        return (src.dtype == torch.bfloat16 and dst.dtype == torch.bfloat16 and src.is_contiguous()
                and dst.is_contiguous() and tuple(dst.shape) == (C, A) and A % 128 == 0 and C % 128 == 0
                and src.data_ptr() % 16 == 0 and dst.data_ptr() % 16 == 0)

    def __init__(self, pairs):
        self.pairs = list(pairs)
        if not self.pairs or not all(self.fits(s_, d_) for s_, d_ in self.pairs):
            raise ValueError("TransposeBatch: every pair must be bf16 [A][C] -> [C][A], A, C % 128 == 0, aligned")
        self._ptrs = None
        self._tab = None
        self.tiles = 0
        self._build()

    def _build(self):
        rows, t = [], 0
        for s_, d_ in self.pairs:
            A, C = s_.shape
            rows.append((s_.data_ptr(), d_.data_ptr(), A, C, t, 0))
            t += (A // 128) * (C // 128)
        self._tab = torch.from_numpy(np.array(rows, dtype=self._DT).view(np.uint8).copy()).to(self.pairs[0][0].device)
        self.tiles = t
        self._ptrs = [(s_.data_ptr(), d_.data_ptr()) for s_, d_ in self.pairs]

    def run(self, pairs=None):
        """pairs: this call's (src, dst) tensors (default: the constructor's); the table is rebuilt
        when any pointer differs from the one it holds."""
        if pairs is not None:
            self.pairs = list(pairs)
        ptrs = [(s_.data_ptr(), d_.data_ptr()) for s_, d_ in self.pairs]
        if ptrs != self._ptrs:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("TransposeBatch: tensors moved during a graph capture")
            self._build()
        _lib.call("ttdk_transpose128_batch_bf16", self._tab.data_ptr(), len(self.pairs), self.tiles, _s())


class WeightPrep:
    """Every data-gradient filter operand of a network in one launch per step (ttdk_wprep):
    [C,R,S,K] transposes of the [K,R,S,C] filters, and for strided 3x3 dgrads the sub-pixel
    phase filters in ttdk_conv_dgrad_subpixel's order — instead of one transpose launch per conv
    (and s*s gathers per strided conv) on the backward's critical chain.

    src: the flat bf16 compute copy that holds every filter; add(name, offset, shape) registers a
    [K,R,S,C] filter at that element offset, add(..., sub=(s, pad_h, pad_w, H, W)) its phase
    filters (the dgrad input is H x W); build() packs the table; run() launches on the current
    stream; crsk(name) / phases(name) return views of the output buffer."""

    _DT = np.dtype([("src_off", "<i8"), ("dst_off", "<i8"), ("K", "<i4"), ("R", "<i4"), ("S", "<i4"),
                    ("C", "<i4"), ("s", "<i4"), ("r0", "<i4"), ("Tr", "<i4"), ("s0", "<i4"), ("Ts", "<i4"),
                    ("tile_begin", "<i4")])

    def __init__(self, src):
        self.src = src
        self._rows = []
        self._views = {}
        self._dst_n = 0
        self._tiles = 0
        self.buf = None

    def _entry(self, off, shape, s, r0, Tr, s0, Ts):
        K, R, S, C = shape
        dst = self._dst_n
        self._rows.append((off, dst, K, R, S, C, s, r0, Tr, s0, Ts, self._tiles))
        self._tiles += Tr * Ts * (-(-K // 32)) * (-(-C // 32))
        self._dst_n += C * Tr * Ts * K
        return dst

    def add(self, name, offset, shape, sub=None):
        K, R, S, C = shape
        if sub is None:
            self._views[name] = ("crsk", self._entry(offset, shape, 1, 0, R, 0, S), (C, R, S, K))
            return
        s, ph, pw, H, W = sub
        start = self._dst_n
        for r0, Tr in subpixel_phases(s, ph, R, H):
            for s0, Ts in subpixel_phases(s, pw, S, W):
                self._entry(offset, shape, s, r0, Tr, s0, Ts)
        self._views[name] = ("phases", start, self._dst_n - start)

    def build(self):
        arr = np.zeros(len(self._rows), dtype=self._DT)
        for i, r in enumerate(self._rows):
            arr[i] = r
        self._tab = torch.from_numpy(arr.view(np.uint8).copy()).to(self.src.device)
        self.buf = torch.empty(max(self._dst_n, 1), dtype=torch.bfloat16, device=self.src.device)
        return self

    def run(self):
        if self._rows:
            _lib.call("ttdk_wprep", self.src.data_ptr(), self.buf.data_ptr(), self._tab.data_ptr(), len(self._rows),
                      self._tiles, _s())

    def has(self, name):
        return name in self._views

    def crsk(self, name):
        kind, off, shape = self._views[name]
        assert kind == "crsk"
        return self.buf[off:off + int(np.prod(shape))].view(shape)

    def phases(self, name):
        kind, off, n = self._views[name]
        assert kind == "phases"
        return self.buf[off:off + n]


def bias_act_dropout(x, bias, act=ACT_NONE, rate=0.0, seed=0, offset=0, out=None):
    C = x.shape[-1]
    if out is None:
        out = torch.empty_like(x)
    _lib.call("ttdk_bias_act_dropout_fwd", x.data_ptr(), _p(bias), out.data_ptr(), x.numel(), C, act, float(rate),
              seed, offset, _DT[x.dtype], _s())
    return out


def bias_act_dropout_bwd(dy, x, bias, act=ACT_NONE, rate=0.0, seed=0, offset=0, out=None):
    C = x.shape[-1]
    if out is None:
        out = torch.empty_like(x)
    _lib.call("ttdk_bias_act_dropout_bwd", dy.data_ptr(), x.data_ptr(), _p(bias), out.data_ptr(), x.numel(), C, act,
              float(rate), seed, offset, _DT[x.dtype], _s())
    return out


def colsum(x2d, out=None, beta=0):
    rows, C = x2d.shape
    if not x2d.is_contiguous():
        raise ValueError("colsum reads dense rows (got strides %s)" % (tuple(x2d.stride()),))
    if out is None:
        out = torch.empty(C, dtype=torch.float32, device=x2d.device)
    nws = _lib.query("ttdk_colsum_ws_floats", rows, C, _DT[x2d.dtype])
    ws = torch.empty(max(1, nws), dtype=torch.float32, device=x2d.device) if nws else None
    _lib.call("ttdk_colsum", x2d.data_ptr(), rows, C, out.data_ptr(), int(beta), _DT[x2d.dtype], _p(ws), _s())
    return out


def add_bf16(a, b, out=None, alpha=1.0, beta=1.0):
    if out is None:
        out = torch.empty_like(a)
    _lib.call("ttdk_add_bf16", a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), float(alpha), float(beta), _s())
    return out


# ------------------------------------------------------------------ fp8 (OCP e4m3fn / e5m2)
def amax(x, out=None, reset=True):
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    _lib.call("ttdk_amax_bf16", x.data_ptr(), x.numel(), out.data_ptr(), int(reset), _s())
    return out


def quant_fp8(x, scale, e5m2=False, out=None):
    if out is None:
        out = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _lib.call("ttdk_quant_fp8", x.data_ptr(), out.data_ptr(), x.numel(), scale.data_ptr(), int(e5m2), _s())
    return out


def dequant_fp8(q, scale, e5m2=False, out=None):
    if out is None:
        out = torch.empty(q.shape, dtype=torch.bfloat16, device=q.device)
    _lib.call("ttdk_dequant_fp8", q.data_ptr(), out.data_ptr(), q.numel(), scale.data_ptr(), int(e5m2), _s())
    return out


# ------------------------------------------------------------------ optimizer primitives
def sumsq(x, out=None):
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=x.device)
    partial = torch.empty(2048, dtype=torch.float32, device=x.device)  # per-block partials (fixed-order fold)
    _lib.call("ttdk_sumsq", x.data_ptr(), x.numel(), out.data_ptr(), partial.data_ptr(), _s())
    return out


# ------------------------------------------------------------------ shape-general ttd.nn kernels (nn_generic.hip)
_lib.register({
    "ttdk_col_stats_parts": [_lib.L, _lib.I],
    "ttdk_col_stats": [_lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.L, _lib.I, _lib.P, _lib.I, _lib.P],
    "ttdk_col_reduce2": [_lib.P, _lib.I, _lib.I, _lib.P, _lib.P, _lib.I, _lib.P],
    "ttdk_col_affine": [_lib.P, _lib.P, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P, _lib.L, _lib.I, _lib.P],
    "ttdk_bn_infer_coef": [_lib.P, _lib.P, _lib.P, _lib.P, _lib.F, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P],
    "ttdk_bn_infer_bwd": [_lib.P, _lib.I, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P],
    "ttdk_maxpool_generic_fwd": [_lib.P, _lib.P, _lib.P, _lib.I] + [_lib.I] * 12 + [_lib.P],
    "ttdk_maxpool_generic_bwd": [_lib.P, _lib.P, _lib.P, _lib.I] + [_lib.I] * 12 + [_lib.P],
    "ttdk_gap_fwd": [_lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P],
    "ttdk_gap_bwd": [_lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P],
    "ttdk_ln_generic_fwd": [_lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.L, _lib.I, _lib.F, _lib.P],
    "ttdk_ln_generic_bwd_dx": [_lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.L, _lib.I, _lib.P],
    "ttdk_gather_generic": [_lib.P, _lib.P, _lib.I, _lib.P, _lib.I, _lib.L, _lib.I, _lib.L, _lib.P],
    "ttdk_scatter_add_generic": [_lib.P, _lib.P, _lib.I, _lib.P, _lib.I, _lib.L, _lib.I, _lib.L, _lib.P],
    "ttdk_in_top_k": [_lib.P, _lib.P, _lib.I, _lib.P, _lib.I, _lib.L, _lib.I, _lib.I, _lib.P],
    "ttdk_unary": [_lib.P, _lib.P, _lib.I, _lib.L, _lib.I, _lib.P],
    "ttdk_unary_bwd": [_lib.P, _lib.P, _lib.P, _lib.I, _lib.L, _lib.I, _lib.P],
})


def _dt(*ts):
    d = ts[0].dtype
    for t in ts:
        if t is not None and (t.dtype != d or not t.is_contiguous()):
            raise ValueError("generic nn kernels need contiguous tensors of one dtype (got %s)"
                             % [(x.dtype, x.is_contiguous()) for x in ts if x is not None])
    if d not in _DT:
        raise ValueError("generic nn kernels support float32/bfloat16, got %s" % d)
    return _DT[d]


def col_stats(a2d, b2d=None, mode=0, mu=None, rs=None):
    """Per-row-block column sums: mode 0 (sum a, sum a^2), 1 (sum a, sum a*b), 2 (sum a,
    sum a*(b-mu[r])*rs[r]). Returns (partial [T, 2, C], T)."""
    M, C = a2d.shape
    T = _lib.query("ttdk_col_stats_parts", M, C)
    part = torch.empty((T, 2, C), dtype=torch.float32, device=a2d.device)
    _lib.call("ttdk_col_stats", a2d.data_ptr(), _p(b2d), _p(mu), _p(rs), _dt(a2d, b2d), int(mode), M, C,
              part.data_ptr(), T, _s())
    return part, T


def col_reduce2(part, T, o0=None, o1=None, accumulate=False):
    C = part.shape[-1]
    _lib.call("ttdk_col_reduce2", part.data_ptr(), T, C, _p(o0), _p(o1), int(accumulate), _s())
    return o0, o1


def col_affine(a, c0, b=None, c1=None, c2=None, out=None):
    """out = a*c0[c] + b*c1[c] + c2[c] over the last (channel) axis."""
    if out is None:
        out = torch.empty_like(a)
    _lib.call("ttdk_col_affine", a.data_ptr(), _p(b), _dt(a, b, out), c0.data_ptr(), _p(c1), _p(c2), out.data_ptr(),
              a.numel(), a.shape[-1], _s())
    return out


def bn_infer_coef(mm, mv, gamma, beta, eps):
    C = mm.numel()
    buf = torch.empty((3, C), dtype=torch.float32, device=mm.device)
    _lib.call("ttdk_bn_infer_coef", mm.data_ptr(), mv.data_ptr(), _p(gamma), _p(beta), float(eps), C,
              buf[0].data_ptr(), buf[1].data_ptr(), buf[2].data_ptr(), _s())
    return buf[0], buf[1], buf[2]


def bn_infer_bwd(part, T, mm, rstd, dgamma, dbeta):
    _lib.call("ttdk_bn_infer_bwd", part.data_ptr(), T, part.shape[-1], mm.data_ptr(), rstd.data_ptr(), _p(dgamma),
              _p(dbeta), _s())


def maxpool_generic_fwd(x, R, S, sh, sw, ph, pw, P, Q):
    N, H, W, C = x.shape
    y = torch.empty((N, P, Q, C), dtype=x.dtype, device=x.device)
    arg = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device)
    _lib.call("ttdk_maxpool_generic_fwd", x.data_ptr(), y.data_ptr(), arg.data_ptr(), _dt(x), N, H, W, C, P, Q, R, S,
              sh, sw, ph, pw, _s())
    return y, arg


def maxpool_generic_bwd(dy, arg, x_shape, R, S, sh, sw, ph, pw):
    N, H, W, C = x_shape
    P, Q = dy.shape[1], dy.shape[2]
    dx = torch.empty(tuple(x_shape), dtype=dy.dtype, device=dy.device)
    _lib.call("ttdk_maxpool_generic_bwd", dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), _dt(dy), N, H, W, C, P, Q, R,
              S, sh, sw, ph, pw, _s())
    return dx


def gap_fwd(x):
    N, H, W, C = x.shape
    y = torch.empty((N, C), dtype=x.dtype, device=x.device)
    _lib.call("ttdk_gap_fwd", x.data_ptr(), y.data_ptr(), _dt(x), N, H * W, C, _s())
    return y


def gap_bwd(dy, x_shape):
    N, H, W, C = x_shape
    dx = torch.empty(tuple(x_shape), dtype=dy.dtype, device=dy.device)
    _lib.call("ttdk_gap_bwd", dy.data_ptr(), dx.data_ptr(), _dt(dy), N, H * W, C, _s())
    return dx


def ln_generic_fwd(x2d, gamma, beta, eps):
    rows, H = x2d.shape
    y = torch.empty_like(x2d)
    stats = torch.empty((2, rows), dtype=torch.float32, device=x2d.device)
    _lib.call("ttdk_ln_generic_fwd", x2d.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
              stats[0].data_ptr(), stats[1].data_ptr(), _dt(x2d), rows, H, float(eps), _s())
    return y, stats[0], stats[1]


def ln_generic_bwd(dy2d, x2d, gamma, mean, rstd, dgamma, dbeta, want_dx=True):
    rows, H = x2d.shape
    dx = None
    if want_dx:
        dx = torch.empty_like(x2d)
        _lib.call("ttdk_ln_generic_bwd_dx", dy2d.data_ptr(), x2d.data_ptr(), gamma.data_ptr(), mean.data_ptr(),
                  rstd.data_ptr(), dx.data_ptr(), _dt(dy2d, x2d), rows, H, _s())
    part, T = col_stats(dy2d, x2d, mode=2, mu=mean, rs=rstd)
    col_reduce2(part, T, o0=dbeta, o1=dgamma)
    return dx


def _ids(ids):
    if ids.dtype not in (torch.int32, torch.int64) or not ids.is_contiguous():
        raise ValueError("ids must be a contiguous int32/int64 tensor")
    return 1 if ids.dtype == torch.int64 else 0


def gather_generic(table, ids):
    V, H = table.shape
    out = torch.empty(tuple(ids.shape) + (H,), dtype=table.dtype, device=table.device)
    _lib.call("ttdk_gather_generic", table.data_ptr(), ids.data_ptr(), _ids(ids), out.data_ptr(), _dt(table),
              ids.numel(), H, V, _s())
    return out


def scatter_add_generic(dy, ids, dtable):
    V, H = dtable.shape
    if dtable.dtype != torch.float32:
        raise ValueError("scatter_add_generic accumulates into an fp32 table")
    _lib.call("ttdk_scatter_add_generic", dy.data_ptr(), ids.data_ptr(), _ids(ids), dtable.data_ptr(), _dt(dy),
              ids.numel(), H, V, _s())
    return dtable


def in_top_k(z, targets, k):
    rows, V = z.shape
    out = torch.empty(rows, dtype=torch.uint8, device=z.device)
    _lib.call("ttdk_in_top_k", z.data_ptr(), targets.data_ptr(), _ids(targets), out.data_ptr(), _dt(z), rows, V, int(k),
              _s())
    return out


UNARY_TANH, UNARY_SIGMOID = 0, 1


def unary(x, op):
    y = torch.empty_like(x)
    _lib.call("ttdk_unary", x.data_ptr(), y.data_ptr(), _dt(x), x.numel(), int(op), _s())
    return y


def unary_bwd(dy, y, op):
    dx = torch.empty_like(y)
    _lib.call("ttdk_unary_bwd", dy.data_ptr(), y.data_ptr(), dx.data_ptr(), _dt(dy, y), y.numel(), int(op), _s())
    return dx


_lib.register({
    "ttdk_sum_blocks": [_lib.L],
    "ttdk_sum_all": [_lib.P, _lib.I, _lib.L, _lib.P, _lib.F, _lib.P, _lib.P],
    "ttdk_fill_scaled": [_lib.P, _lib.I, _lib.L, _lib.P, _lib.F, _lib.P],
    "ttdk_row_scale": [_lib.P, _lib.P, _lib.P, _lib.I, _lib.L, _lib.I, _lib.P],
})


def sum_all(x, scale=1.0):
    """0-d tensor = scale * sum(x) (deterministic two-stage reduction), same dtype as x."""
    n = x.numel()
    ws = torch.empty(_lib.query("ttdk_sum_blocks", n), dtype=torch.float32, device=x.device)
    out = torch.empty((), dtype=x.dtype, device=x.device)
    _lib.call("ttdk_sum_all", x.data_ptr(), _dt(x), n, ws.data_ptr(), float(scale), out.data_ptr(), _s())
    return out


def fill_scaled(shape, g, scale, dtype):
    dx = torch.empty(shape, dtype=dtype, device=g.device)
    if g.dtype != dtype:
        raise ValueError("fill_scaled: gradient dtype %s != %s" % (g.dtype, dtype))
    _lib.call("ttdk_fill_scaled", dx.data_ptr(), _dt(dx), dx.numel(), g.data_ptr(), float(scale), _s())
    return dx


def row_scale(a2d, g):
    rows, C = a2d.shape
    out = torch.empty_like(a2d)
    _lib.call("ttdk_row_scale", a2d.data_ptr(), g.data_ptr(), out.data_ptr(), _dt(a2d, out), rows, C, _s())
    return out


_lib.register({"ttdk_zero": [_lib.P, _lib.L, _lib.P], "ttdk_trace_marker": [_lib.I, _lib.P],
               "ttdk_copy": [_lib.P, _lib.P, _lib.L, _lib.P]})


def concat_(out, parts):
    """out = concatenation of the contiguous tensors `parts` (same dtype), by stream-ordered
    device copies (no torch cat kernel in a captured step)."""
    if not out.is_contiguous():
        raise ValueError("concat_ needs a contiguous output")
    o = 0
    es = out.element_size()
    for t in parts:
        if t.dtype != out.dtype or not t.is_contiguous():
            raise ValueError("concat_: parts must be contiguous %s" % out.dtype)
        n = t.numel()
        if o + n > out.numel():
            raise ValueError("concat_: parts exceed the output")
        _lib.call("ttdk_copy", out.data_ptr() + o * es, t.data_ptr(), n * es, _s())
        o += n
    return out


def zero_(t):
    """t.zero_() through hipMemsetAsync on the current stream (contiguous CUDA tensors)."""
    if not t.is_contiguous():
        raise ValueError("zero_ needs a contiguous tensor")
    _lib.call("ttdk_zero", t.data_ptr(), t.numel() * t.element_size(), _s())
    return t


def zeros(shape, dtype=torch.float32, device="cuda"):
    return zero_(torch.empty(shape, dtype=dtype, device=device))


def trace_marker(tag=0):
    _lib.call("ttdk_trace_marker", int(tag), _s())


# ------------------------------------------------------------------ device initialisation (init.hip)
_lib.register({"ttdk_init_random": [_lib.P, _lib.L, _lib.I, _lib.F, _lib.F, _lib.U64, _lib.U64, _lib.P]})

INIT_NORMAL, INIT_TRUNCATED, INIT_UNIFORM, INIT_CONSTANT = 0, 1, 2, 3


def init_random_(t, dist, a, b=0.0, seed=0, offset=0):
    """Fill contiguous fp32 CUDA tensor t on the device: normal(a, b), truncated normal(a, b)
    (+-2 b, resampled), uniform[a, b) or constant a — a pure function of (seed, offset, index)."""
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError("init_random_ needs a contiguous fp32 tensor")
    _lib.call("ttdk_init_random", t.data_ptr(), t.numel(), int(dist), float(a), float(b), int(seed) & (2**64 - 1),
              int(offset) & (2**64 - 1), _s())
    return t
