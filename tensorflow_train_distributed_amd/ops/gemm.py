"""Launch wrappers for the MFMA GEMM / implicit-GEMM convolution kernels (gemm_conv.hip).

Tensors here are CUDA (HIP) tensors in the layouts the kernels expect:
activations NHWC bf16, conv filters [K, R, S, C] bf16 (TF keeps [R, S, C, K]; the layer
converts once per step), weight gradients fp32.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

ACT_NONE, ACT_RELU, ACT_GELU, ACT_TANH, ACT_DGELU = 0, 1, 2, 3, 4

# Optional launch log (kind, M, N, K, splits) for matching rocprofv3 dispatches to layer
# shapes: enable with TTD_GEMM_LOG=1, read/reset via gemm_log().
import os as _os
_LOG = [] if _os.environ.get("TTD_GEMM_LOG") else None


def gemm_log(reset=False):
    out = list(_LOG or [])
    if reset and _LOG is not None:
        _LOG.clear()
    return out


def _log(kind, M, N, K, splits=1):
    if _LOG is not None:
        _LOG.append((kind, int(M), int(N), int(K), int(splits)))
    _lib.label((kind, int(M), int(N), int(K)))


def _epi(out, *, mode=0, ldo=None, bias=None, residual=None, act=0, beta=0, stat=None, alpha=1.0,
         slab_stride=0, aux=None, ascale=(None, None), by=None, bmask=None, by2=None, stat2=None,
         beta_s2=None):
    e = _lib.Epilogue()
    e.mode = mode
    e.out = out.data_ptr()
    e.ldo = ldo if ldo is not None else (out.stride(0) if out.dim() == 2 else out.shape[-1])
    e.slab_stride = slab_stride
    e.bias = bias.data_ptr() if bias is not None else None
    e.residual = residual.data_ptr() if residual is not None else None
    e.ldr = (residual.stride(0) if residual.dim() == 2 else residual.shape[-1]) if residual is not None else 0
    e.act = act
    e.beta = beta
    e.stat = stat.data_ptr() if stat is not None else None
    e.alpha = alpha
    e.aux = aux.data_ptr() if aux is not None else None
    e.ascale0 = ascale[0].data_ptr() if ascale[0] is not None else None
    e.ascale1 = ascale[1].data_ptr() if ascale[1] is not None else None
    e.by = by.data_ptr() if by is not None else None
    e.bmask = bmask.data_ptr() if bmask is not None else None
    e.by2 = by2.data_ptr() if by2 is not None else None
    e.stat2 = stat2.data_ptr() if stat2 is not None else None
    e.bH, e.bW = beta_s2 if beta_s2 is not None else (0, 0)
    return e


def big_bn(M, N, K):
    """Mirror of the C++ big_bn(): tile width (256 / 128) of the 256-row LDS-DMA kernel for an
    M x N x K GEMM, or 0 when the 4-wave kernel is used."""
    if M < 256 or N < 128 or K % 64 or N % 8 or M * N < (1 << 20):
        return 0
    return 256 if N >= 256 else 128


def big_fits(M, N, K):
    return big_bn(M, N, K) != 0


def big_bn_wgrad(M, N, K):
    """Mirror of the C++ big_bn_wgrad() (conv weight gradients: long K, split-K)."""
    if M < 256 or N < 128 or K % 64 or N % 8:
        return 0
    return 256 if N >= 256 else 128


def effective_splits(K, splits, bk=64):
    """Mirror of the kernel launcher's split-K clamping (every split gets >= 1 K-tile)."""
    kt = -(-K // bk)
    splits = max(1, min(splits, kt))
    per = -(-kt // splits)
    return -(-kt // per)


def _check(t, dtype, name):
    if t.dtype != dtype or not t.is_cuda or not t.is_contiguous():
        raise ValueError("%s must be a contiguous CUDA %s tensor (got %s %s contig=%s)"
                         % (name, dtype, t.dtype, t.device, t.is_contiguous()))


def _check2d(t, dtype, name):
    """2-D operand whose rows may be strided (a column slice of a wider buffer)."""
    if t.dtype != dtype or not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("%s must be a row-major 2-D CUDA %s tensor (got %s %s shape %s strides %s)"
                         % (name, dtype, t.dtype, t.device, tuple(t.shape), t.stride()))


def gemm(a, b, *, trans_a=False, trans_b=False, out=None, out_dtype=torch.bfloat16, bias=None,
         act=ACT_NONE, residual=None, beta=0, alpha=1.0, splits=1, tile=(0, 0), aux=None, stat=None):
    """C = alpha * op(a) @ op(b) (+bias) (+residual) (+C if beta) -> act.

    a: [M, K] (or [K, M] with trans_a); b: [K, N] (or [N, K] with trans_b); bf16 2-D with unit
    column stride (row stride = leading dimension, so column slices of fused buffers work).
    out_dtype bf16 (fused epilogue) or float32 (plain / split-K store).
    aux: optional bf16 [M, N] receiving the pre-activation value (bias/residual applied).
    stat: optional fp32 [ceil(M/BM), 2, N] per-tile column (sum, sumsq) of the stored output.
    act=ACT_DGELU multiplies by gelu'(residual) instead of adding the residual.
    """
    _check2d(a, torch.bfloat16, "a")
    _check2d(b, torch.bfloat16, "b")
    M, K = (a.shape[1], a.shape[0]) if trans_a else a.shape
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else b.shape
    if K != Kb:
        raise ValueError("gemm inner dims differ: %d vs %d" % (K, Kb))
    if stat is not None:
        # statistics rows = M tiles of the kernel: the caller names the tile height
        if (tile[0] not in (64, 128, 256) or (tile[0] != 256 and not tile[1]) or stat.shape[0] < -(-M // tile[0])
                or stat.shape[-1] != N):
            raise ValueError("gemm stat needs tile=(BM, ..) with BM in 64/128/256 and >= ceil(M/BM) rows of N "
                             "(got tile %s, stat %s)" % (tile, tuple(stat.shape)))
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    elif tuple(out.shape) != (M, N) or out.stride(-1) != 1:
        raise ValueError("gemm out must be [%d, %d] row-major (got %s strides %s)" % (M, N, tuple(out.shape),
                                                                                   out.stride()))
    _log("gemm_%s%s" % ("t" if trans_a else "n", "t" if trans_b else "n"), M, N, K, splits)
    a_kmajor = 0 if trans_a else 1
    lda = a.stride(0)
    b_kmajor = 1 if trans_b else 0
    ldb = b.stride(0)
    if out.dtype == torch.float32:
        splits = effective_splits(K, splits)
        if splits > 1:
            if not out.is_contiguous():
                raise ValueError("split-K output must be contiguous")
            ws = torch.empty((splits, M, N), dtype=torch.float32, device=a.device)
            # the 256-row kernel folds its own slabs (last split of each tile); else (and with a
            # forced tile, which the slab path honours) a fold pass
            _lib.call("ttdk_gemm_bf16_splitk", a.data_ptr(), lda, a_kmajor, b.data_ptr(), ldb, b_kmajor, M, N, K,
                      splits, ws.data_ptr(), out.data_ptr(), beta, float(alpha), int(tile[0]), int(tile[1]),
                      _lib.stream())
            return out
        e = _epi(out, mode=2, beta=beta, alpha=alpha)
    else:
        e = _epi(out, bias=bias, residual=residual, act=act, beta=beta, alpha=alpha, aux=aux, stat=stat)
    _lib.call("ttdk_gemm_bf16", a.data_ptr(), lda, a_kmajor, b.data_ptr(), ldb, b_kmajor, M, N, K, 1,
              tile[0], tile[1], ctypes.byref(e), _lib.stream())
    return out


_lib.register({"ttdk_gemm4w_bf16": [_lib.P, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.I, _lib.E, _lib.P],
               "ttdk_set_g4_sched": [_lib.I], "ttdk_set_g4_group": [_lib.I],
               "ttdk_set_g4_stagger": [_lib.I]})


def set_g4_stagger(v: int) -> int:
    """Stagger the persistent 4-wave GEMM's workgroup tile phases (1) or not (0); returns the
    previous setting."""
    return int(_lib.query("ttdk_set_g4_stagger", int(v)))


def set_g4_group(v: int) -> int:
    """Tile rows per column-major tile block of the 4-wave GEMM's tile order (1 = row-major).
    Returns the previous setting."""
    return int(_lib.query("ttdk_set_g4_group", int(v)))


def set_g4_sched(v: int) -> int:
    """Main-loop schedule of the 4-wave GEMM (gemm4w.hip g4_sched): 3 = hand-ordered inline asm,
    one tile per workgroup (default), 30 = persistent, 0 = compiler-scheduled (A/B and tests).
    Returns the previous setting."""
    return int(_lib.query("ttdk_set_g4_sched", int(v)))


def gemm4w(a, b, *, out=None, bias=None, act=ACT_NONE, residual=None, beta=0, alpha=1.0, aux=None):
    """C[M,N] = alpha * a[M,K] . b[N,K]^T (+bias) (dGELU(residual) | +C if beta) -> act on the
    4-wave 256x256 AGPR-accumulator kernel (gemm4w.hip). Both operands K-major bf16; raises when
    the kernel does not take the shape (no silent fallback: this entry exists to pin that path)."""
    _check2d(a, torch.bfloat16, "a")
    _check2d(b, torch.bfloat16, "b")
    M, K = a.shape
    N, Kb = b.shape
    if K != Kb:
        raise ValueError("gemm4w inner dims differ: %d vs %d" % (K, Kb))
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    e = _epi(out, bias=bias, residual=residual, act=act, beta=beta, alpha=alpha, aux=aux)
    _log("gemm4w", M, N, K, 1)
    _lib.call("ttdk_gemm4w_bf16", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), M, N, K, ctypes.byref(e),
              _lib.stream())
    return out


_lib.register({"ttdk_gemm_bf16_batched": [_lib.P, _lib.L, _lib.L, _lib.I, _lib.P, _lib.L, _lib.L, _lib.I, _lib.P,
                                          _lib.L, _lib.L, _lib.I, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P],
               "ttdk_gemm_f32_batched": [_lib.P, _lib.L, _lib.L, _lib.I, _lib.P, _lib.L, _lib.L, _lib.I, _lib.P,
                                         _lib.L, _lib.L, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P]})


def gemm_batched(a, b, *, trans_a=False, trans_b=False, out_dtype=torch.float32):
    """Strided-batched C[z] = op(a[z]) @ op(b[z]) for every z in ONE kernel launch (batch index on
    the grid's z). a: [Bt, M, K] ([Bt, K, M] with trans_a), b: [Bt, K, N] ([Bt, N, K] with trans_b),
    contiguous 3-D. bf16 operands -> bf16 / fp32 output on the MFMA GEMM; fp32 operands -> exact
    fp32 (f32 MFMA). The batched MatMul of tf.matmul on rank > 2 operands."""
    if a.dim() != 3 or b.dim() != 3 or a.shape[0] != b.shape[0]:
        raise ValueError("gemm_batched needs [B, ., .] operands with equal batch, got %s and %s"
                         % (tuple(a.shape), tuple(b.shape)))
    a = a.contiguous()
    b = b.contiguous()
    Bt = a.shape[0]
    M, K = (a.shape[2], a.shape[1]) if trans_a else (a.shape[1], a.shape[2])
    Kb, N = (b.shape[2], b.shape[1]) if trans_b else (b.shape[1], b.shape[2])
    if K != Kb:
        raise ValueError("gemm_batched inner dims differ: %d vs %d" % (K, Kb))
    _log("gemm_batched", M, N, K, Bt)
    if a.dtype == torch.float32 and b.dtype == torch.float32:
        out = torch.empty((Bt, M, N), dtype=torch.float32, device=a.device)
        _lib.call("ttdk_gemm_f32_batched", a.data_ptr(), a.stride(1), a.stride(0), int(trans_a), b.data_ptr(),
                  b.stride(1), b.stride(0), int(trans_b), out.data_ptr(), N, M * N, M, N, K, Bt, _lib.stream())
        return out
    _check(a, torch.bfloat16, "a")
    _check(b, torch.bfloat16, "b")
    out = torch.empty((Bt, M, N), dtype=out_dtype, device=a.device)
    _lib.call("ttdk_gemm_bf16_batched", a.data_ptr(), a.stride(1), a.stride(0), 0 if trans_a else 1, b.data_ptr(),
              b.stride(1), b.stride(0), 1 if trans_b else 0, out.data_ptr(), N, M * N,
              1 if out_dtype == torch.float32 else 0, M, N, K, Bt, _lib.stream())
    return out


def wgrad_bias_ok(M, N, K, splits) -> bool:
    """Whether gemm_wgrad_bias takes this weight gradient (dW[M,N] over K tokens, `splits`
    K-slices): the 256-wide ping-pong kernel with >= 16 K-tiles per split."""
    if M % 8 or N % 8 or K % 64:
        return False
    if int(_lib.query("ttdk_gemm_wgrad_bias_ws", int(M), int(N), int(K), int(splits))) < 0:
        return False
    kt = K // 64
    s = max(1, min(int(splits), kt))
    per = -(-kt // s)
    return per >= 16


def gemm_wgrad_bias(dy, x, out, bias_out, splits=1, beta=0, alpha=1.0):
    """Weight AND bias gradient of a dense layer in one pass over dy: out[M,N] (+)= alpha *
    dy^T . x (fp32) and bias_out[M] = column sums of dy (written), with dy [K, M] and x [K, N]
    bf16 row-major (K = tokens). The bias sums are formed from dy's tiles already in LDS by the
    weight-gradient GEMM (gemm256_kernel RS) — the separate column-sum pass over dy disappears.
    Callers check wgrad_bias_ok first."""
    _check2d(dy, torch.bfloat16, "dy")
    _check2d(x, torch.bfloat16, "x")
    K, M = dy.shape
    K2, N = x.shape
    if K != K2:
        raise ValueError("gemm_wgrad_bias: token dims differ (%d vs %d)" % (K, K2))
    if tuple(out.shape) != (M, N) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("gemm_wgrad_bias: out must be a contiguous fp32 [%d, %d]" % (M, N))
    if bias_out.numel() != M or bias_out.dtype != torch.float32 or not bias_out.is_contiguous():
        raise ValueError("gemm_wgrad_bias: bias_out must be a contiguous fp32 [%d]" % M)
    nws = int(_lib.query("ttdk_gemm_wgrad_bias_ws", M, N, K, int(splits)))
    if nws < 0:
        raise ValueError("gemm_wgrad_bias: shape %dx%dx%d not on the 256-wide kernel" % (M, N, K))
    ws = torch.empty(nws, dtype=torch.float32, device=dy.device)
    _log("wgrad_bias", M, N, K, splits)
    _lib.call("ttdk_gemm_wgrad_bias", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), M, N, K, int(splits),
              ws.data_ptr(), out.data_ptr(), int(beta), float(alpha), bias_out.data_ptr(), _lib.stream())
    return out, bias_out


def gemm4t(dy, x, out=None, bias_out=None, *, splits=1, beta=0, alpha=1.0):
    """Weight gradient out[M,N] (+)= alpha * dy^T . x (fp32) on the 4-wave transposed-read kernel
    (gemm4t.hip), dy [K, M] and x [K, N] bf16 row-major (K = tokens), split-K summed inside the
    launch; bias_out[M] (optional) = column sums of dy, written. Raises when the kernel does not
    take the shape (no silent fallback: this entry exists to pin that path)."""
    _check2d(dy, torch.bfloat16, "dy")
    _check2d(x, torch.bfloat16, "x")
    K, M = dy.shape
    K2, N = x.shape
    if K != K2:
        raise ValueError("gemm4t: token dims differ (%d vs %d)" % (K, K2))
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=dy.device)
    if tuple(out.shape) != (M, N) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("gemm4t: out must be a contiguous fp32 [%d, %d]" % (M, N))
    if bias_out is not None and (bias_out.numel() != M or bias_out.dtype != torch.float32
                                 or not bias_out.is_contiguous()):
        raise ValueError("gemm4t: bias_out must be a contiguous fp32 [%d]" % M)
    nws = int(_lib.query("ttdk_gemm4t_ws", M, N, K, int(splits)))
    if nws < 0:
        raise ValueError("gemm4t does not take M=%d N=%d K=%d (K a multiple of 64 >= 128, M / N multiples "
                         "of 8, operands < 2 GiB, TTD_G4T on)" % (M, N, K))
    ws = torch.empty(max(nws, 1), dtype=torch.float32, device=dy.device)
    _log("gemm4t", M, N, K, splits)
    _lib.call("ttdk_gemm4t_wgrad", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), M, N, K, int(splits),
              ws.data_ptr(), out.data_ptr(), int(beta), float(alpha), _lib.ptr(bias_out), _lib.stream())
    return out


_C3 = _os.environ.get("TTD_CONV3", "1") != "0"


_lib.register({"ttdk_set_conv3_s3": [_lib.I]})


def set_conv3_s3(on: bool) -> bool:
    """Switch the stage-3 (28 x 28, 128 -> 128) streamed-filter halo conv on / off (TTD_CONV3_S3);
    returns the previous setting. Takes effect for convs dispatched afterwards."""
    return bool(_lib.query("ttdk_set_conv3_s3", 1 if on else 0))


def conv3_rows(H, W, C, N, pro=0):
    """Output pixels per tile of the halo 3x3 kernel (conv3_halo.hip) for a [*, H, W, C] -> N
    3x3/s1/p1 conv with prologue `pro` (0 none, 1 BN forward, 2 BN backward), or 0 when the
    shape is not compiled in (or TTD_CONV3=0)."""
    return int(_lib.query("ttdk_conv3_rows", int(H), int(W), int(C), int(N), int(pro))) if _C3 else 0


def conv3_halo(x, w, *, prologue=None, flip=False, out=None, stat=False, bn_stat=None):
    """3x3 stride-1 pad-1 conv on the persistent halo kernel (conv3_halo.hip):
    out[N, H, W, Co] = conv(A'(x), w) with A' from the prologue

      None                                   A' = x
      ("bn_fwd", scale, shift, side, mask)   A' = relu(x*scale + shift), stored into side (+ ReLU bits)
      ("bn_bwd", y, mask, coef, side)        A' = coef[0]*(x . mask) + coef[1]*y + coef[2], stored into side

    w: [Co, 3, 3, C] bf16 — the forward filter, or with flip=True the transposed filter
    (K.krsc_to_crsk of the forward filter) of the conv whose data gradient this is.
    stat=True: per-tile BN partial sums of the output -> (out, partial, T); bn_stat=(y, mask):
    ReLU-masked gradient + BN-backward sums of the consuming unit -> (out, partial, T)."""
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w")
    Nimg, H, W, C = x.shape
    Co = w.shape[0]
    if tuple(w.shape) != (Co, 3, 3, C):
        raise ValueError("conv3_halo: filter must be [%d, 3, 3, %d], got %s" % (Co, C, tuple(w.shape)))
    pro_code = 0 if prologue is None else {"bn_fwd": 1, "bn_bwd": 2}.get(prologue[0], -1)
    bm = conv3_rows(H, W, C, Co, max(pro_code, 0))
    if not bm:
        raise ValueError("conv3_halo: shape %s -> %d not compiled in" % (tuple(x.shape), Co))
    if out is None:
        out = torch.empty((Nimg, H, W, Co), dtype=torch.bfloat16, device=x.device)
    T = -(-Nimg * H * W // bm)  # (the stage-3 variant's 8-row tiles may end in a partial one)
    partial = None
    by = bmask = None
    if stat or bn_stat is not None:
        partial = torch.empty((T, 2, Co), dtype=torch.float32, device=x.device)
    if bn_stat is not None:
        by, bmask = bn_stat
        _check(by, torch.bfloat16, "bn_stat y")
    e = _epi(out, ldo=Co, stat=partial, by=by, bmask=bmask)
    P = _lib.ptr
    pro, x2, mask_in, s, b, side, side_mask = 0, None, None, None, None, None, None
    if prologue is not None:
        if prologue[0] == "bn_fwd":
            _, s, b, side, side_mask = prologue
            pro = 1
        elif prologue[0] == "bn_bwd":
            _, x2, mask_in, s, side = prologue
            pro = 2
        else:
            raise ValueError("unknown prologue %r" % (prologue[0],))
    _log("c3_%s" % ("dgrad" if flip else "fwd"), Nimg * H * W, Co, 9 * C)
    _lib.call("ttdk_conv3_halo", x.data_ptr(), P(x2), P(mask_in), P(s), P(b), P(side), P(side_mask), pro, int(flip),
              w.data_ptr(), Nimg, H, W, C, Co, ctypes.byref(e), _lib.stream())
    if partial is not None:
        return out, partial, T
    return out


def gemm_f32(a, b, *, trans_a=False, trans_b=False, out=None, bias=None, beta=0):
    """Exact-fp32 C = op(a) @ op(b) (+bias[N]) (+C if beta) on the f32 MFMA (gemm_f32.hip).

    a: [M, K] (or [K, M] with trans_a); b: [K, N] (or [N, K] with trans_b); fp32 2-D with unit
    column stride. The fp32 MatMul of the reference MLP (distribute_training.py:54,61)."""
    _check2d(a, torch.float32, "a")
    _check2d(b, torch.float32, "b")
    M, K = (a.shape[1], a.shape[0]) if trans_a else a.shape
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else b.shape
    if K != Kb:
        raise ValueError("gemm inner dims differ: %d vs %d" % (K, Kb))
    if out is None:
        if beta:
            raise ValueError("beta=1 needs an out tensor")
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    elif out.dtype != torch.float32 or tuple(out.shape) != (M, N) or out.stride(-1) != 1:
        raise ValueError("gemm_f32 out must be fp32 [%d, %d] row-major" % (M, N))
    if bias is not None:
        _check(bias, torch.float32, "bias")
    _log("gemm_f32_%s%s" % ("t" if trans_a else "n", "t" if trans_b else "n"), M, N, K, 1)
    _lib.call("ttdk_gemm_f32", a.data_ptr(), a.stride(0), int(trans_a), b.data_ptr(), b.stride(0), int(trans_b),
              out.data_ptr(), out.stride(0), _lib.ptr(bias), int(bool(beta)), M, N, K, _lib.stream())
    return out


# workgroups a split-K weight gradient on the 256-row kernel aims for (one per CU: 256 = one
# wave over the chip; fewer leave CUs to the data-gradient chain it overlaps; TTD_WGRAD_WGS).
# ResNet-50 b1024 sweep (2 runs each): 64: 74.1, 96: 70.0, 128: 68.8, 160: 68.8, 256: 69.3 ms (round 3);
# after the untracked MN-major DMA (round 4, images/s): 96: 15,246 / 15,203, 112: 15,101 / 15,117,
# 128: 15,196 / 15,211 (15,227 / 15,173), 144: 15,118 / 15,143, 160: 15,086 / 15,099, 208: 15,056 /
# 15,121, 256: 15,004 / 15,099 -> 128
BIG_WGRAD_WGS = int(_os.environ.get("TTD_WGRAD_WGS", "128"))


def gemm_wgrad_splits(M, N, K, target_blocks=1024, min_ktiles=8, big_wgs=None):
    """Split-K factor for a weight-gradient GEMM (long K = tokens, small M x N). Mirrors the
    launcher's kernel choice: the 256x256 LDS-DMA kernel (M, N >= 256, M*N >= 2^20, one
    workgroup per CU -> aim for ~1-2 waves of 256 workgroups) or the 4-wave 128x128 kernel."""
    bbn = big_bn(M, N, K)
    if bbn:
        tiles = -(-M // 256) * -(-N // bbn)
        return max(1, min((K // 64) // 32, -(-(big_wgs or BIG_WGRAD_WGS) // tiles)))
    bm = 64 if M <= 64 else 128
    bn = 64 if N <= 64 else 128
    tiles = -(-M // bm) * -(-N // bn)
    ktiles = -(-K // 64)
    return max(1, min(ktiles // min_ktiles, -(-target_blocks // tiles)))


def conv_geom(x_shape, w_shape, stride, padding, dilation=(1, 1)):
    N, H, W, C = x_shape
    K, R, S, Cw = w_shape
    if C != Cw:
        raise ValueError("channel mismatch %d vs %d" % (C, Cw))
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    P = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
    Q = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
    g = _lib.ConvGeom(N, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw)
    return g


def pw_rows(N, K, dma=False):
    """Rows per output tile of the streaming pointwise kernel (pw_gemm.hip) for an N x K conv,
    or 0 when that kernel does not take the shape. dma: the launch has an accumulate / BN-statistics
    epilogue without residual or second statistics source (the LDS-DMA epilogue configuration)."""
    return int(_lib.query("ttdk_pw_rows", int(N), int(K), int(bool(dma))))


_PW = _os.environ.get("TTD_PW", "1") != "0"


def pw_ok(M, N, K):
    """The streaming pointwise kernel takes this GEMM (and is enabled: TTD_PW=0 turns it off)."""
    return _PW and pw_rows(N, K) > 0 and N * K <= 65536


def pw_wgrad_fusable(M, N, K, dma=True):
    """ops.gemm.pw_conv(..., wgrad=...) takes this (dz channels K, dx channels N) shape."""
    return _PW and int(_lib.query("ttdk_pw_wgrad_slabs", int(M), int(N), int(K), int(bool(dma)), 0)) > 0


def pw_conv(x, w, *, prologue=None, out=None, stat=False, beta=0, residual=None, bn_stat=None, bn_stat2=None,
            beta_s2=None, wgrad=None, max_wgs=0, fold_stream=None, keep=None):
    """Unit-stride 1x1 conv / dense GEMM out[M, N] = A'[M, K] . w[N, K]^T on the persistent
    streaming kernel (pw_gemm.hip), A' = prologue(x):

    prologue None                                    A' = x
    ("bn_fwd", scale, shift, residual, rscale, rshift, side, side_mask)
                                                     A' = relu(x*scale+shift [+ residual(*rscale+rshift)])
                                                     stored into `side` (+ ReLU bits into side_mask)
    ("bn_bwd", y, mask, coef, side)                  A' = a*(x . mask) + b*y + c, stored into `side`

    x: bf16 [..., K] contiguous (rows = the leading dims); w: bf16 [N, K] (or [N, 1, 1, K]).
    stat=True: also per-tile BN partial sums of the stored output -> returns (out, partial, T).
    bn_stat=(y, mask) [+ bn_stat2=y2]: dgrad-style ReLU-masked gradient + BN-backward sums of the
    consuming unit (see conv_dgrad) -> returns (out, partial, T[, partial2]).
    beta / residual / beta_s2: as conv_dgrad / gemm.
    wgrad=(xw, dw[, beta_w]) with the "bn_bwd" prologue (its side None): the same conv's weight
    gradient dw[K, N] (fp32; += when beta_w) = dz^T . xw is formed in the kernel from the dz tile
    in LDS (dz is never stored); xw: the conv input, bf16 [..., N] (pw_gemm.hip pw_kernel WG).
    max_wgs > 0 caps its persistent grid (launches on a side stream next to the main chain).
    fold_stream: fold the per-workgroup dw slabs on that stream (after a fork from the current
    one) instead of behind the kernel, so the data-gradient chain does not wait for the fold;
    the slab buffer is appended to `keep`, which must stay referenced until that stream joins."""
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w")
    K = x.shape[-1]
    M = x.numel() // K
    N = w.shape[0]
    if w.numel() != N * K:
        raise ValueError("pw_conv: weight must be [N, K] = [%d, %d] (got %s)" % (N, K, tuple(w.shape)))
    dma = bool(beta or bn_stat is not None) and residual is None and bn_stat2 is None
    bm = pw_rows(N, K, dma)
    if not bm:
        raise ValueError("pw_conv: N=%d K=%d not handled by the streaming kernel" % (N, K))
    if out is None:
        out = torch.empty(tuple(x.shape[:-1]) + (N,), dtype=torch.bfloat16, device=x.device)
    T = -(-M // bm)
    partial = partial2 = None
    by = bmask = by2 = None
    if stat or bn_stat is not None:
        partial = torch.empty((T, 2, N), dtype=torch.float32, device=x.device)
    if bn_stat is not None:
        by, bmask = bn_stat
        _check(by, torch.bfloat16, "bn_stat y")
        if bn_stat2 is not None:
            by2 = bn_stat2
            partial2 = torch.empty((T, 2, N), dtype=torch.float32, device=x.device)
    e = _epi(out, ldo=N, beta=beta, residual=residual, stat=partial, by=by, bmask=bmask, by2=by2, stat2=partial2,
             beta_s2=beta_s2 if beta else None)
    P = _lib.ptr
    pro, x2, mask_in, s, b, rs, rb, side, side_mask = 0, None, None, None, None, None, None, None, None
    if prologue is not None:
        if prologue[0] == "bn_fwd":
            _, s, b, x2, rs, rb, side, side_mask = prologue
            pro = 1
        elif prologue[0] == "bn_bwd":
            _, x2, mask_in, s, side = prologue
            pro = 2
        else:
            raise ValueError("pw_conv: unknown prologue %r" % (prologue[0],))
    _log("pw_%s" % ("fwd" if pro != 2 else "dgrad"), M, N, K)
    if wgrad is not None:
        xw, dw = wgrad[0], wgrad[1]
        beta_w = int(wgrad[2]) if len(wgrad) > 2 else 0
        if pro != 2 or side is not None:
            raise ValueError("pw_conv: wgrad= needs the bn_bwd prologue without a dz store")
        _check(xw, torch.bfloat16, "wgrad x")
        if xw.numel() != M * N or dw.dtype != torch.float32 or dw.numel() != K * N or not dw.is_contiguous():
            raise ValueError("pw_conv: wgrad x must be [M, N] = [%d, %d] bf16 and dw [K, N] fp32" % (M, N))
        slabs = int(_lib.query("ttdk_pw_wgrad_slabs", M, N, K, int(dma), int(max_wgs)))
        if slabs <= 0:
            raise ValueError("pw_conv: N=%d K=%d has no fused weight-gradient kernel" % (N, K))
        _log("pw_wgrad", K, N, M)
        ws = torch.empty(slabs * K * N, dtype=torch.float32, device=x.device)
        _lib.call("ttdk_pw_conv_wgrad", x.data_ptr(), P(x2), P(mask_in), P(s), xw.data_ptr(), w.data_ptr(), K, M, N,
                  K, ctypes.byref(e), None if fold_stream is not None else dw.data_ptr(), ws.data_ptr(), beta_w,
                  int(max_wgs), _lib.stream())
        if fold_stream is not None:
            # slab fold on the given (side) stream: the caller keeps ws alive until that stream joins
            from ..utils import graphs
            graphs.fork(torch.cuda.current_stream(), fold_stream)
            with torch.cuda.stream(fold_stream):
                _lib.call("ttdk_splitk_reduce", ws.data_ptr(), slabs, K * N, dw.data_ptr(), beta_w, _lib.stream())
            if keep is not None:
                keep.append(ws)
        if partial is None:
            return out
        if partial2 is not None:
            return out, partial, T, partial2
        return out, partial, T
    _lib.call("ttdk_pw_conv", x.data_ptr(), P(x2), P(mask_in), P(s), P(b), P(rs), P(rb), P(side), P(side_mask), 1, pro,
              w.data_ptr(), K, M, N, K, ctypes.byref(e), _lib.stream())
    if partial is None:
        return out
    if partial2 is not None:
        return out, partial, T, partial2
    return out, partial, T


def conv_fwd(x, w, stride=(1, 1), padding=(0, 0), *, out=None, residual=None, act=ACT_NONE,
             bias=None, stat=None, tile=(0, 0)):
    """y[N,P,Q,K] = conv(x[N,H,W,C], w[K,R,S,C]) with optional fused epilogue.

    stat: optional fp32 [ceil(N*P*Q/BM), 2, K] buffer receiving per-tile BN partial sums.
    """
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w")
    g = conv_geom(x.shape, w.shape, stride, padding)
    if out is None:
        out = torch.empty((g.N, g.P, g.Q, g.K), dtype=torch.bfloat16, device=x.device)
    _log("fwd_%dx%d_s%d" % (g.R, g.S, g.sh), g.N * g.P * g.Q, g.K, g.R * g.S * g.C)
    e = _epi(out, ldo=g.K, bias=bias, residual=residual, act=act, stat=stat)
    _lib.call("ttdk_conv_fwd", x.data_ptr(), w.data_ptr(), ctypes.byref(g), tile[0], tile[1], ctypes.byref(e),
              _lib.stream())
    return out


# forward convolutions on the 4-wave GEMM (gemm4w.hip ttdk_conv_fwd4w: SCHED 3 main loop, BN
# statistics from the register epilogue, im2col gather by the operand DMA). TTD_CONV4W: 1
# (default) where it measured faster than the 256-row kernel at b1024 (tools/conv4w_bench.py,
# profiles/r6_conv4w_bench_b1024.txt): >= 256 output channels, reduction K = R*S*C >= 1024 and
# K * N >= 512 * 1024 (the stage-4/5 3x3 convs 1.19-1.40x, stage-5 1x1 1.11-1.17x; the short-K
# shapes lose 3-12 % to the statistics epilogue); 2 every conv conv_fwd4w takes; 0 off.
_CONV4W = int(_os.environ.get("TTD_CONV4W", "1"))


def conv_fwd4w_pays(x_shape, w_shape, stride=(1, 1), padding=(0, 0)) -> bool:
    """The engine's policy for conv_fwd4w (TTD_CONV4W) on top of conv_fwd4w_ok."""
    if _CONV4W <= 0 or not conv_fwd4w_ok(x_shape, w_shape, stride, padding):
        return False
    K, N = w_shape[1] * w_shape[2] * w_shape[3], w_shape[0]
    return _CONV4W >= 2 or (N >= 256 and K >= 1024 and K * N >= 512 * 1024)


def conv_fwd4w_ok(x_shape, w_shape, stride=(1, 1), padding=(0, 0)) -> bool:
    """Whether conv_fwd4w takes this conv: C % 64 == 0, K % 8 == 0, R*S*C >= 128, operands in range."""
    g = conv_geom(tuple(x_shape), tuple(w_shape), stride, padding)
    xb = g.N * g.H * g.W * g.C * 2
    shift = (g.ph * g.W + g.pw) * g.C * 2
    return (g.C % 64 == 0 and g.K % 8 == 0 and g.R * g.S * g.C >= 128 and g.R * g.S <= 32
            and g.dh == 1 and g.dw == 1 and xb + shift < (1 << 31))


def conv_fwd4w(x, w, stride=(1, 1), padding=(0, 0), *, stat=True, out=None):
    """y[N,P,Q,K] = conv(x[N,H,W,C], w[K,R,S,C]) on the 4-wave kernel; with stat, also the BN
    partial sums of the stored output per 128-row block. Returns (y, partial [T, 2, K], T) (partial
    None without stat). Raises when the kernel does not take the conv (conv_fwd4w_ok)."""
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w")
    if not conv_fwd4w_ok(tuple(x.shape), tuple(w.shape), stride, padding):
        raise ValueError("conv_fwd4w does not take x %s, w %s" % (tuple(x.shape), tuple(w.shape)))
    g = conv_geom(x.shape, w.shape, stride, padding)
    M = g.N * g.P * g.Q
    if out is None:
        out = torch.empty((g.N, g.P, g.Q, g.K), dtype=torch.bfloat16, device=x.device)
    T = 2 * -(-M // 256)
    partial = torch.empty((T, 2, g.K), dtype=torch.float32, device=x.device) if stat else None
    e = _epi(out, ldo=g.K, stat=partial)
    _log("fwd4w_%dx%d_s%d" % (g.R, g.S, g.sh), M, g.K, g.R * g.S * g.C)
    _lib.call("ttdk_conv_fwd4w", x.data_ptr(), w.data_ptr(), ctypes.byref(g), ctypes.byref(e), _lib.stream())
    return out, partial, T


# unit-stride 3x3 data gradients with the feeding-BN epilogue on the 4-wave GEMM (gemm4w.hip
# ttdk_conv_dgrad4w: dy gathered as a forward conv with reversed taps). TTD_DGRAD4W: 1 (default)
# the long-K shapes (>= 256 input channels, R*S*K >= 1024, K * N >= 512 * 1024), 0 off.
_DGRAD4W = int(_os.environ.get("TTD_DGRAD4W", "1"))


def conv_dgrad4w_pays(x_shape, wt_shape, stride=(1, 1), padding=(0, 0)) -> bool:
    """conv_dgrad takes the 4-wave kernel for this unit-stride, non-pointwise data gradient."""
    C, R, S, K = wt_shape
    if _DGRAD4W <= 0 or tuple(stride) != (1, 1) or R * S == 1 or K % 64 or C % 8:
        return False
    g = conv_geom(tuple(x_shape), (K, R, S, C), stride, padding)
    if g.ph > R - 1 or g.pw > S - 1 or g.N * g.P * g.Q * K * 2 + ((R - 1 - g.ph) * g.Q + S - 1 - g.pw) * K * 2 >= (1 << 31):
        return False
    KK = R * S * K
    return _DGRAD4W >= 2 or (C >= 256 and KK >= 1024 and KK * C >= 512 * 1024)


def conv_fwd_bnpro_ok(x_shape, w_shape):
    """Whether conv_fwd_bnpro runs: a 1x1 unit-stride conv on the 256-row kernel."""
    N, H, W, C = x_shape
    K = w_shape[0]
    return (tuple(w_shape[1:3]) == (1, 1) and C % 64 == 0 and C == w_shape[3]
            and big_bn(N * H * W, K, C) != 0)


def conv_fwd_bnpro(y3, w, coef, res, h_out, mask_out, *, proj=False):
    """1x1 conv whose input is the RAW output y3 of the previous conv+BN+residual+ReLU unit: the
    kernel forms h = relu(sc*y3 + sh + res) (proj: + rsc*res + rsh) in LDS as its operand and
    stores h and its ReLU bits (the apply pass that would have produced them disappears).
    coef: fp32 [2, C] = (sc, sh) or [4, C] with proj. Returns (y, partial [T, 2, K], T): the
    conv output and its per-256-row-tile BN (sum, sum of squares)."""
    _check(y3, torch.bfloat16, "y3")
    _check(w, torch.bfloat16, "w")
    _check(res, torch.bfloat16, "res")
    if not conv_fwd_bnpro_ok(tuple(y3.shape), tuple(w.shape)):
        raise ValueError("conv_fwd_bnpro: needs a 1x1 conv on the 256-row kernel")
    if tuple(res.shape) != tuple(y3.shape) or tuple(h_out.shape) != tuple(y3.shape) or \
            mask_out.numel() * 8 != y3.numel() or coef.dtype != torch.float32 or not coef.is_contiguous() or \
            coef.numel() != (4 if proj else 2) * y3.shape[-1]:
        raise ValueError("conv_fwd_bnpro: operand shapes")
    g = conv_geom(y3.shape, w.shape, (1, 1), (0, 0))
    M = g.N * g.P * g.Q
    T = -(-M // 256)
    out = torch.empty((g.N, g.P, g.Q, g.K), dtype=torch.bfloat16, device=y3.device)
    partial = torch.empty((T, 2, g.K), dtype=torch.float32, device=y3.device)
    e = _epi(out, ldo=g.K, stat=partial)
    _log("fwd_bnpro_1x1", M, g.K, g.C)
    _lib.call("ttdk_conv_fwd_bnpro", y3.data_ptr(), w.data_ptr(), ctypes.byref(g), res.data_ptr(), coef.data_ptr(),
              1 if proj else 0, h_out.data_ptr(), mask_out.data_ptr(), ctypes.byref(e), _lib.stream())
    return out, partial, T


# strided (non-pointwise) dgrad via sub-pixel phase decomposition; TTD_SUBPIXEL_DGRAD=0 keeps
# the direct strided gather (A/B comparisons)
_SUBPIXEL = _os.environ.get("TTD_SUBPIXEL_DGRAD", "1") != "0"


def _phases(s, pad, R, H):
    """(taps, extent) of each sub-pixel phase along one axis (mirror of gemm_conv.hip phase_of)."""
    out = []
    for a in range(s):
        r0 = (a + pad) % s
        T = (R - r0 + s - 1) // s if r0 < R else 0
        n = (H - a + s - 1) // s if a < H else 0
        if n:
            out.append((T, n))
    return out


def _pick_tile(M, N):
    """Mirror of the C++ pick_tile() (4-wave kernel tile)."""
    return (64 if M <= 64 else 128), (64 if N <= 64 else 128)


def _subpixel_ok(g, R, S, stride, padding):
    return (_SUBPIXEL and not (R == 1 and S == 1 and tuple(padding) == (0, 0)) and g.sh == g.sw and g.sh > 1
            and R >= g.sh and S >= g.sw)


def dgrad_stat_rows(x_shape, wt_shape, stride=(1, 1), padding=(0, 0)):
    """Partial-sum rows the data-gradient launcher writes when its epilogue also emits the
    consuming BN's backward statistics (conv_dgrad(bn_stat=...)), or None when that fusion is
    not available (strided 1x1: only the sampled pixels are computed)."""
    C, R, S, K = wt_shape
    N, H, W, _ = x_shape
    if C % 8:
        return None
    if tuple(stride) != (1, 1):
        g = conv_geom(tuple(x_shape), (K, R, S, C), stride, padding)
        if not _subpixel_ok(g, R, S, stride, padding):
            return None
        return int(_lib.fn("ttdk_conv_dgrad_subpixel_stat_rows")(ctypes.byref(g)))
    return dgrad_stat_tile(x_shape, wt_shape)[2]


# short-K pointwise data gradients with the BN-statistics epilogue up to this K run on the
# 4-wave kernel instead of the 256-row one (TTD_DGRAD_STAT_4W_K; 0 = never)
DGRAD_STAT_4W_K = int(_os.environ.get("TTD_DGRAD_STAT_4W_K", "0"))


def dgrad_stat_tile(x_shape, wt_shape, stride=(1, 1), padding=(0, 0)):
    """(bm, bn, rows) of a unit-stride data-gradient launch with the BN-statistics epilogue
    (mirror of ttdk_conv_dgrad's tile choice when `stat` is set)."""
    C, R, S, K = wt_shape
    N, H, W, _ = x_shape
    if tuple(stride) != (1, 1):
        return None
    pointwise = R == 1 and S == 1 and tuple(padding) == (0, 0)
    M = N * H * W
    Kg = R * S * K
    bbn = big_bn(M, C, Kg)
    if pointwise and Kg <= DGRAD_STAT_4W_K:
        bbn = 0  # 4-wave kernel, two workgroups per CU (A/B: tools/dgrad_epi_ab.py)
    if bbn and (pointwise or K % 64 == 0):
        return 256, bbn, -(-M // 256)
    bm, bn = _pick_tile(M, C)
    return bm, bn, -(-M // bm)


def _bnpro_call(dy, wt, g, bn_pro, e):
    y, coef, dz = bn_pro
    C, R, S, K = wt.shape
    if not _lib.fn("ttdk_conv_dgrad_bnpro_ok")(ctypes.byref(g)):
        raise ValueError("conv_dgrad: the BN-backward operand prologue needs a 1x1 unit-stride dgrad on the 256-row "
                         "kernel")
    _check(y, torch.bfloat16, "bn_pro y")
    _check(dz, torch.bfloat16, "bn_pro dz")
    if tuple(y.shape) != tuple(dy.shape) or tuple(dz.shape) != tuple(dy.shape) or coef.dtype != torch.float32 \
            or coef.numel() != 3 * K or not coef.is_contiguous():
        raise ValueError("conv_dgrad: bn_pro operands must match dy ([..., K]) and coef [3, K] fp32")
    _log("dgrad_bnpro_1x1", g.N * g.H * g.W, C, K)
    _lib.call("ttdk_conv_dgrad_bnpro", dy.data_ptr(), wt.data_ptr(), ctypes.byref(g), y.data_ptr(), coef.data_ptr(),
              dz.data_ptr(), ctypes.byref(e), _lib.stream())


def dgrad_bnpro_ok(x_shape, wt_shape, stride=(1, 1), padding=(0, 0)):
    """Whether conv_dgrad(bn_pro=...) runs: a 1x1 unit-stride data gradient on the 256-row
    kernel (K % 64 == 0)."""
    C, R, S, K = wt_shape
    g = conv_geom(tuple(x_shape), (K, R, S, C), stride, padding)
    return bool(_lib.fn("ttdk_conv_dgrad_bnpro_ok")(ctypes.byref(g)))


def conv_dgrad(dy, wt, x_shape, stride=(1, 1), padding=(0, 0), *, out=None, beta=0, residual=None,
               tile=(0, 0), bn_stat=None, bn_stat2=None, sampled_only=False, beta_s2=None, bn_pro=None, ws=None):
    """dx[N,H,W,C] from dy[N,P,Q,K] and wt = w transposed to [C,R,S,K].

    For strided 1x1 convs only the sampled pixels are written: pass a zero-initialised `out`
    or beta=1 with `out` already holding another gradient contribution. sampled_only=True
    leaves the other pixels of a fresh `out` unwritten (no zero fill): its consumer must read
    it with beta_s2.

    beta_s2=(H, W): with beta=1, `out` is such a sampled-only gradient of an [N, H, W, C]
    tensor — the accumulate reads it only at pixels with h and w even and takes 0 elsewhere.

    bn_stat=(y, mask): dx is the output gradient of a conv+BN(+ReLU) unit whose pre-BN conv
    output is y (same shape as dx) and ReLU bit mask is `mask` (or None). The epilogue then
    stores g = dx * mask and per-tile BN-backward partial sums (sum g, sum g*y); returns
    (out, partial [T, 2, C], T). bn_stat2=y2: a second BN fed by the same g (projection
    shortcut); returns (out, partial, T, partial2). Requires dgrad_stat_rows(...) not None.

    ws: for a strided (sub-pixel) dgrad, the phase filters already gathered in the launcher's
    phase order (ops.kernels.WeightPrep, once per step): wt is then not read.
    """
    _check(dy, torch.bfloat16, "dy")
    _check(wt, torch.bfloat16, "wt")
    if beta_s2 is not None and beta and tuple(stride) != (1, 1):
        # the sampled-beta row test works on the GEMM row index, which only equals the output
        # pixel for unit-stride dgrads (strided ones remap rows to pixels / sub-pixel phases)
        raise ValueError("conv_dgrad: beta_s2 needs a unit-stride dgrad")
    C, R, S, K = wt.shape
    g = conv_geom(x_shape, (K, R, S, C), stride, padding)
    strided_pw = R == 1 and S == 1 and padding == (0, 0) and tuple(stride) != (1, 1)
    if out is None:
        alloc = torch.zeros if (strided_pw and not beta and not sampled_only) else torch.empty
        out = alloc(tuple(x_shape), dtype=torch.bfloat16, device=dy.device)
    if bn_stat is not None:
        y, mask = bn_stat
        T = dgrad_stat_rows(tuple(x_shape), tuple(wt.shape), stride, padding)
        if T is None or residual is not None or tuple(y.shape) != tuple(x_shape):
            raise ValueError("conv_dgrad: BN-statistics epilogue not available for this conv")
        _check(y, torch.bfloat16, "bn_stat y")
        partial = torch.empty((T, 2, C), dtype=torch.float32, device=dy.device)
        partial2 = None
        if bn_stat2 is not None:
            _check(bn_stat2, torch.bfloat16, "bn_stat2")
            if tuple(bn_stat2.shape) != tuple(x_shape) or tuple(stride) != (1, 1):
                raise ValueError("conv_dgrad: second BN statistics need a unit-stride dgrad of the same shape")
            partial2 = torch.empty((T, 2, C), dtype=torch.float32, device=dy.device)
        e = _epi(out, ldo=C, beta=beta, stat=partial, by=y, bmask=mask, by2=bn_stat2, stat2=partial2,
                 beta_s2=beta_s2 if beta else None)
        if tuple(stride) != (1, 1):
            if _LOG is not None:
                for pa in _phases(g.sh, g.ph, R, g.H):
                    for pb in _phases(g.sw, g.pw, S, g.W):
                        _log("dgrad_%dx%d_s%d_phase%dx%d" % (R, S, g.sh, pa[0], pb[0]), g.N * pa[1] * pb[1], C,
                             pa[0] * pb[0] * K)
            ready = ws is not None
            ws = torch.empty_like(wt) if ws is None else ws
            _lib.call("ttdk_conv_dgrad_subpixel", dy.data_ptr(), wt.data_ptr(), ctypes.byref(g), ws.data_ptr(),
                      int(ready), ctypes.byref(e), _lib.stream())
        elif bn_pro is not None:
            _bnpro_call(dy, wt, g, bn_pro, e)
        elif (not beta and partial2 is None and residual is None
              and conv_dgrad4w_pays(tuple(x_shape), tuple(wt.shape), stride, padding)):
            # the 4-wave kernel: statistics rows are 128-pixel blocks
            T = 2 * -(-(g.N * g.H * g.W) // 256)
            partial = torch.empty((T, 2, C), dtype=torch.float32, device=dy.device)
            e = _epi(out, ldo=C, stat=partial, by=y, bmask=mask)
            _log("dgrad4w_%dx%d_s1" % (R, S), g.N * g.H * g.W, C, R * S * K)
            _lib.call("ttdk_conv_dgrad4w", dy.data_ptr(), wt.data_ptr(), ctypes.byref(g), ctypes.byref(e),
                      _lib.stream())
        else:
            bm, bn, _ = dgrad_stat_tile(tuple(x_shape), tuple(wt.shape))
            _log("dgrad_%dx%d_s%d" % (R, S, stride[0]), g.N * g.H * g.W, C, R * S * K)
            _lib.call("ttdk_conv_dgrad", dy.data_ptr(), wt.data_ptr(), ctypes.byref(g), bm, bn, ctypes.byref(e),
                      _lib.stream())
        return (out, partial, T) if partial2 is None else (out, partial, T, partial2)
    e = _epi(out, ldo=C, beta=beta, residual=residual, beta_s2=beta_s2 if beta else None)
    if bn_pro is not None:
        _bnpro_call(dy, wt, g, bn_pro, e)
        return out
    if _subpixel_ok(g, R, S, stride, padding) and residual is None and tile == (0, 0):
        # strided dgrad as s*s unit-stride phase GEMMs (skips the zero taps of the direct gather)
        if _LOG is not None:  # one GEMM per phase, in ttdk_conv_dgrad_subpixel's launch order
            for pa in _phases(g.sh, g.ph, R, g.H):
                for pb in _phases(g.sw, g.pw, S, g.W):
                    _log("dgrad_%dx%d_s%d_phase%dx%d" % (R, S, g.sh, pa[0], pb[0]), g.N * pa[1] * pb[1], C,
                         pa[0] * pb[0] * K)
        ready = ws is not None
        ws = torch.empty_like(wt) if ws is None else ws
        _lib.call("ttdk_conv_dgrad_subpixel", dy.data_ptr(), wt.data_ptr(), ctypes.byref(g), ws.data_ptr(),
                  int(ready), ctypes.byref(e), _lib.stream())
        return out
    _log("dgrad_%dx%d_s%d" % (R, S, stride[0]), g.N * (g.P * g.Q if strided_pw else g.H * g.W), C, R * S * K)
    _lib.call("ttdk_conv_dgrad", dy.data_ptr(), wt.data_ptr(), ctypes.byref(g), tile[0], tile[1], ctypes.byref(e),
              _lib.stream())
    return out


_WGRAD_GATHER_X3 = _os.environ.get("TTD_WGRAD_GATHER_X3", "1") != "0"  # A/B switch


# split-K block target of the 4-wave weight-gradient kernel (im2col-gather / small-tile shapes):
# ResNet-50 b1024, interleaved pairs on one box: 256: 14,956 / 14,974, 512: 15,107 / 15,061,
# 1024: 15,053 / 15,008 images/s (fewer slab bytes competing with the HBM-bound main chain)
_WGRAD_TARGET_BLOCKS = int(_os.environ.get("TTD_WGRAD_TARGET_BLOCKS", "512"))


def wgrad_splits(g, target_blocks=None, min_ktiles=8):
    """Split-K factor for the weight gradient: enough blocks to fill 256 CUs twice, but every
    split keeps >= min_ktiles K-steps (the slab write + reduce is pure overhead)."""
    if target_blocks is None:
        target_blocks = _WGRAD_TARGET_BLOCKS
    M, N, K = g.K, g.R * g.S * g.C, g.N * g.P * g.Q
    bbn = big_bn_wgrad(M, N, K)
    if bbn:  # mirrors ttdk_conv_wgrad's choice of the 256-row LDS-DMA kernel
        # ~1 wave of 256 workgroups, but >= 32 K-tiles per split: fp32 slabs cost 8 B per output
        # element per split (write + reduce read)
        tiles = -(-M // 256) * -(-N // bbn)
        return max(1, min((K // 64) // 32, -(-BIG_WGRAD_WGS // tiles)))
    bm = 64 if M <= 64 else 128
    bn = 64 if N <= 64 else 128
    tiles = -(-M // bm) * -(-N // bn)
    ktiles = -(-K // 64)
    if (g.R > 1 or g.S > 1) and tiles <= 16 and _WGRAD_GATHER_X3:
        # im2col-gather wgrads with few output tiles (stem 7x7: 4, 3x3 64->64: 5, 128->128: 9)
        # are latency-bound on the gather: more blocks hide it (b1024, with the kernel's
        # split-major XCD order: stem 2.10 -> 1.6-1.8 ms — the last kernel of every backward —,
        # 3x3 64->64 0.70 -> 0.52 ms, 128->128 0.47 -> 0.42 ms; tools/wgrad_split_sweep.py)
        target_blocks *= 3 if tiles <= 8 else 2
    s = max(1, min(ktiles // min_ktiles, -(-target_blocks // tiles)))
    return s


# weight gradients on the 4-wave transposed-read kernel (gemm4t.hip: im2col gather of x for
# strided / 3x3 convs, split-K summed in the launch). TTD_WGRAD4T: 0 off; 1 (default) the convs
# where it measured faster standalone at b1024 (tools/wgrad4t_bench.py,
# profiles/r6_wgrad4t_bench_b1024.txt): filters larger than 1x1 with >= 256 output channels, and
# 1x1 convs with M, N >= 256 and M * N >= 512 * 1024 (the smaller 1x1 shapes have 4 output tiles
# and need 32-64 K-splits: the in-kernel sum of that many slabs by one workgroup outweighs the
# faster main loop); 2 every conv with M >= 256 and R*S*C >= 128; 3 the filters larger than 1x1 only.
_WGRAD4T = int(_os.environ.get("TTD_WGRAD4T", "1"))
# workgroup target per launch: 128 (in the two-stream step 256 for the 1x1 shapes, faster
# standalone, cost 0.5 ms: profiles/r6_wgrad4t_step_ab.txt); 0: per shape (128 3x3, 256 1x1)
_WGRAD4T_WGS = int(_os.environ.get("TTD_WGRAD4T_WGS", "128"))
_WGRAD4T_MIN_KT = int(_os.environ.get("TTD_WGRAD4T_MIN_KT", "32"))
# fp8 weight gradients (conv_wgrad_fp8) on the 4-wave transposed-read kernel's fp8 form
# (gemm4t.hip gemm4t8_kernel); TTD_WGRAD4T8=0: the 8-wave 256x128 kernel (conv_wgrad.hip)
_WGRAD4T8 = _os.environ.get("TTD_WGRAD4T8", "1") != "0"
# convs with fewer than 256 output channels (>= TTD_WGRAD4T_MINM) on the kernel's 128-row tile form
# (gemm4t.hip g4t_bm): TTD_WGRAD4T_SMALL "c3" the filters larger than 1x1, "all" the 1x1 ones too,
# "none" (default) the previous kernels. Measured (profiles/r6_wgrad4t_small_m.txt): the 128-row
# form needs 37 % less CU time on the stage-3 3x3 weight gradients (77 vs 121 CU-ms at 128
# workgroups) but holds each CU ~590 us; in the two-stream step the data-gradient chain waits
# for those CUs (66.61 / 66.79 vs 66.54 / 66.67 ms), so it stays opt-in
_WGRAD4T_SMALL = _os.environ.get("TTD_WGRAD4T_SMALL", "none")
_WGRAD4T_MINM = int(_os.environ.get("TTD_WGRAD4T_MINM", "128"))


def wgrad4t_rows(M: int) -> int:
    """Output rows per tile of the 4-wave weight-gradient kernel (mirror of gemm4t.hip g4t_bm)."""
    return 128 if (M <= 128 and _os.environ.get("TTD_G4T_BM128", "1") != "0") else 256


def conv_wgrad4t_splits(g, target_blocks=None, min_ktiles=None):
    """Split-K factor of the 4-wave weight gradient: ~target_blocks workgroups (the side stream
    shares the CUs with the data-gradient chain; default 128 for gathered filters, 256 for 1x1),
    >= min_ktiles K-tiles of 64 pixels per split."""
    target = target_blocks or _WGRAD4T_WGS or (128 if g.R * g.S > 1 else 256)
    mk = _WGRAD4T_MIN_KT if min_ktiles is None else min_ktiles
    M, N, K = g.K, g.R * g.S * g.C, g.N * g.P * g.Q
    bm = wgrad4t_rows(M)
    tiles = -(-M // bm) * -(-N // 256)
    return max(1, min((K // 64) // mk, -(-target // tiles)))


def conv_wgrad4t_ok(g, mode=None) -> bool:
    """Whether conv_wgrad runs this conv on the 4-wave kernel (TTD_WGRAD4T policy + the kernel's
    own admission: C, K % 8, pixels % 64, operands < 2 GiB, no dilation)."""
    mode = _WGRAD4T if mode is None else mode
    M, N = g.K, g.R * g.S * g.C
    if mode <= 0 or N < 128:
        return False
    if M < 256:
        if M < _WGRAD4T_MINM or mode == 3 and g.R * g.S == 1:
            return False
        if mode == 1 and (_WGRAD4T_SMALL == "none" or (_WGRAD4T_SMALL == "c3" and g.R * g.S == 1)
                          or (g.R * g.S > 1 and N < 256)):
            return False
    elif mode in (1, 3):
        if g.R * g.S == 1 and (mode == 3 or N < 256 or M * N < 512 * 1024):
            return False
        if g.R * g.S > 1 and N < 256:
            return False
    return int(_lib.query("ttdk_conv_wgrad4t_ws", ctypes.byref(g), 1)) >= 0


def conv_wgrad4t(x, dy, w_shape, stride=(1, 1), padding=(0, 0), *, out=None, beta=0, splits=None):
    """dw[K,R,S,C] (fp32) (+)= sum over pixels of dy x im2col(x) on the 4-wave transposed-read
    kernel (gemm4t.hip; the im2col of x gathered by the operand DMA, split-K summed inside the
    launch). Raises when the kernel does not take the conv (no silent fallback)."""
    _check(x, torch.bfloat16, "x")
    _check(dy, torch.bfloat16, "dy")
    g = conv_geom(x.shape, w_shape, stride, padding)
    if out is None:
        out = torch.empty(tuple(w_shape), dtype=torch.float32, device=x.device)
    if splits is None:
        splits = conv_wgrad4t_splits(g)
    nws = int(_lib.query("ttdk_conv_wgrad4t_ws", ctypes.byref(g), int(splits)))
    if nws < 0:
        raise ValueError("conv_wgrad4t does not take x %s, w %s, stride %s, pad %s"
                         % (tuple(x.shape), tuple(w_shape), stride, padding))
    ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x.device)
    _log("wgrad4t_%dx%d_s%d" % (g.R, g.S, g.sh), g.K, g.R * g.S * g.C, g.N * g.P * g.Q, splits)
    _lib.call("ttdk_conv_wgrad4t", x.data_ptr(), dy.data_ptr(), ctypes.byref(g), out.data_ptr(), ws.data_ptr(),
              int(splits), int(beta), _lib.stream())
    return out


def conv_wgrad(x, dy, w_shape, stride=(1, 1), padding=(0, 0), *, out=None, beta=0, splits=None,
               tile=(0, 0)):
    """dw[K,R,S,C] (fp32) = sum over pixels of dy x im2col(x). Convs the 4-wave kernel takes
    (conv_wgrad4t_ok) run there unless a split / tile is forced."""
    _check(x, torch.bfloat16, "x")
    _check(dy, torch.bfloat16, "dy")
    g = conv_geom(x.shape, w_shape, stride, padding)
    if splits is None and tile == (0, 0) and conv_wgrad4t_ok(g):
        return conv_wgrad4t(x, dy, w_shape, stride, padding, out=out, beta=beta)
    if out is None:
        out = torch.empty(tuple(w_shape), dtype=torch.float32, device=x.device)
    if splits is None:
        splits = wgrad_splits(g)
    _log("wgrad_%dx%d_s%d" % (g.R, g.S, g.sh), g.K, g.R * g.S * g.C, g.N * g.P * g.Q, splits)
    ws = None
    if splits > 1:
        ws = torch.empty((splits,) + tuple(w_shape), dtype=torch.float32, device=x.device)
    _lib.call("ttdk_conv_wgrad", x.data_ptr(), dy.data_ptr(), ctypes.byref(g), out.data_ptr(),
              ws.data_ptr() if ws is not None else None, splits, beta, tile[0], tile[1], _lib.stream())
    return out


def conv_wgrad_fp8_ok(x_shape, w_shape, stride=(1, 1), padding=(0, 0)):
    """Whether conv_wgrad_fp8 takes this weight gradient: C and K multiples of 16, the pixel
    count a multiple of 128, R*S*C >= 256, the fp8 input under 4 GiB."""
    g = conv_geom(tuple(x_shape), tuple(w_shape), stride, padding)
    pixels = g.N * g.P * g.Q
    return (g.C % 16 == 0 and g.K % 16 == 0 and pixels % 128 == 0 and g.R * g.S * g.C >= 256
            and g.N * g.H * g.W * g.C < (1 << 32))


def conv_wgrad_fp8(x8, dy8, w_shape, stride=(1, 1), padding=(0, 0), *, ascale, out=None, beta=0, splits=None):
    """fp8 weight gradient dw[K,R,S,C] (fp32) = sum over pixels of dy8 x im2col(x8): dy8 [N,P,Q,K]
    OCP e5m2, x8 [N,H,W,C] e4m3 (uint8 codes), ascale = (inverse scale of dy8, of x8) as device
    fp32 scalars (conv_wgrad_fp8.hip: both operands MN-major on the block-scaled fp8 MFMA)."""
    if x8.dtype != torch.uint8 or dy8.dtype != torch.uint8:
        raise ValueError("conv_wgrad_fp8 wants uint8 operands")
    if not conv_wgrad_fp8_ok(x8.shape, w_shape, stride, padding):
        raise ValueError("conv_wgrad_fp8: shape not supported (%s, %s)" % (tuple(x8.shape), tuple(w_shape)))
    g = conv_geom(x8.shape, w_shape, stride, padding)
    if out is None:
        out = torch.empty(tuple(w_shape), dtype=torch.float32, device=x8.device)
    M, N, K = g.K, g.R * g.S * g.C, g.N * g.P * g.Q
    # (1x1 convs with a 4-tile output or less need 64 K-splits whose in-kernel sum by one workgroup
    # outweighs the faster loop: 0.85-0.89x there, 1.33x at 512x2048; 3x3 1.27-1.54x:
    # tools/wgrad_fp8_bench.py, profiles/r6_wgrad_fp8_bench_b1024.txt)
    big1 = M >= 256 and N >= 256 and M * N >= 512 * 1024
    if (_WGRAD4T8 and (g.R * g.S > 1 or big1 or splits is not None)
            and int(_lib.query("ttdk_conv_wgrad4t8_ws", ctypes.byref(g), 1)) >= 0):
        # the 4-wave transposed-read kernel (gemm4t.hip gemm4t8_kernel: 32x32x64 fp8 MFMA, split-K
        # summed in the launch); splits sized like the bf16 one's (K-tiles of 128 pixels)
        if splits is None:
            tiles = -(-M // 256) * -(-N // 256)
            target = _WGRAD4T_WGS or (128 if g.R * g.S > 1 else 256)
            splits = max(1, min((K // 128) // max(1, _WGRAD4T_MIN_KT // 2), -(-target // tiles)))
        nws = int(_lib.query("ttdk_conv_wgrad4t8_ws", ctypes.byref(g), int(splits)))
        ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x8.device)
        _log("wgrad4t8_%dx%d_s%d" % (g.R, g.S, g.sh), M, N, K, splits)
        _lib.call("ttdk_conv_wgrad4t8", x8.data_ptr(), dy8.data_ptr(), ctypes.byref(g), out.data_ptr(), ws.data_ptr(),
                  int(splits), int(beta), ascale[0].data_ptr(), ascale[1].data_ptr(), _lib.stream())
        return out
    if splits is None:
        tiles = -(-M // 256) * -(-N // 128)
        splits = max(1, min((K // 128) // 16, -(-BIG_WGRAD_WGS // tiles)))
    _log("wgrad8_%dx%d_s%d" % (g.R, g.S, g.sh), M, N, K, splits)
    ws = None
    if splits > 1:
        ws = torch.empty((splits,) + tuple(w_shape), dtype=torch.float32, device=x8.device)
    _lib.call("ttdk_conv_wgrad_fp8", x8.data_ptr(), dy8.data_ptr(), ctypes.byref(g), out.data_ptr(),
              ws.data_ptr() if ws is not None else None, splits, beta, ascale[0].data_ptr(), ascale[1].data_ptr(),
              _lib.stream())
    return out


def conv_wgrad_bn_fusable(x_shape, w_shape, stride=(1, 1), padding=(0, 0)):
    """Whether conv_wgrad_bn runs for this conv (non-pointwise, 4-wave im2col-gather kernel)."""
    g = conv_geom(x_shape, w_shape, stride, padding)
    M, N, K = g.K, g.R * g.S * g.C, g.N * g.P * g.Q
    pointwise = g.R == 1 and g.S == 1 and g.sh == 1 and g.sw == 1 and g.ph == 0 and g.pw == 0
    return not pointwise and g.C % 8 == 0 and g.K % 8 == 0 and not big_bn_wgrad(M, N, K)


def conv_wgrad_bn(x, g_out, y, coef, w_shape, stride=(1, 1), padding=(0, 0), *, out=None, beta=0, splits=None):
    """conv_wgrad(x, dy) with dy = coef[0]*g_out + coef[1]*y + coef[2] per output channel (the
    BatchNorm backward of the conv's output, coef from ops.kernels.bn_backward_coef) applied as
    the kernel loads dy: the BN-backward result is never stored. conv_wgrad_bn_fusable() shapes."""
    _check(x, torch.bfloat16, "x")
    _check(g_out, torch.bfloat16, "g_out")
    _check(y, torch.bfloat16, "y")
    g = conv_geom(x.shape, w_shape, stride, padding)
    if out is None:
        out = torch.empty(tuple(w_shape), dtype=torch.float32, device=x.device)
    if splits is None:
        splits = wgrad_splits(g)
    ws = None
    if splits > 1:
        ws = torch.empty((splits,) + tuple(w_shape), dtype=torch.float32, device=x.device)
    _lib.call("ttdk_conv_wgrad_bn", x.data_ptr(), g_out.data_ptr(), y.data_ptr(), coef.data_ptr(), ctypes.byref(g),
              out.data_ptr(), ws.data_ptr() if ws is not None else None, splits, beta, 0, 0, _lib.stream())
    return out


def stem_fwd_ok(x_shape, w_shape, stride, padding, cin_real):
    """The ResNet stem shape the dedicated forward kernel (stem_fwd.hip) handles: 224 x 224 RGB
    stored with 8 channels, 64 7x7/2 filters."""
    return (len(x_shape) == 4 and tuple(x_shape[1:3]) == (224, 224) and x_shape[3] in (3, 8)
            and tuple(w_shape) == (64, 7, 7, 8)
            and tuple(stride) == (2, 2) and tuple(padding) == (3, 3) and cin_real <= 3)


def stem_fwd(x, w):
    """Stem convolution (7x7/2, pad 3) over the 3 real input channels of x [N,224,224,3 or 8] ->
    (y [N,112,112,64] bf16, partial [T,2,64] per-workgroup BN (sum, sum of squares) of y, T)."""
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w")
    N, H, W, _ = x.shape
    y = torch.empty((N, 112, 112, 64), dtype=torch.bfloat16, device=x.device)
    T = int(_lib.query("ttdk_stem_fwd_blocks", N))
    partial = torch.empty((T, 2, 64), dtype=torch.float32, device=x.device)
    _log("stem_fwd", N * 112 * 112, 64, 147)
    _lib.call("ttdk_stem_fwd", x.data_ptr(), w.data_ptr(), y.data_ptr(), partial.data_ptr(), N, H, W, x.shape[3],
              _lib.stream())
    return y, partial, T


def stem_wgrad_ok(x_shape, w_shape, stride, padding, cin_real):
    """The ResNet stem shape the dedicated weight-gradient kernel (stem_wgrad.hip) handles."""
    return (len(x_shape) == 4 and x_shape[-1] in (3, 8) and tuple(w_shape) == (64, 7, 7, 8) and tuple(stride) == (2, 2)
            and tuple(padding) == (3, 3) and cin_real <= 3)


def stem_wgrad(x, g_out, y, coef, *, out=None, beta=0):
    """Stem weight gradient with the stem BN backward on the fly: dz = coef[0]*g + coef[1]*y +
    coef[2], dW[64][7][7][8] = sum over pixels of dz x im2col(x) for the 3 real input channels
    (the padded channels get 0). x [N,H,W,3] or [N,H,W,8]; g_out / y [N,P,Q,64]."""
    _check(x, torch.bfloat16, "x")
    _check(g_out, torch.bfloat16, "g_out")
    _check(y, torch.bfloat16, "y")
    N, H, W, _ = x.shape
    P, Q = y.shape[1], y.shape[2]
    if out is None:
        out = torch.empty((64, 7, 7, 8), dtype=torch.float32, device=x.device)
    nb = int(_lib.query("ttdk_stem_wgrad_blocks", N, P, Q))
    ws = torch.empty(nb * 64 * 160 + 64 * 160, dtype=torch.float32, device=x.device)
    _log("stem_wgrad", 64, 147, N * P * Q)
    _lib.call("ttdk_stem_wgrad", x.data_ptr(), g_out.data_ptr(), y.data_ptr(), coef.data_ptr(), out.data_ptr(),
              ws.data_ptr(), N, H, W, P, Q, int(beta), x.shape[3], _lib.stream())
    return out


# ------------------------------------------------------------------ fp8 (gfx950 block-scaled MFMA)
_lib.register({
    "ttdk_conv_fwd_fp8": [_lib.P, _lib.P, _lib.G, _lib.I, _lib.E, _lib.P],
    "ttdk_gemm_fp8": [_lib.P, _lib.L, _lib.P, _lib.L, _lib.I, _lib.I, _lib.I, _lib.I, _lib.I, _lib.E, _lib.P],
    "ttdk_conv_dgrad_fp8": [_lib.P, _lib.P, _lib.G, _lib.E, _lib.P],
})


def gemm_fp8(a8, b8, *, alpha=1.0, out=None, out_dtype=torch.bfloat16, bias=None, act=ACT_NONE, residual=None,
             beta=0, splits=1, a_e5m2=False, aux=None):
    """C[M, N] = alpha * A[M, K] . B[N, K]^T with fp8 operands (uint8 storage: OCP e4m3, or
    e5m2 for A when a_e5m2); alpha carries the per-tensor dequantisation scales."""
    M, K = a8.shape
    N, Kb = b8.shape
    if K != Kb or a8.dtype != torch.uint8 or b8.dtype != torch.uint8:
        raise ValueError("gemm_fp8 wants uint8 [M,K] x [N,K]")
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=a8.device)
    if out.dtype == torch.float32:
        splits = effective_splits(K, splits, bk=128)
        if splits > 1:
            ws = torch.empty((splits, M, N), dtype=torch.float32, device=a8.device)
            e = _epi(ws, mode=1, ldo=N, slab_stride=M * N, alpha=alpha)
            _lib.call("ttdk_gemm_fp8", a8.data_ptr(), a8.stride(0), b8.data_ptr(), b8.stride(0), int(a_e5m2), M, N, K,
                      splits, ctypes.byref(e), _lib.stream())
            _lib.call("ttdk_splitk_reduce", ws.data_ptr(), splits, M * N, out.data_ptr(), beta, _lib.stream())
            return out
        e = _epi(out, mode=2, beta=beta, alpha=alpha)
    else:
        e = _epi(out, bias=bias, residual=residual, act=act, beta=beta, alpha=alpha, aux=aux)
    _lib.call("ttdk_gemm_fp8", a8.data_ptr(), a8.stride(0), b8.data_ptr(), b8.stride(0), int(a_e5m2), M, N, K, 1,
              ctypes.byref(e), _lib.stream())
    return out


def conv_fwd_fp8(x8, w8, stride=(1, 1), padding=(0, 0), *, alpha=1.0, out=None, stat=None, residual=None,
                 act=ACT_NONE, ascale=(None, None)):
    """fp8 e4m3 implicit-GEMM conv: x8 [N,H,W,C] uint8, w8 [K,R,S,C] uint8, C % 128 == 0; bf16
    output with the fused epilogue (stat rows per 256-pixel tile)."""
    g = conv_geom(x8.shape, w8.shape, stride, padding)
    if out is None:
        out = torch.empty((g.N, g.P, g.Q, g.K), dtype=torch.bfloat16, device=x8.device)
    M, N, K = g.N * g.P * g.Q, g.K, g.R * g.S * g.C
    bn = 256 if N >= 256 else 128
    _log("fwd8_%dx%d_s%d" % (g.R, g.S, g.sh), M, N, K)
    e = _epi(out, ldo=g.K, residual=residual, act=act, stat=stat, alpha=alpha, ascale=ascale)
    _lib.call("ttdk_conv_fwd_fp8", x8.data_ptr(), w8.data_ptr(), ctypes.byref(g), bn, ctypes.byref(e), _lib.stream())
    return out


# fp8 forward convs on the 4-wave kernel's fp8 K-major form (gemm4w.hip gemm4k8_kernel: 32x32x64
# block-scaled MFMA, implicit-GEMM DMA gather, BN statistics per 128 rows); TTD_CONV4K8=0: the
# 8-wave conv_fwd_fp8 kernel
_CONV4K8 = _os.environ.get("TTD_CONV4K8", "1") != "0"
# ... and the unit-stride fp8 data gradients with >= 1024-element reductions and >= 256 input
# channels (gemm4w.hip gemm4k8_kernel with reversed taps and the feeding-BN epilogue, its y / ReLU
# loads issued per column block ahead of the stores): ResNet-50 fp8 step 62.43 / 62.59 vs 63.55 /
# 63.34 ms with the 8-wave kernel (TTD_DGRAD4K8=0)
_DGRAD4K8 = _os.environ.get("TTD_DGRAD4K8", "1") != "0"
_DGRAD4K8_MINK = int(_os.environ.get("TTD_DGRAD4K8_MINK", "512"))  # (1024: 63.60 / 63.28 vs 63.32 / 62.98 ms)
_DGRAD4K8_MINC = int(_os.environ.get("TTD_DGRAD4K8_MINC", "256"))
# ... including the accumulating (shortcut-gradient) ones: TTD_DGRAD4K8_BETA=1 (the stage-4 c1 data
# gradients then: 63.88 / 63.82 vs 63.57 / 63.42 ms with them on the 8-wave kernel; off)
_DGRAD4K8_BETA = _os.environ.get("TTD_DGRAD4K8_BETA", "0") != "0"


def conv_fwd4k8_ok(x_shape, w_shape, stride=(1, 1), padding=(0, 0)) -> bool:
    """Whether conv_fwd4k8 takes this conv (mirror of ttdk_conv_fwd4k8's admission)."""
    if not _CONV4K8:
        return False
    g = conv_geom(tuple(x_shape), tuple(w_shape), stride, padding)
    M, N, K = g.N * g.P * g.Q, g.K, g.R * g.S * g.C
    xb = g.N * g.H * g.W * g.C + (g.ph * g.W + g.pw) * g.C
    return (g.C % 128 == 0 and N % 8 == 0 and N >= 8 and M >= 1 and g.R * g.S <= 32 and xb < (1 << 31)
            and (N + 256) * K < (1 << 32) and M * g.C < (1 << 32))


def conv_fwd4k8_pays(x_shape, w_shape, stride=(1, 1), padding=(0, 0)) -> bool:
    """The engine's policy: the 4-wave fp8 forward where it measured faster than the 8-wave one
    (tools/fp8_conv_ab.py, profiles/r6_fp8_conv_fwd_ab_b1024.txt): reductions of >= 1024 with >= 256
    output channels (stage-3/4 3x3 1.54x / 1.95x, 1024 -> 256 1x1 1.14x); the short-K and
    128-channel shapes are 0.75-0.92x."""
    K = w_shape[1] * w_shape[2] * w_shape[3]
    return conv_fwd4k8_ok(x_shape, w_shape, stride, padding) and K >= 1024 and w_shape[0] >= 256


def conv_fwd4k8(x8, w8, stride=(1, 1), padding=(0, 0), *, ascale, stat=True, out=None):
    """fp8 forward conv on the 4-wave kernel: x8 [N,H,W,C] e4m3 (uint8), w8 [K,R,S,C] e4m3, ascale
    = (inverse scale of x8, of w8) as device fp32 scalars; bf16 output. stat=True: also the BN
    partial sums of the stored output per 128 rows -> (out, partial [T][2][K], T = 2 ceil(M/256)).
    Raises when the kernel does not take the conv."""
    g = conv_geom(x8.shape, w8.shape, stride, padding)
    M = g.N * g.P * g.Q
    if out is None:
        out = torch.empty((g.N, g.P, g.Q, g.K), dtype=torch.bfloat16, device=x8.device)
    T = 2 * (-(-M // 256))
    partial = torch.empty((T, 2, g.K), dtype=torch.float32, device=x8.device) if stat else None
    _log("fwd4k8_%dx%d_s%d" % (g.R, g.S, g.sh), M, g.K, g.R * g.S * g.C)
    _lib.call("ttdk_conv_fwd4k8", x8.data_ptr(), w8.data_ptr(), ctypes.byref(g), out.data_ptr(),
              partial.data_ptr() if partial is not None else None, ascale[0].data_ptr(), ascale[1].data_ptr(),
              _lib.stream())
    return (out, partial, T) if stat else out


def conv_dgrad_fp8_ok(x_shape, wt_shape, stride=(1, 1), padding=(0, 0)):
    """Whether conv_dgrad_fp8 takes this data gradient: unit stride, the output gradient's
    channels (wt_shape[-1]) a multiple of 128, wt_shape = [C, R, S, K]."""
    C, R, S, K = wt_shape
    return tuple(stride) == (1, 1) and K % 128 == 0 and C % 8 == 0


def conv_dgrad_fp8(dy8, wt8, x_shape, stride=(1, 1), padding=(0, 0), *, ascale, out=None, beta=0, bn_stat=None,
                   beta_s2=None):
    """fp8 data gradient: dy8 [N,P,Q,K] OCP e5m2 (uint8), wt8 [C,R,S,K] e4m3 (uint8), unit
    stride; ascale = (inv scale of dy8, inv scale of wt8) as device fp32 scalars. Epilogues as
    conv_dgrad: beta accumulate (beta_s2 sampled rows), bn_stat=(y, mask) -> (out, partial, T)
    with 256-row statistics tiles."""
    if dy8.dtype != torch.uint8 or wt8.dtype != torch.uint8:
        raise ValueError("conv_dgrad_fp8 wants uint8 operands")
    C, R, S, K = wt8.shape
    if not conv_dgrad_fp8_ok(x_shape, wt8.shape, stride, padding):
        raise ValueError("conv_dgrad_fp8: unit stride and K % 128 == 0 required")
    g = conv_geom(tuple(x_shape), (K, R, S, C), stride, padding)
    if out is None:
        out = torch.empty(tuple(x_shape), dtype=torch.bfloat16, device=dy8.device)
    M = g.N * g.H * g.W
    if (_DGRAD4K8 and (not beta or (_DGRAD4K8_BETA and bn_stat is not None and beta_s2 is None))
            and R * S * K >= _DGRAD4K8_MINK and C >= _DGRAD4K8_MINC):
        # the 4-wave fp8 kernel (gemm4w.hip gemm4k8_kernel, reversed-tap gather of dy8) on the
        # long-reduction shapes; its statistics come per 128 rows
        T = 2 * (-(-M // 256))
        y, mask = bn_stat if bn_stat is not None else (None, None)
        partial = torch.empty((T, 2, C), dtype=torch.float32, device=dy8.device) if bn_stat is not None else None
        _log("dgrad4k8_%dx%d_s%d" % (R, S, stride[0]), M, C, R * S * K)
        _lib.call("ttdk_conv_dgrad4k8", dy8.data_ptr(), wt8.data_ptr(), ctypes.byref(g), out.data_ptr(),
                  y.data_ptr() if y is not None else None, mask.data_ptr() if mask is not None else None,
                  partial.data_ptr() if partial is not None else None, int(bool(beta)), ascale[0].data_ptr(),
                  ascale[1].data_ptr(), _lib.stream())
        return (out, partial, T) if bn_stat is not None else out
    _log("dgrad8_%dx%d_s%d" % (R, S, stride[0]), M, C, R * S * K)
    if bn_stat is not None:
        y, mask = bn_stat
        T = -(-M // 256)
        partial = torch.empty((T, 2, C), dtype=torch.float32, device=dy8.device)
        e = _epi(out, ldo=C, beta=beta, stat=partial, by=y, bmask=mask, beta_s2=beta_s2 if beta else None,
                 ascale=ascale)
        _lib.call("ttdk_conv_dgrad_fp8", dy8.data_ptr(), wt8.data_ptr(), ctypes.byref(g), ctypes.byref(e),
                  _lib.stream())
        return out, partial, T
    e = _epi(out, ldo=C, beta=beta, beta_s2=beta_s2 if beta else None, ascale=ascale)
    _lib.call("ttdk_conv_dgrad_fp8", dy8.data_ptr(), wt8.data_ptr(), ctypes.byref(g), ctypes.byref(e), _lib.stream())
    return out
