"""ctypes bindings for ``libttd_hip.so`` (the gfx950 kernel library).

Every kernel launcher has the C signature ``int ttdk_*(..., hipStream_t)``; this module
declares the argument types once and launches on PyTorch's *current* HIP stream, so the
kernels compose with torch's stream semantics, ``torch.cuda.graphs`` capture (hipGraph) and
the collective engine's side streams. A non-zero return (hipError_t) raises immediately.

There is deliberately no fallback here: a GPU op whose kernel library is missing or fails
to load raises (the CPU path of each op lives in :mod:`.reference`).
"""
from __future__ import annotations

import ctypes
from ctypes import c_float, c_int, c_longlong, c_uint64, c_void_p

import torch

from .. import _native

P = c_void_p
I = c_int
L = c_longlong
F = c_float
U64 = c_uint64


class Epilogue(ctypes.Structure):
    """Mirror of ``TtdkEpilogue`` in gemm_conv.hip."""

    _fields_ = [
        ("mode", c_int), ("out", c_void_p), ("ldo", c_longlong), ("slab_stride", c_longlong),
        ("bias", c_void_p), ("residual", c_void_p), ("ldr", c_longlong), ("act", c_int),
        ("beta", c_int), ("remap", c_int), ("rP", c_int), ("rQ", c_int), ("rOH", c_int),
        ("rOW", c_int), ("rs", c_int), ("stat", c_void_p), ("alpha", c_float), ("aux", c_void_p),
        ("ascale0", c_void_p), ("ascale1", c_void_p), ("by", c_void_p), ("bmask", c_void_p),
        ("by2", c_void_p), ("stat2", c_void_p), ("bH", c_int), ("bW", c_int),
    ]


class ConvGeom(ctypes.Structure):
    """Mirror of ``TtdkConv``: input NHWC [N,H,W,C], filter [K,R,S,C], output [N,P,Q,K]."""

    _fields_ = [(n, c_int) for n in ("N", "H", "W", "C", "K", "R", "S", "P", "Q", "sh", "sw", "ph", "pw", "dh", "dw")]


E = ctypes.POINTER(Epilogue)
G = ctypes.POINTER(ConvGeom)

# name -> argtypes (restype is always int = hipError_t). Structs are passed by reference.
_SIGS = {
    # gemm_conv.hip
    "ttdk_gemm_bf16": [P, L, I, P, L, I, I, I, I, I, I, I, E, P],
    "ttdk_gemm_bf16_splitk": [P, L, I, P, L, I, I, I, I, I, P, P, I, F, I, I, P],
    "ttdk_gemm_wgrad_bias": [P, L, P, L, I, I, I, I, P, P, I, F, P, P],
    "ttdk_gemm_wgrad_bias_ws": [I, I, I, I],
    "ttdk_gemm4t_wgrad": [P, L, P, L, I, I, I, I, P, P, I, F, P, P],
    "ttdk_gemm4t_ws": [I, I, I, I],
    "ttdk_conv_fwd": [P, P, G, I, I, E, P],
    "ttdk_conv_fwd4w": [P, P, G, E, P],
    "ttdk_conv_dgrad4w": [P, P, G, E, P],
    "ttdk_conv_dgrad": [P, P, G, I, I, E, P],
    "ttdk_conv_dgrad_bnpro": [P, P, G, P, P, P, E, P],
    "ttdk_conv_dgrad_bnpro_ok": [G],
    "ttdk_set_inkernel_fold": [I],
    "ttdk_conv_fwd_bnpro": [P, P, G, P, P, I, P, P, E, P],
    "ttdk_conv_dgrad_subpixel": [P, P, G, P, I, E, P],
    "ttdk_conv_dgrad_subpixel_stat_rows": [G],
    "ttdk_conv_wgrad": [P, P, G, P, P, I, I, I, I, P],
    "ttdk_conv_wgrad4t": [P, P, G, P, P, I, I, P],
    "ttdk_conv_wgrad4t_ws": [G, I],
    "ttdk_conv_wgrad_bn": [P, P, P, P, G, P, P, I, I, I, I, P],
    "ttdk_conv_wgrad_fp8": [P, P, G, P, P, I, I, P, P, P],
    "ttdk_conv_wgrad4t8": [P, P, G, P, P, I, I, P, P, P],
    "ttdk_conv_fwd4k8": [P, P, G, P, P, P, P, P],
    "ttdk_conv_dgrad4k8": [P, P, G, P, P, P, P, I, P, P, P],
    "ttdk_conv_wgrad4t8_ws": [G, I],
    "ttdk_splitk_reduce": [P, I, L, P, I, P],
    "ttdk_set_big_pers": [I],
    # gemm_f32.hip
    "ttdk_gemm_f32": [P, L, I, P, L, I, P, L, P, I, I, I, I, P],
    # stem_fwd.hip / stem_wgrad.hip
    "ttdk_stem_fwd_blocks": [I],
    "ttdk_stem_fwd": [P, P, P, P, I, I, I, I, P],
    "ttdk_stem_wgrad_blocks": [I, I, I],
    "ttdk_stem_wgrad": [P, P, P, P, P, P, I, I, I, I, I, I, I, P],
    # conv3_halo.hip
    "ttdk_conv3_rows": [I, I, I, I, I],
    "ttdk_conv3_halo": [P, P, P, P, P, P, P, I, I, P, I, I, I, I, I, E, P],
    # pw_gemm.hip
    "ttdk_pw_rows": [I, I, I],
    "ttdk_pw_conv": [P, P, P, P, P, P, P, P, P, I, I, P, L, I, I, I, E, P],
    "ttdk_pw_wgrad_slabs": [I, I, I, I, I],
    "ttdk_pw_conv_wgrad": [P, P, P, P, P, P, L, I, I, I, E, P, P, I, I, P],
    # batchnorm.hip
    "ttdk_bn_num_partials": [L, I],
    "ttdk_bn_stats_partial": [P, L, I, P, I, P],
    "ttdk_bn_bwd_partial": [P, P, P, P, L, I, P, I, P, P],
    "ttdk_bn_reduce_partials": [P, I, I, P, P],
    "ttdk_bn_fwd_finalize": [P, F, I, P, P, F, F, P, P, P, P, P, P, P],
    "ttdk_bn_finalize_slices": [I],
    "ttdk_bn_reduce_finalize": [P, I, I, P, I, F, P, P, F, F, P, P, P, P, P, P, P, P, P, I, P],
    "ttdk_bn_bwd_finalize": [P, F, I, P, P, P, P, P, P, I, P],
    "ttdk_bn_apply": [P, P, P, P, P, P, P, P, P, P, L, I, I, P],
    "ttdk_bn_bwd_apply": [P, P, P, P, P, P, L, I, P],
    "ttdk_bn_bwd_apply_q8": [P, P, P, P, P, P, P, P, L, I, P],
    # pool.hip
    "ttdk_maxpool_fwd": [P, P, P] + [I] * 12 + [P],
    "ttdk_maxpool_bwd": [P, P, P] + [I] * 12 + [P],
    "ttdk_avgpool_fwd": [P, P, P, I, I, I, P],
    "ttdk_bn_relu_maxpool": [P, P, P, P, P, P, I, I, I, I, I, I, P],
    "ttdk_maxpool_bwd_bnstat_blocks": [I, I, I, I],
    "ttdk_maxpool_bwd_bnstat": [P, P, P, P, P, P, I, I, I, I, I, I, P],
    "ttdk_avgpool_bwd": [P, P, I, I, I, P],
    # xent.hip
    "ttdk_sparse_xent": [P, I, P, I, I, I, F, P, P, P, P, P, P],
    # optim.hip
    "ttdk_opt_sgd": [P, P, P, P, P, I, P, P, P, I, P],
    "ttdk_opt_adam": [P, P, P, P, P, P, I, P, P, P, I, P],
    "ttdk_opt_lamb": [P, P, P, P, P, P, P, I, I, P, P, P, P, P, P],
    "ttdk_sumsq": [P, L, P, P, P],
    "ttdk_lr_schedule": [P, P, I, P, F, F, I, P],
    # elementwise.hip
    "ttdk_f32_to_bf16": [P, P, L, P],
    "ttdk_bf16_to_f32": [P, P, L, P],
    "ttdk_bf16_round_probe": [P, P, P, P, L, P],
    "ttdk_pad_channels": [P, P, L, I, I, P],
    "ttdk_unpad_channels": [P, P, L, I, I, P],
    "ttdk_transpose_aca_bf16": [P, P, I, I, I, P],
    "ttdk_transpose128_batch_bf16": [P, I, I, P],
    "ttdk_wprep": [P, P, P, I, I, P],
    "ttdk_transpose2d_f32": [P, P, I, I, P],
    "ttdk_bias_act_dropout_fwd": [P, P, P, L, I, I, F, U64, U64, I, P],
    "ttdk_bias_act_dropout_bwd": [P, P, P, P, L, I, I, F, U64, U64, I, P],
    "ttdk_colsum": [P, L, I, P, I, I, P, P],
    "ttdk_colsum_ws_floats": [L, I, I],
    "ttdk_add_bf16": [P, P, P, L, F, F, P],
    "ttdk_amax_bf16": [P, L, P, I, P],
    "ttdk_quant_fp8": [P, P, L, P, I, P],
    "ttdk_dequant_fp8": [P, P, L, P, I, P],
    # fp8.hip
    "ttdk_fp8_rollover": [P, I, F, F, P],
    "ttdk_fp8_quant_weights": [P, P, P, I, I, P, I, P],
}

_fns = {}


def register(sigs: dict):
    _SIGS.update(sigs)


_RESTYPE = {"ttdk_conv_dgrad_subpixel_stat_rows": c_longlong, "ttdk_colsum_ws_floats": c_longlong,
            "ttdk_gemm_wgrad_bias_ws": c_longlong, "ttdk_gemm4t_ws": c_longlong,
            "ttdk_conv_wgrad4t_ws": c_longlong, "ttdk_conv_wgrad4t8_ws": c_longlong}


def fn(name):
    f = _fns.get(name)
    if f is None:
        lib = _native.hip()
        f = getattr(lib, name)
        f.argtypes = _SIGS[name]
        f.restype = _RESTYPE.get(name, c_int)
        _fns[name] = f
    return f


class HipKernelError(RuntimeError):
    pass


# Per-launch timing for profiling tools (TTD_OP_TIMING=1): every call is bracketed by HIP
# events on the current stream and labelled with the GEMM shapes ops.gemm logged for it.
import os as _os
TIMING = [] if _os.environ.get("TTD_OP_TIMING") else None
_labels = []


def label(x):
    if TIMING is not None:
        _labels.append(x)


def call(name, *args):
    if TIMING is not None:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn(name)(*args)
        e.record()
        TIMING.append((name, list(_labels), s, e))
        _labels.clear()
    else:
        rc = fn(name)(*args)
    if rc != 0:
        raise HipKernelError("%s failed with hipError_t %d" % (name, rc))


def query(name, *args):
    """Call a host-side helper that returns a plain int (not a hipError_t)."""
    return fn(name)(*args)


def stream():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return None if t is None else c_void_p(t.data_ptr())
