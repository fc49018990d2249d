"""Launch wrappers for the transformer kernels (attention.hip, transformer.hip) plus exact
CPU re-implementations of their dropout hash (used by the numerics tests as oracles).

All device tensors are bf16 token-major [tokens, features] unless noted; statistics fp32.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import F, I, L, P

_lib.register({
    "ttdk_attn_fwd": [P, L, P, L, P, L, P, L, P, P, I, I, I, F, P, I, P],
    "ttdk_attn_bwd": [P, L, P, L, P, L, P, L, P, L, P, P, P, L, P, L, P, L, P, I, I, I, F, P, I, P],
    "ttdk_attn_set_fused_bwd": [I],
    "ttdk_ln_fwd": [P, P, P, P, P, P, P, P, I, I, F, F, I, F, I, P, P],
    "ttdk_ln_bwd_num_blocks": [I],
    "ttdk_ln_bwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, F, I, F, I, P, P],
    "ttdk_colreduce": [P, I, I, I, P, I, P],
    "ttdk_embed_fwd": [P, P, P, P, P, P, L, I, I, P],
    "ttdk_embed_bwd": [P, P, P, P, P, P, I, I, I, I, I, P],
    "ttdk_gather_rows": [P, L, P, I, L, P, I, I, P],
    "ttdk_scatter_rows": [P, P, I, L, P, L, I, I, I, P],
    "ttdk_rng_advance": [P, P],
    "ttdk_count_valid": [P, I, F, P, P],
    "ttdk_count_valid2": [P, I, F, P, P],
    "ttdk_xent_vocab": [P, L, I, P, I, P, P, P, P, P],
    "ttdk_tanh_bf16": [P, L, P],
    "ttdk_dact_bf16": [P, P, P, L, I, P],
})


def _p(t):
    return None if t is None else t.data_ptr()


def _s():
    return _lib.stream()


class RngState:
    """Device-resident dropout RNG state [seed, step]. Kernels read it from HBM, so a
    hipGraph-captured step draws new masks after `advance()` (itself a captured kernel)."""

    def __init__(self, seed: int, device):
        self.t = torch.tensor([int(seed), 0], dtype=torch.int64, device=device)

    def advance(self):
        if self.t.is_cuda:
            _lib.call("ttdk_rng_advance", self.t.data_ptr(), _s())
        else:
            self.t[1:2].add_(1)

    def host(self):
        v = self.t.cpu().tolist()
        return int(v[0]), int(v[1])


# ------------------------------------------------------------------ attention
def attention_fwd(q, k, v, out, lse, B, H, S, *, seqlen=None, p_drop=0.0, rng=None, site=0):
    """q/k/v/out: 2-D bf16 views [B*S, >= H*64] (row stride = .stride(0)); lse fp32 [B*H, S]."""
    _lib.call("ttdk_attn_fwd", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0),
              out.data_ptr(), out.stride(0), lse.data_ptr(), _p(seqlen), B, H, S, float(p_drop),
              _p(rng.t if rng is not None else None), int(site), _s())
    return out, lse


def set_fused_attention_bwd(on: bool):
    """Select the single-kernel attention backward (S in {128, 256, 512}; opt-in, measured slower
    at BERT-Large: attention.hip) or the split dQ / dK-dV kernels (default;
    TTD_ATTN_FUSED_BWD=1 at start-up selects the fused one)."""
    _lib.call("ttdk_attn_set_fused_bwd", int(bool(on)))


def attention_bwd(q, k, v, o, dout, lse, dq, dk, dv, B, H, S, *, delta=None, seqlen=None, p_drop=0.0, rng=None,
                  site=0):
    if delta is None:
        delta = torch.empty((B * H, S), dtype=torch.float32, device=q.device)
    _lib.call("ttdk_attn_bwd", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0),
              o.data_ptr(), o.stride(0), dout.data_ptr(), dout.stride(0), lse.data_ptr(), delta.data_ptr(),
              dq.data_ptr(), dq.stride(0), dk.data_ptr(), dk.stride(0), dv.data_ptr(), dv.stride(0), _p(seqlen),
              B, H, S, float(p_drop), _p(rng.t if rng is not None else None), int(site), _s())
    return dq, dk, dv


# ------------------------------------------------------------------ LayerNorm
def layernorm_fwd(x, gamma, beta, *, res=None, eps=1e-12, p_in=0.0, site_in=0, p_out=0.0, site_out=0, rng=None,
                  save_s=True, out=None, s_out=None, mean=None, rstd=None):
    rows, H = x.shape
    dev = x.device
    out = out if out is not None else torch.empty_like(x)
    need_s = save_s and (res is not None or p_in > 0)
    s_out = s_out if s_out is not None else (torch.empty_like(x) if need_s else None)
    mean = mean if mean is not None else torch.empty(rows, dtype=torch.float32, device=dev)
    rstd = rstd if rstd is not None else torch.empty(rows, dtype=torch.float32, device=dev)
    _lib.call("ttdk_ln_fwd", x.data_ptr(), _p(res), _p(s_out), out.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), rows, H, float(eps), float(p_in), int(site_in), float(p_out),
              int(site_out), _p(rng.t if rng is not None else None), _s())
    return out, (s_out if s_out is not None else x), mean, rstd


def ln_bwd_workspace(rows, H, device):
    nb = _lib.query("ttdk_ln_bwd_num_blocks", rows)
    return torch.empty((nb, 2, H), dtype=torch.float32, device=device)


def layernorm_bwd(dy, s, mean, rstd, gamma, dgamma, dbeta, *, ds_out=None, want_dx=False, accumulate=False,
                  p_in=0.0, site_in=0, p_out=0.0, site_out=0, rng=None, work=None, dx_out=None):
    rows, H = dy.shape
    ds_out = ds_out if ds_out is not None else torch.empty_like(dy)
    if want_dx and dx_out is None:
        dx_out = torch.empty_like(dy)
    work = work if work is not None else ln_bwd_workspace(rows, H, dy.device)
    _lib.call("ttdk_ln_bwd", dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(),
              ds_out.data_ptr(), _p(dx_out if want_dx else None), work.data_ptr(), dgamma.data_ptr(),
              dbeta.data_ptr(), int(accumulate), rows, H, float(p_in), int(site_in), float(p_out), int(site_out),
              _p(rng.t if rng is not None else None), _s())
    return ds_out, (dx_out if want_dx else None)


# ------------------------------------------------------------------ embeddings / rows
def embed_fwd(ids, tt, word, pos, typ, S, out=None):
    rows = ids.numel()
    H = word.shape[1]
    out = out if out is not None else torch.empty((rows, H), dtype=torch.bfloat16, device=ids.device)
    _lib.call("ttdk_embed_fwd", ids.data_ptr(), _p(tt), word.data_ptr(), pos.data_ptr(), typ.data_ptr(),
              out.data_ptr(), rows, S, H, _s())
    return out


def embed_bwd(ds, ids, tt, dword, dpos, dtype, B, S, pos_beta=0):
    H = ds.shape[1]
    T = dtype.shape[0] if dtype is not None else 0
    _lib.call("ttdk_embed_bwd", ds.data_ptr(), ids.data_ptr(), _p(tt), dword.data_ptr(), dpos.data_ptr(),
              _p(dtype), B, S, H, T, int(pos_beta), _s())


def gather_rows(src, idx, out=None, *, group=(1, 0), n=None):
    """out[r] = src[(idx[r] if idx is not None else 0) + (r // per) * gs], group = (per, gs): e.g.
    per-sequence positions [B, P] of a [B*S, H] activation with group = (P, S); idx None and
    group (1, S) picks every sequence's first row. idx: contiguous int32."""
    per, gs = group
    n = idx.numel() if idx is not None else n
    H = src.shape[1]
    out = out if out is not None else torch.empty((n, H), dtype=src.dtype, device=src.device)
    _lib.call("ttdk_gather_rows", src.data_ptr(), src.stride(0), _p(idx), int(per), int(gs), out.data_ptr(), n, H,
              _s())
    return out


def scatter_rows(src, idx, dst, accumulate=False, *, group=(1, 0)):
    """dst[(idx[r] or 0) + (r // per) * gs] (+)= src[r] (the inverse of gather_rows)."""
    n, H = src.shape
    per, gs = group
    _lib.call("ttdk_scatter_rows", src.data_ptr(), _p(idx), int(per), int(gs), dst.data_ptr(), dst.stride(0), n, H,
              int(accumulate), _s())
    return dst


def count_valid(labels, scale, out):
    _lib.call("ttdk_count_valid", labels.data_ptr(), labels.numel(), float(scale), out.data_ptr(), _s())
    return out


def count_valid2(labels, scale, out):
    """out[0] = 1 / count, out[1] = scale / count (count = labels >= 0), one launch."""
    _lib.call("ttdk_count_valid2", labels.data_ptr(), labels.numel(), float(scale), out.data_ptr(), _s())
    return out


def xent_vocab(logits, V, labels, gscale, *, dlogits=None, sums=None, mscale=None):
    rows = logits.shape[0]
    _lib.call("ttdk_xent_vocab", logits.data_ptr(), logits.stride(0), int(V), labels.data_ptr(), rows,
              gscale.data_ptr(), _p(dlogits), _p(sums), _p(mscale), _s())
    return dlogits


def dact(dy, aux, kind, out=None):
    """dy * act'(aux): kind 0 = tanh-GELU (aux = pre-activation), 1 = tanh (aux = tanh output)."""
    out = out if out is not None else torch.empty_like(dy)
    _lib.call("ttdk_dact_bf16", dy.data_ptr(), aux.data_ptr(), out.data_ptr(), dy.numel(), int(kind), _s())
    return out


def tanh_(x):
    _lib.call("ttdk_tanh_bf16", x.data_ptr(), x.numel(), _s())
    return x


# ------------------------------------------------------------------ CPU mirror of the dropout hash
M32 = np.uint64(0xFFFFFFFF)


def _fmix32(h):
    h = np.asarray(h, dtype=np.uint64) & M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & M32
    h ^= h >> np.uint64(16)
    return h


def _attn_mix(h):
    """tile_common.h attn_mix: xorshift, 24 x 24-bit multiply-add of the high byte
    (v_mad_u32_u24), xorshift."""
    h = np.asarray(h, dtype=np.uint64) & M32
    h ^= h >> np.uint64(16)
    h = ((h & np.uint64(0xFFFFFF)) * np.uint64(0x9E3779) + (h >> np.uint64(24))) & M32
    h ^= h >> np.uint64(16)
    return h


def drop_key(seed: int, step: int, site: int) -> int:
    seed &= (1 << 64) - 1
    step &= (1 << 64) - 1
    k = _fmix32(np.uint64((seed & 0xFFFFFFFF) ^ 0x243F6A88))
    k = _fmix32(k ^ np.uint64(seed >> 32) ^ np.uint64((site * 0x9E3779B9) & 0xFFFFFFFF))
    k = _fmix32(k ^ (np.uint64(((step & 0xFFFFFFFF) * 0x85EBCA77) & 0xFFFFFFFF) ^ np.uint64(step >> 32)))
    return int(k)


def drop_threshold(p: float) -> int:
    if p <= 0:
        return 0
    if p >= 1:
        return 0xFFFFFFFF
    # the kernel computes (uint32)(double(float(p)) * 2^32)
    return int(float(np.float32(p)) * 4294967296.0)


def keep_mask(seed: int, step: int, site: int, p: float, idx) -> np.ndarray:
    """Boolean keep mask for flat element indices `idx` (int64 array)."""
    key = np.uint64(drop_key(seed, step, site))
    idx = np.asarray(idx, dtype=np.uint64)
    lo = idx & M32
    hi = idx >> np.uint64(32)
    mixed = ((lo * np.uint64(0x9E3779B1)) + (hi * np.uint64(0x7FEB352D))) & M32
    h = _fmix32(key ^ mixed)
    return h >= np.uint64(drop_threshold(p))


def attention_keep_mask(seed: int, step: int, site: int, p: float, B: int, H: int, S: int) -> np.ndarray:
    """Keep mask [B, H, S(query), S(key)] of the attention-probability dropout (mirror of
    tile_common.h attn_pair_hash / attn_keep_half: keys k and k + 16 of an aligned 32-key block
    share one hash, pair ((k >> 5) << 4) | (k & 15), 16-bit half (k >> 4) & 1)."""
    key = np.uint64(drop_key(seed, step, site))
    thr = 0 if p <= 0 else (0x10000 if p >= 1 else int(float(np.float32(p)) * 65536.0))
    rowid = np.arange(B * H * S, dtype=np.uint64).reshape(B * H, S, 1)
    k = np.arange(S, dtype=np.uint64).reshape(1, 1, S)
    pair = ((k >> np.uint64(5)) << np.uint64(4)) | (k & np.uint64(15))
    mixed = ((rowid * np.uint64(0x9E3779B1)) + (pair * np.uint64(0x7FEB352D))) & M32
    h = _attn_mix(key ^ mixed)
    half = np.where(((k >> np.uint64(4)) & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    return (half >= np.uint64(thr)).reshape(B, H, S, S)


def attention_drop_scale(p: float) -> float:
    """The kernels' 1/keep-probability for the realised 16-bit threshold."""
    if p <= 0:
        return 1.0
    thr = int(float(np.float32(p)) * 65536.0)
    return 65536.0 / (65536.0 - thr)
