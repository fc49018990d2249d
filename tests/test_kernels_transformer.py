"""Transformer kernels (attention.hip, transformer.hip, GEMM GELU/tanh epilogues) vs plain
PyTorch fp32 references of the same ops; dropout masks checked against the CPU mirror of
the kernels' counter hash."""
import math

import numpy as np
import pytest
import torch

from tensorflow_train_distributed_amd.ops import transformer as T

gpu = pytest.mark.gpu


def test_dropout_hash_mirror_statistics():
    idx = np.arange(200000, dtype=np.int64)
    keep = T.keep_mask(1234, 7, 3, 0.1, idx)
    assert abs(keep.mean() - 0.9) < 0.005
    keep2 = T.keep_mask(1234, 8, 3, 0.1, idx)  # a new step draws a different mask
    assert (keep != keep2).mean() > 0.1
    assert T.drop_threshold(0.0) == 0 and T.drop_threshold(1.0) == 0xFFFFFFFF


def _attn_ref(q, k, v, B, H, S, seqlen=None, keep=None, p=0.0):
    # q/k/v: [B*S, H*64] fp32
    def heads(t):
        return t.view(B, S, H, 64).transpose(1, 2)
    qh, kh, vh = heads(q), heads(k), heads(v)
    sc = qh @ kh.transpose(-1, -2) / 8.0
    if seqlen is not None:
        ar = torch.arange(S, device=q.device)
        m = ar[None, :] < seqlen[:, None].long()
        sc = sc.masked_fill(~m[:, None, None, :], float("-inf"))
    pr = sc.softmax(-1)
    if keep is not None:
        pr = pr * keep * T.attention_drop_scale(p)
    return (pr @ vh).transpose(1, 2).reshape(B * S, H * 64)


def _keep_tensor(rng_state, site, p, B, H, S, device):
    seed, step = rng_state
    return torch.from_numpy(T.attention_keep_mask(seed, step, site, p, B, H, S)).float().to(device)


def test_attention_dropout_pair_hash_statistics():
    keep = T.attention_keep_mask(1234, 7, 3, 0.1, 2, 4, 256)
    assert abs(keep.mean() - 0.9) < 0.005
    # the two keys of a pair (k and k + 16 of an aligned 32-key block) use different halves of
    # one hash: not correlated; nor are adjacent keys (different hashes)
    kk = keep.reshape(*keep.shape[:-1], -1, 2, 16)
    for a, b in ((kk[..., 0, :], kk[..., 1, :]), (keep[..., 0::2], keep[..., 1::2])):
        a, b = a.ravel(), b.ravel()
        assert abs(np.mean(a & b) - np.mean(a) * np.mean(b)) < 0.01
    # neighbouring pairs of a row, the same key in neighbouring rows, and the same (query, key)
    # of neighbouring heads are independent too (one multiply-xorshift round per pair hash)
    for u, v in ((keep[..., 0:-2:2], keep[..., 2::2]), (keep[..., :-1, :], keep[..., 1:, :]),
                 (keep[:, :-1], keep[:, 1:])):
        u, v = u.ravel(), v.ravel()
        assert abs(np.mean(u & v) - np.mean(u) * np.mean(v)) < 0.005
    # other sites / steps give different masks with the same rate
    keep2 = T.attention_keep_mask(1234, 8, 3, 0.1, 2, 4, 256)
    assert abs(keep2.mean() - 0.9) < 0.005 and np.mean(keep == keep2) < 0.85
    assert abs(T.attention_drop_scale(0.1) - 1 / 0.9) < 1e-4


def test_attention_pair_hash_has_full_32_bit_range():
    """Every input bit reaches the pair hash (a bare 24 x 24-bit multiply had at most
    2^24 outputs, x and x ^ 0x01000100 collided and each keep pattern repeated ~16 times per
    BERT-Large layer). Exact collisions over 2^21 consecutive (row, pair) inputs stay at the
    birthday rate of a 32-bit hash (n^2 / 2^33 = 512 expected; a 24-bit range gives ~131k)."""
    rng = np.random.default_rng(0)
    x = rng.integers(0, 1 << 32, size=1 << 16, dtype=np.uint64)
    assert np.all(T._attn_mix(x) != T._attn_mix(x ^ np.uint64(0x01000100)))
    key = np.uint64(T.drop_key(1234, 7, 3))
    rowid = np.arange(1 << 13, dtype=np.uint64).reshape(-1, 1)
    pair = np.arange(256, dtype=np.uint64).reshape(1, -1)
    mixed = ((rowid * np.uint64(0x9E3779B1)) + (pair * np.uint64(0x7FEB352D))) & np.uint64(0xFFFFFFFF)
    h = T._attn_mix(key ^ mixed).ravel()
    dup = h.size - np.unique(h).size
    assert dup < 2000, dup


@gpu
@pytest.mark.parametrize("S,masked,p,fused", [(256, False, 0.0, True), (256, True, 0.0, True), (256, False, 0.1, True),
                                             (512, True, 0.1, True), (128, False, 0.1, True), (512, False, 0.0, True),
                                             (256, True, 0.1, False), (512, False, 0.1, False)])
def test_attention_fwd_bwd_matches_reference(S, masked, p, fused):
    """fp32 autograd oracle; the backward on the single-kernel path (fused, S in {128, 256, 512})
    and on the split dQ / dK-dV kernels."""
    torch.manual_seed(0)
    B, H = 2, 3
    D = H * 64
    dev = "cuda"
    qkv = (torch.randn(B * S, 3 * D, device=dev) * 1.5).bfloat16()
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    seqlen = torch.tensor([S, S // 2 + 22], dtype=torch.int32, device=dev) if masked else None
    rng = T.RngState(99, dev) if p > 0 else None
    if rng is not None:
        rng.advance()
    o = torch.empty(B * S, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, S, dtype=torch.float32, device=dev)
    T.attention_fwd(q, k, v, o, lse, B, H, S, seqlen=seqlen, p_drop=p, rng=rng, site=5)
    keep = _keep_tensor(rng.host(), 5, p, B, H, S, dev) if p > 0 else None
    qf, kf, vf = [t.float().requires_grad_(True) for t in (q, k, v)]
    ref = _attn_ref(qf, kf, vf, B, H, S, seqlen, keep, p)
    torch.testing.assert_close(o.float(), ref, atol=3e-2, rtol=3e-2)
    # lse (log2 domain) vs reference logsumexp
    sc = (qf.view(B, S, H, 64).transpose(1, 2) @ kf.view(B, S, H, 64).transpose(1, 2).transpose(-1, -2)) / 8.0
    if masked:
        ar = torch.arange(S, device=dev)
        sc = sc.masked_fill(~(ar[None, :] < seqlen[:, None].long())[:, None, None, :], float("-inf"))
    lse_ref = torch.logsumexp(sc, -1).reshape(B * H, S) / math.log(2)
    torch.testing.assert_close(lse, lse_ref.detach(), atol=2e-2, rtol=1e-3)
    # backward
    do = torch.randn(B * S, D, device=dev).bfloat16()
    ref.backward(do.float())
    dqkv = torch.empty_like(qkv)
    T.set_fused_attention_bwd(fused)
    try:
        T.attention_bwd(q, k, v, o, do, lse, dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:], B, H, S, seqlen=seqlen,
                        p_drop=p, rng=rng, site=5)
    finally:
        T.set_fused_attention_bwd(False)
    for name, got, want in (("dq", dqkv[:, :D], qf.grad), ("dk", dqkv[:, D:2 * D], kf.grad),
                            ("dv", dqkv[:, 2 * D:], vf.grad)):
        rel = float((got.float() - want).norm() / want.norm())
        assert rel < 2e-2, (name, rel)


@gpu
@pytest.mark.parametrize("H,rows", [(512, 300), (1024, 300), (1024, 5003), (512, 4099), (1536, 300), (2048, 77),
                                    (4096, 300)])
def test_layernorm_residual_dropout_fwd_bwd(H, rows):
    # rows >= 4096 take the many-rows-per-block backward path (odd tails: a wave's second row
    # missing, a short last block); each H has its own (waves, rows-in-flight) variant
    torch.manual_seed(1)
    dev = "cuda"
    x = torch.randn(rows, H, device=dev).bfloat16()
    res = torch.randn(rows, H, device=dev).bfloat16()
    gamma = torch.randn(H, device=dev) * 0.5 + 1
    beta = torch.randn(H, device=dev) * 0.1
    p_in, p_out = 0.1, 0.2
    rng = T.RngState(7, dev)
    y, s, mean, rstd = T.layernorm_fwd(x, gamma, beta, res=res, eps=1e-12, p_in=p_in, site_in=11, p_out=p_out,
                                       site_out=12, rng=rng)
    seed, step = rng.host()
    idx = np.arange(rows * H, dtype=np.int64)
    kin = torch.from_numpy(T.keep_mask(seed, step, 11, p_in, idx).reshape(rows, H)).float().to(dev)
    kout = torch.from_numpy(T.keep_mask(seed, step, 12, p_out, idx).reshape(rows, H)).float().to(dev)
    xf = x.float().requires_grad_(True)
    rf = res.float().requires_grad_(True)
    gf = gamma.clone().requires_grad_(True)
    bf = beta.clone().requires_grad_(True)
    sref = rf + xf * kin / (1 - p_in)
    yref = torch.nn.functional.layer_norm(sref, (H,), gf, bf, 1e-12) * kout / (1 - p_out)
    torch.testing.assert_close(s.float(), sref.detach(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(y.float(), yref.detach(), atol=5e-2, rtol=2e-2)
    dy = torch.randn(rows, H, device=dev).bfloat16()
    yref.backward(dy.float())
    dg = torch.empty(H, device=dev)
    db = torch.empty(H, device=dev)
    ds, dx = T.layernorm_bwd(dy, s, mean, rstd, gamma, dg, db, want_dx=True, p_in=p_in, site_in=11, p_out=p_out,
                             site_out=12, rng=rng)
    for name, got, want in (("dres", ds, rf.grad), ("dx", dx, xf.grad), ("dgamma", dg, gf.grad),
                            ("dbeta", db, bf.grad)):
        rel = float((got.float() - want).norm() / want.norm())
        assert rel < 2e-2, (name, rel)


@gpu
def test_embedding_fwd_bwd():
    torch.manual_seed(2)
    dev = "cuda"
    B, S, H, V = 3, 128, 512, 1000
    word = torch.randn(V, H, device=dev).bfloat16()
    pos = torch.randn(512, H, device=dev).bfloat16()
    typ = torch.randn(2, H, device=dev).bfloat16()
    ids = torch.randint(0, V, (B * S,), device=dev, dtype=torch.int32)
    tt = torch.randint(0, 2, (B * S,), device=dev, dtype=torch.int32)
    s = T.embed_fwd(ids, tt, word, pos, typ, S)
    ref = word.float()[ids.long()] + pos.float()[torch.arange(B * S, device=dev) % S] + typ.float()[tt.long()]
    torch.testing.assert_close(s.float(), ref, atol=3e-2, rtol=1e-2)
    ds = torch.randn(B * S, H, device=dev).bfloat16()
    dword = torch.zeros(V, H, device=dev)
    dpos = torch.empty(512, H, device=dev)
    dtyp = torch.empty(2, H, device=dev)
    T.embed_bwd(ds, ids, tt, dword, dpos[:S], dtyp, B, S)
    rw = torch.zeros(V, H, device=dev).index_add_(0, ids.long(), ds.float())
    rp = ds.float().view(B, S, H).sum(0)
    rt = torch.zeros(2, H, device=dev).index_add_(0, tt.long(), ds.float())
    torch.testing.assert_close(dword, rw, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(dpos[:S], rp, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(dtyp, rt, atol=1e-2, rtol=1e-4)


@gpu
def test_xent_vocab_padded_ignore_index():
    torch.manual_seed(3)
    dev = "cuda"
    rows, V, Vp = 40, 1000, 1024
    logits = (torch.randn(rows, Vp, device=dev) * 3).bfloat16()
    labels = torch.randint(0, V, (rows,), device=dev, dtype=torch.int32)
    labels[::7] = -1
    inv = torch.empty(1, device=dev)
    T.count_valid(labels, 1.0, inv)
    nvalid = int((labels >= 0).sum())
    assert abs(float(inv) - 1.0 / nvalid) < 1e-7
    sums = torch.zeros(2, device=dev)
    lf = logits.float()[:, :V].clone()
    dl = logits.clone()
    T.xent_vocab(dl, V, labels, inv, dlogits=dl, sums=sums, mscale=inv)
    valid = labels >= 0
    ce = torch.nn.functional.cross_entropy(lf[valid], labels[valid].long())
    assert abs(float(sums[0]) - float(ce)) < 1e-3 * float(ce)
    acc = float((lf[valid].argmax(1) == labels[valid].long()).float().mean())
    assert abs(float(sums[1]) - acc) < 1e-5
    lf.requires_grad_(True)
    torch.nn.functional.cross_entropy(lf[valid], labels[valid].long()).backward()
    torch.testing.assert_close(dl[:, :V].float(), lf.grad, atol=2e-4, rtol=2e-2)
    assert float(dl[:, V:].float().abs().sum()) == 0.0
    assert float(dl[~valid].float().abs().sum()) == 0.0


@gpu
def test_gemm_gelu_aux_and_dgelu_tanh_epilogues():
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(4)
    dev = "cuda"
    M, N, K = 300, 256, 192
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
    bias = torch.randn(N, device=dev) * 0.1
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    y = G.gemm(a, w, trans_b=True, bias=bias, act=G.ACT_GELU, aux=pre)
    z = a.float() @ w.float().t() + bias
    gelu = 0.5 * z * (1 + torch.tanh(0.7978845608028654 * (z + 0.044715 * z ** 3)))
    torch.testing.assert_close(pre.float(), z, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(y.float(), gelu, atol=3e-2, rtol=2e-2)
    # dgelu: d_pre = (dy @ w2) * gelu'(pre)
    w2 = (torch.randn(64, N, device=dev) * 0.1).bfloat16()
    dy = torch.randn(M, 64, device=dev).bfloat16()
    dpre = G.gemm(dy, w2, act=G.ACT_DGELU, residual=pre)
    zf = pre.float().requires_grad_(True)
    g = 0.5 * zf * (1 + torch.tanh(0.7978845608028654 * (zf + 0.044715 * zf ** 3)))
    g.backward(dy.float() @ w2.float())
    torch.testing.assert_close(dpre.float(), zf.grad, atol=3e-2, rtol=3e-2)
    t = G.gemm(a, w, trans_b=True, bias=bias, act=G.ACT_TANH)
    torch.testing.assert_close(t.float(), torch.tanh(z), atol=2e-2, rtol=2e-2)
    dt = T.dact(dy[:, :64].contiguous(), t[:, :64].contiguous(), 1)
    torch.testing.assert_close(dt.float(), dy[:, :64].float() * (1 - t[:, :64].float() ** 2), atol=2e-2, rtol=2e-2)


@gpu
def test_gather_scatter_rows():
    dev = "cuda"
    src = torch.randn(50, 512, device=dev).bfloat16()
    idx = torch.tensor([3, 7, 0, 49], dtype=torch.int32, device=dev)
    g = T.gather_rows(src, idx)
    assert torch.equal(g, src[idx.long()])
    dst = torch.zeros(50, 512, dtype=torch.bfloat16, device=dev)
    T.scatter_rows(g, idx, dst)
    assert torch.equal(dst[idx.long()], g)
    T.scatter_rows(g[:1], idx[:1], dst, accumulate=True)
    torch.testing.assert_close(dst[3].float(), 2 * src[3].float(), atol=1e-2, rtol=1e-2)


@gpu
def test_gather_scatter_rows_grouped_and_rng_advance():
    """Per-sequence positions [B, P] against a [B*S, H] activation (row b*S + pos) and the CLS
    rows (b*S, no index tensor), both directions; the dropout RNG step advanced on the stream."""
    dev = "cuda"
    B, S, P, H = 3, 16, 5, 256
    src = torch.randn(B * S, H, device=dev).bfloat16()
    pos = torch.randint(0, S, (B, P), dtype=torch.int32, device=dev)
    rows = (pos.long() + torch.arange(B, device=dev)[:, None] * S).reshape(-1)
    g = T.gather_rows(src, pos.reshape(-1), group=(P, S))
    assert torch.equal(g, src[rows])
    c = T.gather_rows(src, None, group=(1, S), n=B)
    assert torch.equal(c, src[::S])
    dst = torch.zeros(B * S, H, dtype=torch.bfloat16, device=dev)
    T.scatter_rows(c, None, dst, group=(1, S))
    assert torch.equal(dst[::S], c)
    T.scatter_rows(c, None, dst, accumulate=True, group=(1, S))
    torch.testing.assert_close(dst[::S].float(), 2 * c.float(), atol=1e-2, rtol=1e-2)
    dst.zero_()
    uniq = torch.arange(P, dtype=torch.int32, device=dev).repeat(B, 1)  # no duplicate rows
    T.scatter_rows(g, uniq.reshape(-1), dst, group=(P, S))
    r2 = (uniq.long() + torch.arange(B, device=dev)[:, None] * S).reshape(-1)
    assert torch.equal(dst[r2], g)
    rng = T.RngState(7, dev)
    for _ in range(3):
        rng.advance()
    assert rng.host() == (7, 3)
