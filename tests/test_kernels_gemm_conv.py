"""Numerics of the MFMA GEMM / implicit-GEMM conv kernels vs a PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1000, 200, 784), (128, 1000, 2048), (4096, 64, 64),
                                   (72, 136, 520), (128, 100, 200), (128, 25, 50), (77, 10, 25), (3, 5, 7)])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_layouts(M, N, K, ta, tb):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    ref = a.float() @ b.float()
    A = a.t().contiguous() if ta else a
    B = b.t().contiguous() if tb else b
    out = G.gemm(A, B, trans_a=ta, trans_b=tb)
    assert _rel(out, ref) < 1e-2
    out32 = G.gemm(A, B, trans_a=ta, trans_b=tb, out_dtype=torch.float32)
    assert _rel(out32, ref) < 1e-3
    out_split = G.gemm(A, B, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splits=3)
    assert _rel(out_split, ref) < 1e-3


def test_gemm_epilogue_bias_act_residual():
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(1)
    a = torch.randn(300, 128, device="cuda").bfloat16()
    b = torch.randn(128, 96, device="cuda").bfloat16()
    bias = torch.randn(96, device="cuda")
    res = torch.randn(300, 96, device="cuda").bfloat16()
    out = G.gemm(a, b, bias=bias, residual=res, act=G.ACT_RELU)
    ref = torch.relu(a.float() @ b.float() + bias + res.float())
    assert _rel(out, ref) < 1e-2
    out = G.gemm(a, b, bias=bias, act=G.ACT_GELU)
    ref = F.gelu(a.float() @ b.float() + bias, approximate="tanh")
    assert _rel(out, ref) < 1e-2


CONVS = [
    # N, H, W, C, K, R, stride, pad
    (2, 16, 16, 64, 64, 3, 1, 1),
    (2, 15, 15, 32, 128, 3, 2, 1),
    (2, 14, 14, 64, 256, 1, 1, 0),
    (2, 14, 14, 64, 128, 1, 2, 0),
    (2, 32, 32, 8, 64, 7, 2, 3),
    (3, 7, 7, 512, 512, 3, 1, 1),
    # 256-row LDS-DMA paths (fwd BN=128 gather; fwd/dgrad/wgrad BN=256 gathers; strided gathers)
    (8, 32, 32, 64, 128, 3, 1, 1),
    (16, 16, 16, 256, 256, 3, 1, 1),
    (16, 32, 32, 128, 256, 3, 2, 1),
    (16, 32, 32, 256, 512, 1, 2, 0),
    (16, 16, 16, 128, 256, 1, 1, 0),
]


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd_dgrad_wgrad(cfg):
    from tensorflow_train_distributed_amd.ops import gemm as G
    N, H, W, C, K, R, s, p = cfg
    torch.manual_seed(2)
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
    xr = _nchw(x.float()).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    y = G.conv_fwd(x, w, (s, s), (p, p))
    assert y.shape == (N, yr.shape[2], yr.shape[3], K)
    assert _rel(y, _nhwc(yr)) < 1e-2
    dy = torch.randn_like(y)
    yr.backward(_nchw(dy.float()))
    wt = w.permute(3, 1, 2, 0).contiguous()  # [C,R,S,K]
    dx = G.conv_dgrad(dy, wt, x.shape, (s, s), (p, p))
    assert _rel(dx, _nhwc(xr.grad)) < 1e-2
    dw = G.conv_wgrad(x, dy, w.shape, (s, s), (p, p))
    assert _rel(dw, wr.grad.permute(0, 2, 3, 1)) < 1e-2
    dw1 = G.conv_wgrad(x, dy, w.shape, (s, s), (p, p), splits=1)
    assert _rel(dw1, wr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("cfg", [
    # N, H, W, C, K, R, stride, pad — odd extents (unequal phases), stride 3, 5x5, big-tile phases
    (2, 15, 13, 32, 64, 3, 2, 1),
    (2, 12, 12, 16, 64, 3, 3, 1),
    (2, 9, 9, 16, 64, 5, 2, 2),
    (8, 56, 56, 128, 128, 3, 2, 1),
])
def test_conv_dgrad_subpixel_phases(cfg):
    """Strided dgrad as s*s unit-stride phase GEMMs vs the fp32 reference, vs the direct
    strided gather, and with beta accumulation into an existing gradient."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    N, H, W, C, K, R, s, p = cfg
    torch.manual_seed(7)
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
    xr = _nchw(x.float()).requires_grad_(True)
    yr = F.conv2d(xr, w.float().permute(0, 3, 1, 2), stride=s, padding=p)
    dy = torch.randn(N, yr.shape[2], yr.shape[3], K, device="cuda").bfloat16()
    yr.backward(_nchw(dy.float()))
    ref = _nhwc(xr.grad)
    wt = w.permute(3, 1, 2, 0).contiguous()
    assert G._SUBPIXEL
    dx = G.conv_dgrad(dy, wt, x.shape, (s, s), (p, p))
    assert _rel(dx, ref) < 1e-2
    G._SUBPIXEL = False
    try:
        dx_direct = G.conv_dgrad(dy, wt, x.shape, (s, s), (p, p))
    finally:
        G._SUBPIXEL = True
    assert _rel(dx, dx_direct.float()) < 1e-2
    prev = torch.randn_like(dx)
    acc = prev.clone()
    G.conv_dgrad(dy, wt, x.shape, (s, s), (p, p), out=acc, beta=1)
    assert _rel(acc, ref + prev.float()) < 1e-2


def test_conv_bn_stat_epilogue_big_tile():
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(4)
    x = torch.randn(16, 16, 16, 128, device="cuda").bfloat16()
    w = (torch.randn(256, 3, 3, 128, device="cuda") / 34).bfloat16()
    M = 16 * 16 * 16
    assert G.big_bn(M, 256, 9 * 128) == 256
    stat = torch.zeros((M + 255) // 256, 2, 256, device="cuda")
    y = G.conv_fwd(x, w, (1, 1), (1, 1), stat=stat, tile=(256, 256))
    ref = F.conv2d(_nchw(x.float()), w.float().permute(0, 3, 1, 2), padding=1)
    assert _rel(y, _nhwc(ref)) < 1e-2
    s = stat.sum(0)
    yf = y.float().reshape(-1, 256)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-3, atol=2e-2)


def _q8(t, e5m2=False):
    """Per-tensor scaled fp8 quantisation; returns (uint8 codes, dequantised fp32, inv scale)."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    fmax = 57344.0 if e5m2 else 448.0
    amax = float(t.float().abs().max())
    scale = torch.tensor([fmax / amax], device="cuda")
    q = K.quant_fp8(t.bfloat16().contiguous(), scale, e5m2=e5m2)
    deq = K.dequant_fp8(q, scale, e5m2=e5m2).float()  # dequant divides by the quant scale
    return q, deq, 1.0 / float(scale)


@pytest.mark.parametrize("M,N,K,e5m2", [(512, 768, 512, False), (1024, 128, 256, False), (300, 520, 384, True)])
def test_gemm_fp8_block_scaled_mfma(M, N, K, e5m2):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(M + N)
    a, b = torch.randn(M, K, device="cuda"), torch.randn(N, K, device="cuda")
    a8, ad, sa = _q8(a, e5m2)
    b8, bd, sb = _q8(b)
    ref = ad @ bd.t()
    y = G.gemm_fp8(a8, b8, alpha=sa * sb, a_e5m2=e5m2)
    assert _rel(y, ref) < 1e-2
    y32 = G.gemm_fp8(a8, b8, alpha=sa * sb, a_e5m2=e5m2, out_dtype=torch.float32, splits=2)
    assert _rel(y32, ref) < 5e-3  # reference operands are bf16-rounded dequantisations


@pytest.mark.parametrize("cfg", [(16, 16, 16, 128, 256, 3, 1, 1), (16, 32, 32, 256, 128, 1, 1, 0)])
def test_conv_fwd_fp8(cfg):
    from tensorflow_train_distributed_amd.ops import gemm as G
    N, H, W, C, K, R, s, p = cfg
    torch.manual_seed(5)
    x = torch.randn(N, H, W, C, device="cuda")
    w = torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5
    x8, xd, sx = _q8(x)
    w8, wd, sw = _q8(w)
    ref = F.conv2d(_nchw(xd), wd.permute(0, 3, 1, 2), stride=s, padding=p)
    y = G.conv_fwd_fp8(x8, w8, (s, s), (p, p), alpha=sx * sw)
    assert _rel(y, _nhwc(ref)) < 1e-2


def test_conv_bn_stat_epilogue():
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(3)
    x = torch.randn(2, 20, 20, 64, device="cuda").bfloat16()
    w = (torch.randn(128, 3, 3, 64, device="cuda") / 24).bfloat16()
    M = 2 * 20 * 20
    stat = torch.zeros((M + 127) // 128, 2, 128, device="cuda")
    y = G.conv_fwd(x, w, (1, 1), (1, 1), stat=stat, tile=(128, 128))
    s = stat.sum(0)
    yf = y.float().reshape(-1, 128)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (300, 520, 192)])
def test_gemm256_lds_dma_path_all_layouts(ta, tb, M, N, K):
    """The 256x256 global_load_lds kernel (forced with tile=(256, 256)) vs fp32 matmul, bf16
    and split-K fp32 outputs, edge tiles included."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 2 * ta + tb)
    a = torch.randn((K, M) if ta else (M, K), device="cuda").bfloat16()
    b = torch.randn((N, K) if tb else (K, N), device="cuda").bfloat16()
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda").bfloat16()
    aux = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    y = G.gemm(a, b, trans_a=ta, trans_b=tb, bias=bias, residual=res, act=G.ACT_GELU, aux=aux, tile=(256, 256))
    pre = ref + bias + res.float()
    torch.testing.assert_close(aux.float(), pre, atol=0.15, rtol=2e-2)
    gel = 0.5 * pre * (1 + torch.tanh(0.7978845608028654 * (pre + 0.044715 * pre ** 3)))
    torch.testing.assert_close(y.float(), gel, atol=0.15, rtol=2e-2)
    for splits in (1, 3):
        out = torch.full((M, N), 1.0, device="cuda")
        G.gemm(a, b, trans_a=ta, trans_b=tb, out=out, splits=splits, beta=1, tile=(256, 256))
        torch.testing.assert_close(out, ref + 1.0, atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("cfg", [
    # N, H, W, C, K, R, stride, pad — 4-wave tiles, 256-row tiles (1x1 dense + 3x3 gather),
    # strided 3x3 as sub-pixel phases (4-wave and 256-row phase GEMMs); dx is [N, H, W, C]
    (2, 14, 14, 64, 64, 3, 1, 1),
    (16, 16, 16, 128, 256, 1, 1, 0),
    (8, 32, 32, 128, 128, 3, 1, 1),
    (16, 32, 32, 256, 64, 1, 1, 0),
    (2, 16, 16, 64, 128, 3, 2, 1),
    (8, 56, 56, 128, 128, 3, 2, 1),
])
@pytest.mark.parametrize("beta", [0, 1])
def test_conv_dgrad_bn_backward_stat_epilogue(cfg, beta):
    """dgrad whose epilogue stores g = dx * relu_mask and per-tile (sum g, sum g*y) of the
    consuming BN (the fused BN-backward statistics), plus (sum g, sum g*y2) of a second BN fed
    by the same gradient (projection shortcut), vs an fp32 reference."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    N, H, W, C, K, R, s, p = cfg
    torch.manual_seed(11)
    P = (H + 2 * p - R) // s + 1
    dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()
    y = torch.randn(N, H, W, C, device="cuda").bfloat16()
    y2 = torch.randn(N, H, W, C, device="cuda").bfloat16()
    keep = torch.rand(N * H * W * C, device="cuda") > 0.3
    bits = keep.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)
    mask = bits.sum(1).to(torch.uint8)
    old = torch.randn(N, H, W, C, device="cuda").bfloat16()
    ref = G.conv_dgrad(dy, wt, (N, H, W, C), (s, s), (p, p)).float()
    if beta:
        ref = ref + old.float()
    ref_g = ref * keep.view(N, H, W, C)
    out = old.clone() if beta else None
    second = s == 1
    res = G.conv_dgrad(dy, wt, (N, H, W, C), (s, s), (p, p), out=out, beta=beta, bn_stat=(y, mask),
                       bn_stat2=y2 if second else None)
    got, partial, T = res[:3]
    assert _rel(got, ref_g) < 1e-2
    assert bool(((got.float() != 0) <= keep.view(N, H, W, C)).all())  # masked elements are exact zeros
    gs = got.float().view(-1, C)
    sums = partial.sum(0)
    torch.testing.assert_close(sums[0], gs.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(sums[1], (gs * y.float().view(-1, C)).sum(0), rtol=1e-3, atol=1e-2)
    if second:
        sums2 = res[3].sum(0)
        torch.testing.assert_close(sums2[0], gs.sum(0), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(sums2[1], (gs * y2.float().view(-1, C)).sum(0), rtol=1e-3, atol=1e-2)
    assert T == G.dgrad_stat_rows((N, H, W, C), tuple(wt.shape), (s, s), (p, p))
    # strided 1x1 convs compute only the sampled pixels: no fused statistics
    assert G.dgrad_stat_rows((N, 2 * H, 2 * W, C), (C, 1, 1, K), (2, 2), (0, 0)) is None


@pytest.mark.parametrize("splits", [2, 7, 64, 300])
def test_splitk_reduce_many_slabs_with_accumulate(splits):
    """Split-K fp32 output over many slabs (single-pass and two-pass fold) with beta
    accumulation into an existing gradient, vs fp32 reference."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(3)
    M, N, K = 130, 70, 64 * 320
    a = torch.randn(K, M, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    ref = a.float().t() @ b.float()
    base = torch.randn(M, N, device="cuda")
    out = base.clone()
    G.gemm(a, b, trans_a=True, out=out, splits=splits, beta=1)
    assert _rel(out, ref + base) < 1e-4
    out2 = G.gemm(a, b, trans_a=True, out_dtype=torch.float32, splits=splits)
    assert _rel(out2, ref) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [((2, 32, 32, 8), (64, 7, 7, 8), 2, 3), ((4, 16, 16, 64), (64, 3, 3, 64), 1, 1)])
def test_conv_wgrad_with_fused_bn_backward_operand(shape):
    """conv_wgrad_bn (BN backward applied in the dy operand load) matches bn_backward_from_partial
    followed by conv_wgrad (same bf16 rounding of dy, same split-K partition)."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    xs, ws, st, pd = shape
    torch.manual_seed(11)
    x = torch.randn(xs, device="cuda").bfloat16()
    y = G.conv_fwd(x, (torch.randn(ws, device="cuda") * 0.1).bfloat16(), (st, st), (pd, pd))
    N, P, Q, C = y.shape
    M = N * P * Q
    g = torch.randn_like(y)
    partial, T = K.bn_stats_partial(y.view(M, C))  # any per-tile partial sums will do for the plumbing
    gamma = torch.rand(C, device="cuda") + 0.5
    state = K.BNState(C, "cuda")
    K.bn_fwd_finalize(K.bn_reduce_partials(partial, T, C), M, gamma, torch.zeros(C, device="cuda"), 1e-5, 0.9,
                      torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"), state)
    dg1, db1, dg2, db2 = (torch.empty(C, device="cuda") for _ in range(4))
    dz = K.bn_backward_from_partial(g.view(M, C), y.view(M, C), gamma, state, dg1, db1, partial, T).view(y.shape)
    ref = G.conv_wgrad(x, dz, ws, (st, st), (pd, pd))
    assert G.conv_wgrad_bn_fusable(x.shape, ws, (st, st), (pd, pd))
    coef = K.bn_backward_coef(M, C, gamma, state, dg2, db2, partial, T)
    got = G.conv_wgrad_bn(x, g, y, coef, ws, (st, st), (pd, pd))
    # the two kernels may contract a*g + b*y + c into FMAs differently: dy can differ by one
    # bf16 ulp in a few elements
    assert float((got - ref).norm() / ref.norm()) < 2e-3
    assert torch.equal(dg1, dg2) and torch.equal(db1, db2)


def test_stem_weight_gradient_kernel_matches_oracle():
    """stem_wgrad.hip: 7x7/s2/p3 weight gradient over the 3 real channels of an 8-channel
    image with dz = coef0*g + coef1*y + coef2 formed on the fly, vs fp32 torch."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(9)
    N, H = 3, 224
    x = torch.zeros(N, H, H, 8, device="cuda")
    x[..., :3] = torch.randn(N, H, H, 3, device="cuda")
    x = x.bfloat16()
    P = 112
    g = torch.randn(N, P, P, 64, device="cuda").bfloat16()
    y = torch.randn(N, P, P, 64, device="cuda").bfloat16()
    coef = torch.randn(3, 64, device="cuda") * torch.tensor([[1.0], [0.1], [0.05]], device="cuda")
    out = G.stem_wgrad(x, g, y, coef)
    dz = (coef[0] * g.float() + coef[1] * y.float() + coef[2]).bfloat16().float()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 8, 7, 7), dz.permute(0, 3, 1, 2),
                                      stride=2, padding=3).permute(0, 2, 3, 1)
    assert _rel(out, ref) < 1e-2
    assert bool((out[..., 3:] == 0).all())
    old = torch.randn_like(out)
    out2 = G.stem_wgrad(x, g, y, coef, out=old.clone(), beta=1)
    assert _rel(out2, ref + old) < 1e-2
    # packed [N, H, W, 3] input: same sums (same LDS contents, same order)
    out3 = G.stem_wgrad(x[..., :3].contiguous(), g, y, coef)
    assert torch.equal(out3, out)


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("epi", ["bias_gelu_aux", "dgelu", "bias_residual", "beta"])
def test_persistent_register_epilogue_gemm_matches_one_tile_kernel(ta, tb, epi):
    """More than one round of 256 x 256 tiles with K >= 1024 and an elementwise epilogue runs on
    the persistent kernel (gemm256p_kernel: next tile's operand DMA under this tile's register
    epilogue). Compared with the one-tile-per-workgroup kernel (switched off at run time) and an
    fp32 oracle; ragged M exercises the row guard."""
    from tensorflow_train_distributed_amd.ops import _lib
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(3)
    M, N, K = 8192 + 72, 2048, 1024  # 33 x 8 = 264 tiles > 256 CUs
    a = (torch.randn((K, M) if ta else (M, K), device="cuda") / K ** 0.25).bfloat16()
    b = (torch.randn((N, K) if tb else (K, N), device="cuda") / K ** 0.25).bfloat16()
    af = a.float().t() if ta else a.float()
    bf = b.float().t() if tb else b.float()
    ref = af @ bf
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda").bfloat16()
    old = torch.randn(M, N, device="cuda").bfloat16()

    def run():
        kw = dict(trans_a=ta, trans_b=tb)
        if epi == "bias_gelu_aux":
            aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            y = G.gemm(a, b, bias=bias, act=G.ACT_GELU, aux=aux, **kw)
            return y, aux
        if epi == "dgelu":
            return G.gemm(a, b, act=G.ACT_DGELU, residual=res, **kw), None
        if epi == "bias_residual":
            return G.gemm(a, b, bias=bias, residual=res, **kw), None
        out = old.clone()
        return G.gemm(a, b, out=out, beta=1, **kw), None

    prev = _lib.query("ttdk_set_big_pers", 1)
    try:
        y1, x1 = run()
        _lib.query("ttdk_set_big_pers", 0)
        y0, x0 = run()
    finally:
        _lib.query("ttdk_set_big_pers", prev)
    torch.cuda.synchronize()
    if epi == "bias_gelu_aux":
        pre = ref + bias
        want = F.gelu(pre, approximate="tanh")
        assert _rel(x1, pre) < 1e-2
        assert _rel(x1, x0) < 1e-2
    elif epi == "dgelu":
        xr = res.float()
        t = torch.tanh(0.7978845608028654 * (xr + 0.044715 * xr ** 3))
        gg = 0.5 * (1 + t) + 0.5 * xr * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * xr * xr)
        want = ref * gg
    elif epi == "bias_residual":
        want = ref + bias + res.float()
    else:
        want = ref + old.float()
    assert _rel(y1, want) < 1e-2
    # the one-tile kernel rounds the accumulator to bf16 before the epilogue: same result to
    # within bf16 rounding
    assert _rel(y1, y0) < 1e-2
    assert torch.isfinite(y1.float()).all()


@pytest.mark.parametrize("N,cin", [(3, 8), (257, 8), (3, 3)])
def test_stem_forward_kernel_matches_conv_oracle(N, cin):
    """Dedicated stem forward (stem_fwd.hip: K = 7 taps x (s, c4) over the 3 real channels, no
    im2col) vs the fp32 convolution, and its per-workgroup BN sums vs the stored output."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(21)
    x = torch.zeros(N, 224, 224, 8, device="cuda", dtype=torch.bfloat16)
    x[..., :3] = torch.randn(N, 224, 224, 3, device="cuda").bfloat16()
    w = (torch.randn(64, 7, 7, 8, device="cuda") * 0.1).bfloat16()
    w[..., 3:] = 0
    assert G.stem_fwd_ok(x.shape, w.shape, (2, 2), (3, 3), 3)
    y, part, T = G.stem_fwd(x if cin == 8 else x[..., :3].contiguous(), w)
    torch.cuda.synchronize()
    n_chk = min(N, 4)
    xs = torch.cat([x[:2], x[-2:]]) if N > 4 else x
    ys = torch.cat([y[:2], y[-2:]]) if N > 4 else y
    ref = F.conv2d(xs.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2, padding=3).permute(0, 2, 3, 1)
    assert ys.shape[0] == n_chk
    assert _rel(ys, ref) < 8e-3
    yf = y.float().view(-1, 64)
    torch.testing.assert_close(part[:T, 0].sum(0), yf.sum(0), rtol=1e-3, atol=1.0)
    torch.testing.assert_close(part[:T, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=1.0)
    # same values as the generic implicit-GEMM conv (both round the fp32 sum once)
    y2 = G.conv_fwd(xs, w, (2, 2), (3, 3))
    assert _rel(ys, y2) < 8e-3


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [
    # (N, H, C = dx channels, K = dz channels, R): ResNet-50 b1024 per-image stage shapes of the
    # c1 data gradients that accumulate into the shortcut gradient (stage 2, 3, 4) and a 3x3
    (48, 56, 256, 64, 1),
    (96, 28, 512, 128, 1),
    (192, 14, 1024, 256, 1),
    (64, 28, 128, 128, 3),
])
def test_pipelined_feeding_bn_epilogue_vs_fp32_conv(cfg):
    """The 256-row kernel's prefetched feeding-BN epilogue (dgrad + accumulate into the shortcut
    gradient + ReLU mask of the feeding unit + its BN-backward sums, gemm_conv.h feed_epilogue)
    against an fp32 torch convolution oracle (torch.nn.grad.conv2d_input), not the engine's own
    un-fused dgrad."""
    from torch.nn.grad import conv2d_input
    from tensorflow_train_distributed_amd.ops import gemm as G
    N, H, C, K, R = cfg
    p = R // 2
    torch.manual_seed(5)
    dz = torch.randn(N, H, H, K, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") / (R * R * K) ** 0.5).bfloat16()  # [K, R, S, C]
    wt = w.permute(3, 1, 2, 0).contiguous()  # the dgrad operand [C, R, S, K]
    y = torch.randn(N, H, H, C, device="cuda").bfloat16()
    keep = torch.rand(N * H * H * C, device="cuda") > 0.4
    bits = keep.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)
    mask = bits.sum(1).to(torch.uint8)
    old = torch.randn(N, H, H, C, device="cuda").bfloat16()
    dx = conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), dz.float().permute(0, 3, 1, 2),
                      padding=p).permute(0, 2, 3, 1)
    ref_g = (dx + old.float()) * keep.view(N, H, H, C)
    out = old.clone()
    got, partial, T = G.conv_dgrad(dz, wt, (N, H, H, C), (1, 1), (p, p), out=out, beta=1, bn_stat=(y, mask))[:3]
    assert _rel(got, ref_g) < 1e-2
    assert bool(((got.float() != 0) <= keep.view(N, H, H, C)).all())
    sums = partial.sum(0)
    gs, yf = ref_g.view(-1, C), y.float().view(-1, C)
    # statistics of the fused gradient vs the fp32 oracle's (bf16 storage of g: ~1e-3 relative)
    assert _rel(sums[0], gs.sum(0)) < 2e-2
    assert _rel(sums[1], (gs * yf).sum(0)) < 2e-2
    # ... and exactly consistent with the gradient it stored
    torch.testing.assert_close(sums[1], (got.float().view(-1, C) * yf).sum(0), rtol=2e-3, atol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [
    # (N, H, K = dz channels, C = dx channels, feed): ResNet-50 1x1 dgrads at per-image stage shapes —
    # c3 (4*mid -> mid, BN = 128 / 256 tiles) and c1 (mid -> 4*mid, accumulate + feeding-BN epilogue)
    (32, 28, 512, 128, False),
    (64, 14, 1024, 256, False),
    (16, 28, 128, 512, True),
    (48, 14, 256, 1024, True),
    (17, 17, 256, 256, True),  # ragged M (4913 rows): clamped operand rows, partial last tile
])
def test_dgrad_with_bn_backward_operand_prologue(cfg):
    """conv_dgrad(bn_pro=...): the 1x1 data gradient whose A operand is the BN backward of the
    unit's masked output gradient, formed in LDS (dz = a*g + b*y + c), stored once for the weight
    gradient — vs an fp32 oracle: torch BN-backward formula + torch.nn.grad.conv2d_input."""
    from torch.nn.grad import conv2d_input
    from tensorflow_train_distributed_amd.ops import gemm as G
    N, H, K, C, feed = cfg
    torch.manual_seed(7)
    M = N * H * H
    g = torch.randn(N, H, H, K, device="cuda").bfloat16()       # masked output gradient of the unit
    y = torch.randn(N, H, H, K, device="cuda").bfloat16()       # the unit's conv output (BN input)
    coef = torch.randn(3, K, device="cuda") * torch.tensor([[1.0], [0.1], [0.01]], device="cuda")
    w = (torch.randn(K, 1, 1, C, device="cuda") / K ** 0.5).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()
    assert G.dgrad_bnpro_ok((N, H, H, C), tuple(wt.shape))
    dz_ref = coef[0] * g.float() + coef[1] * y.float() + coef[2]
    dx_ref = conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), dz_ref.bfloat16().float().permute(0, 3, 1, 2)
                          ).permute(0, 2, 3, 1)
    dz = torch.empty_like(g)
    if feed:
        fy = torch.randn(N, H, H, C, device="cuda").bfloat16()
        keep = torch.rand(M * C, device="cuda") > 0.4
        bits = keep.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)
        mask = bits.sum(1).to(torch.uint8)
        old = torch.randn(N, H, H, C, device="cuda").bfloat16()
        out = old.clone()
        got, partial, T = G.conv_dgrad(g, wt, (N, H, H, C), out=out, beta=1, bn_stat=(fy, mask), bn_pro=(y, coef, dz))
        ref = (dx_ref + old.float()) * keep.view(N, H, H, C)
        assert _rel(got, ref) < 1e-2
        sums = partial.sum(0)
        gs = got.float().view(-1, C)
        torch.testing.assert_close(sums[0], gs.sum(0), rtol=2e-3, atol=5e-2)
        torch.testing.assert_close(sums[1], (gs * fy.float().view(-1, C)).sum(0), rtol=2e-3, atol=5e-2)
    else:
        got = G.conv_dgrad(g, wt, (N, H, H, C), bn_pro=(y, coef, dz))
        assert _rel(got, dx_ref) < 1e-2
    # dz stored once for the weight gradient: every element, bf16 of the same expression
    assert _rel(dz, dz_ref) < 4e-3


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,splits,beta", [(1024, 1536, 64 * 96, 8, 1), (768, 384, 64 * 40, 5, 0),
                                                (1000, 1032, 64 * 33, 4, 1)])
def test_splitk_in_kernel_fold_256row(M, N, K, splits, beta):
    """Split-K on the 256-row kernel folds its own fp32 slabs: the last split to finish a tile
    (per-tile arrival counter) sums the tile's slabs in split order into the output (+= with
    beta). vs fp32 reference; bitwise deterministic across runs; counters left at zero (a second
    launch on the same stream is also right)."""
    from tensorflow_train_distributed_amd.ops import _lib
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(4)
    a = torch.randn(K, M, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    ref = a.float().t() @ b.float()
    base = torch.randn(M, N, device="cuda")
    outs = []
    old = _lib.query("ttdk_set_inkernel_fold", 1)  # opt-in path (measured slower in the steps)
    try:
        for _ in range(3):
            out = base.clone()
            G.gemm(a, b, trans_a=True, out=out, splits=splits, beta=beta)
            outs.append(out)
    finally:
        _lib.query("ttdk_set_inkernel_fold", old)
    want = ref + base if beta else ref
    assert _rel(outs[0], want) < 1e-4
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [((64, 28, 28, 256), (512, 1, 1, 256), 1, 0), ((32, 14, 14, 256), (256, 3, 3, 256), 1, 1)])
def test_conv_wgrad_in_kernel_fold(shape):
    """Conv weight gradients on the 256-row kernel with split-K fold inside the launch vs fp32."""
    from torch.nn.grad import conv2d_weight
    from tensorflow_train_distributed_amd.ops import gemm as G
    xs, ws, st, pd = shape
    torch.manual_seed(8)
    x = torch.randn(xs, device="cuda").bfloat16()
    N, H, W, C = xs
    K, R, S, _ = ws
    P = (H + 2 * pd - R) // st + 1
    dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
    from tensorflow_train_distributed_amd.ops import _lib
    old = _lib.query("ttdk_set_inkernel_fold", 1)
    try:
        got = G.conv_wgrad(x, dy, ws, (st, st), (pd, pd))
        got2 = G.conv_wgrad(x, dy, ws, (st, st), (pd, pd))
    finally:
        _lib.query("ttdk_set_inkernel_fold", old)
    ref = conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, R, S), dy.float().permute(0, 3, 1, 2), stride=st,
                        padding=pd).permute(0, 2, 3, 1)
    assert _rel(got, ref) < 1e-3
    assert torch.equal(got, got2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(32, 28, 512, 128, False), (64, 14, 1024, 256, True), (17, 17, 512, 256, False)])
def test_conv_fwd_with_bn_apply_operand_prologue(cfg):
    """conv_fwd_bnpro: the 1x1 conv consuming the RAW output y3 of a conv+BN+residual+ReLU unit
    forms h = relu(sc*y3 + sh + r) (projection: + rsc*r + rsh) as its operand in LDS, stores h
    and its ReLU bits, and emits its own BN partial sums — vs the unfused engine ops (bn_apply
    pass + conv) and an fp32 conv of the same h."""
    import torch.nn.functional as F
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    N, H, C, Kout, proj = cfg
    torch.manual_seed(9)
    y3 = torch.randn(N, H, H, C, device="cuda").bfloat16()
    r = torch.randn(N, H, H, C, device="cuda").bfloat16()
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    rsc, rsh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    w = (torch.randn(Kout, 1, 1, C, device="cuda") / C ** 0.5).bfloat16()
    coef = torch.cat([sc, sh, rsc, rsh]) if proj else torch.cat([sc, sh])
    M = N * H * H
    h = torch.empty_like(y3)
    hm = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda")
    y, partial, T = G.conv_fwd_bnpro(y3, w, coef, r, h, hm, proj=proj)
    # reference: the engine's own apply pass (same arithmetic) and an fp32 conv of its output
    mask_ref = torch.empty_like(hm)
    h_ref = K.bn_apply(y3.view(M, C), sc, sh, residual=r.view(M, C), residual_bn=(rsc, rsh) if proj else None,
                       relu=True, mask=mask_ref).view(N, H, H, C)
    assert torch.equal(h, h_ref)
    assert torch.equal(hm, mask_ref)
    y_ref = F.conv2d(h_ref.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert _rel(y, y_ref) < 1e-2
    yf = y.float().view(-1, Kout)
    sums = partial.sum(0)
    torch.testing.assert_close(sums[0], yf.sum(0), rtol=2e-3, atol=5e-2)
    torch.testing.assert_close(sums[1], (yf * yf).sum(0), rtol=2e-3, atol=5e-1)
    assert T == -(-M // 256)


@pytest.mark.gpu
def test_weight_prep_matches_per_conv_transposes_and_phase_filters():
    """ttdk_wprep (one launch for every filter of a network) vs the per-conv transpose and the
    sub-pixel dgrad's own phase gathers: bitwise equal filters, and a strided dgrad fed the
    prepared phase filters (ws=...) equals the one that gathers them itself."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(3)
    shapes = [(64, 1, 1, 256), (128, 3, 3, 128), (256, 3, 3, 64), (40, 5, 5, 24), (2048, 1, 1, 512)]
    sizes = [int(torch.tensor(s).prod()) for s in shapes]
    flat = torch.randn(sum(sizes) + 3, device="cuda").bfloat16()
    wp = K.WeightPrep(flat)
    offs, o = [], 3  # unaligned start on purpose
    for i, (s, n) in enumerate(zip(shapes, sizes)):
        offs.append(o)
        wp.add("w%d" % i, o, s)
        if s[1] > 1:
            wp.add("w%d/phases" % i, o, s, sub=(2, s[1] // 2, s[2] // 2, 15, 13))
        o += n
    wp.build().run()
    for i, (s, n) in enumerate(zip(shapes, sizes)):
        w = flat[offs[i]:offs[i] + n].view(s)
        assert torch.equal(wp.crsk("w%d" % i), K.krsc_to_crsk(w))
    # strided dgrad with the prepared phase filters
    Kc, R, _, C = shapes[1]
    w = flat[offs[1]:offs[1] + sizes[1]].view(shapes[1])
    wt = K.krsc_to_crsk(w)
    x_shape = (2, 15, 13, C)
    dy = torch.randn(2, 8, 7, Kc, device="cuda").bfloat16()
    a = G.conv_dgrad(dy, wt, x_shape, (2, 2), (1, 1))
    b = G.conv_dgrad(dy, torch.zeros_like(wt), x_shape, (2, 2), (1, 1), ws=wp.phases("w1/phases"))
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("four_wave", [True, False])
@pytest.mark.parametrize("cfg", [(8, 14, 14, 256, 256), (4, 28, 28, 128, 128), (2, 7, 7, 512, 512), (3, 9, 11, 264, 128)])
def test_conv_dgrad_fp8_e5m2_vs_fp32_oracle(monkeypatch, cfg, four_wave):
    """fp8 data gradient (e5m2 dy x e4m3 transposed filter, block-scaled MFMA) of a 3x3/s1 conv vs
    F.conv2d's fp32 input gradient on the DEQUANTISED operands (tight), vs the bf16 operands
    (fp8 rounding: loose), and with the feeding-BN statistics epilogue vs the bf16 dgrad's."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    # four_wave: the 4-wave fp8 kernel (reversed-tap gather, feeding-BN epilogue) where the engine
    # takes it (>= 1024-element reduction, >= 256 channels; the 4th shape has partial tiles)
    monkeypatch.setattr(G, "_DGRAD4K8", four_wave)
    N, H, W, C, Kc = cfg
    torch.manual_seed(11)
    w = (torch.randn(Kc, 3, 3, C, device="cuda") / (9 * C) ** 0.5).bfloat16()
    dy = (torch.randn(N, H, W, Kc, device="cuda") * 3e-4).bfloat16()
    s_dy = torch.tensor([57344.0 * 0.5 / float(dy.float().abs().max())], device="cuda")
    s_w = torch.tensor([448.0 / float(w.float().abs().max())], device="cuda")
    dy8 = K.quant_fp8(dy, s_dy, e5m2=True)
    wt = K.krsc_to_crsk(w)
    wt8 = K.quant_fp8(wt, s_w)
    inv = (1.0 / s_dy, 1.0 / s_w)
    dx = G.conv_dgrad_fp8(dy8, wt8, (N, H, W, C), (1, 1), (1, 1), ascale=inv)
    dyq = K.dequant_fp8(dy8, s_dy, e5m2=True).float()
    wq = K.dequant_fp8(wt8, s_w).float()  # [C,3,3,K]
    x = torch.zeros(N, C, H, W, device="cuda", requires_grad=True)
    y = F.conv2d(x, wq.permute(3, 0, 1, 2), padding=1)  # w [K,C,3,3] from the transposed copy
    y.backward(dyq.permute(0, 3, 1, 2))
    ref = x.grad.permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 1e-2
    ref_bf = G.conv_dgrad(dy, wt, (N, H, W, C), (1, 1), (1, 1)).float()
    assert _rel(dx, ref_bf) < 0.12
    # feeding-BN epilogue: masked gradient + (sum g, sum g*y) partial sums
    yb = torch.randn(N, H, W, C, device="cuda").bfloat16()
    mask = torch.randint(0, 256, (N * H * W * C // 8,), dtype=torch.uint8, device="cuda")
    out8, part8, T8 = G.conv_dgrad_fp8(dy8, wt8, (N, H, W, C), (1, 1), (1, 1), ascale=inv, bn_stat=(yb, mask))
    bits = ((mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).view(N, H, W, C).float()
    g_ref = (dx.float() * bits)
    assert _rel(out8, g_ref) < 1e-2
    sums = part8[:T8].sum(0)
    assert torch.allclose(sums[0], out8.float().view(-1, C).sum(0), rtol=2e-2, atol=1e-6)
    assert torch.allclose(sums[1], (out8.float() * yb.float()).view(-1, C).sum(0), rtol=2e-2, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("four_wave", [True, False])
@pytest.mark.parametrize("cfg", [(32, 14, 14, 1024, 256), (128, 7, 7, 512, 2048), (8, 28, 28, 512, 128),
                                 (32, 14, 14, 256, 512)])
def test_conv1x1_fp8_units_vs_fp32_oracle(monkeypatch, cfg, four_wave):
    """The 1x1 fp8 unit of precision="fp8" (ResNet._fp8_conv with fp8_1x1): forward e4m3 x e4m3,
    data gradient e5m2 dz x e4m3 filter accumulating into the shortcut gradient (beta = 1) with the
    feeding BN's masked gradient + (sum g, sum g*y) epilogue, weight gradient e5m2 x e4m3 — each
    vs the fp32 op on the dequantised operands (tight) and vs the bf16 kernels (fp8 rounding)."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    # four_wave: the data gradient (with the accumulate) on the 4-wave fp8 kernel wherever it takes
    # the shape (thresholds lowered for the test), else the 8-wave kernel
    monkeypatch.setattr(G, "_DGRAD4K8", four_wave)
    monkeypatch.setattr(G, "_DGRAD4K8_MINK", 128)
    monkeypatch.setattr(G, "_DGRAD4K8_MINC", 8)
    monkeypatch.setattr(G, "_DGRAD4K8_BETA", True)
    N, H, W, C, Kc = cfg
    torch.manual_seed(23 + C)
    M = N * H * W
    x = torch.randn(N, H, W, C, device="cuda").relu().bfloat16()
    w = (torch.randn(Kc, 1, 1, C, device="cuda") / C ** 0.5).bfloat16()
    dy = (torch.randn(N, H, W, Kc, device="cuda") * 1e-3).bfloat16()
    s_x = torch.tensor([448.0 / float(x.float().abs().max())], device="cuda")
    s_w = torch.tensor([448.0 / float(w.float().abs().max())], device="cuda")
    s_dy = torch.tensor([57344.0 * 0.5 / float(dy.float().abs().max())], device="cuda")
    x8, w8 = K.quant_fp8(x, s_x), K.quant_fp8(w, s_w)
    dy8 = K.quant_fp8(dy, s_dy, e5m2=True)
    wt = K.krsc_to_crsk(w)
    wt8 = K.quant_fp8(wt, s_w)
    # exact decodes (fp8 values are bf16-representable at unit scale), scaled in fp32
    one = torch.ones(1, device="cuda")
    xq = K.dequant_fp8(x8, one).float() / s_x
    wq = K.dequant_fp8(w8, one).float().view(Kc, C) / s_w
    dyq = K.dequant_fp8(dy8, one, e5m2=True).float() / s_dy
    # forward
    y = G.conv_fwd_fp8(x8, w8, (1, 1), (0, 0), ascale=(1.0 / s_x, 1.0 / s_w))
    assert _rel(y, (xq.view(M, C) @ wq.t()).view(N, H, W, Kc)) < 1e-2
    assert _rel(y, G.conv_fwd(x, w, (1, 1), (0, 0)).float()) < 0.08
    # data gradient: dx = old + dz . W, masked, with the feeding BN's sums
    old = (torch.randn(N, H, W, C, device="cuda") * 1e-3).bfloat16()
    out = old.clone()
    yb = torch.randn(N, H, W, C, device="cuda").bfloat16()
    mask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda")
    inv = (1.0 / s_dy, 1.0 / s_w)
    _, part, T = G.conv_dgrad_fp8(dy8, wt8, (N, H, W, C), (1, 1), (0, 0), ascale=inv, out=out, beta=1,
                                  bn_stat=(yb, mask))
    bits = ((mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).view(N, H, W, C).float()
    wtq = K.dequant_fp8(wt8, one).float().view(C, Kc) / s_w
    ref = ((dyq.view(M, Kc) @ wtq.t()).view(N, H, W, C) + old.float()) * bits
    assert _rel(out, ref) < 1e-2
    sums = part[:T].sum(0)
    assert torch.allclose(sums[0], out.float().view(-1, C).sum(0), rtol=2e-2, atol=1e-5)
    assert torch.allclose(sums[1], (out.float() * yb.float()).view(-1, C).sum(0), rtol=2e-2, atol=1e-4)
    ref_bf = (G.conv_dgrad(dy, wt, (N, H, W, C), (1, 1), (0, 0)).float() + old.float()) * bits
    assert _rel(out, ref_bf) < 0.12
    # weight gradient
    assert G.conv_wgrad_fp8_ok(x8.shape, (Kc, 1, 1, C))
    dw = G.conv_wgrad_fp8(x8, dy8, (Kc, 1, 1, C), (1, 1), (0, 0), ascale=(1.0 / s_dy, 1.0 / s_x))
    ref_w = (dyq.view(M, Kc).t() @ xq.view(M, C)).view(Kc, 1, 1, C)
    assert _rel(dw, ref_w) < 1e-4
    assert _rel(dw, G.conv_wgrad(x, dy, (Kc, 1, 1, C), (1, 1), (0, 0))) < 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(4, 14, 14, 256, 256, 3, 1, 1), (8, 7, 7, 512, 512, 3, 1, 1), (4, 28, 28, 128, 128, 3, 2, 1),
                                 (16, 14, 14, 1024, 256, 1, 1, 0), (8, 14, 14, 512, 1024, 1, 2, 0),
                                 (3, 9, 11, 128, 200, 3, 1, 1)])
def test_conv_fwd4k8_vs_fp32_oracle(cfg):
    """fp8 forward conv on the 4-wave kernel (gemm4w.hip gemm4k8_kernel: 32x32x64 block-scaled MFMA,
    K-major fragments, implicit-GEMM DMA gather / dense 1x1 rows) vs F.conv2d on the exactly
    decoded operands (tight), with the BN partial sums per 128 rows vs the stored output, and vs
    the 8-wave fp8 kernel; partial row / column tiles in the last case."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    N, H, W, C, Kc, R, s, p = cfg
    torch.manual_seed(31 + C)
    x = torch.randn(N, H, W, C, device="cuda").relu().bfloat16()
    w = (torch.randn(Kc, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
    s_x = torch.tensor([448.0 / float(x.float().abs().max())], device="cuda")
    s_w = torch.tensor([448.0 / float(w.float().abs().max())], device="cuda")
    x8, w8 = K.quant_fp8(x, s_x), K.quant_fp8(w, s_w)
    one = torch.ones(1, device="cuda")
    xq = K.dequant_fp8(x8, one).float() / s_x
    wq = K.dequant_fp8(w8, one).float() / s_w
    assert G.conv_fwd4k8_ok(x8.shape, w8.shape, (s, s), (p, p))
    y, part, T = G.conv_fwd4k8(x8, w8, (s, s), (p, p), ascale=(1.0 / s_x, 1.0 / s_w))
    ref = F.conv2d(_nchw(xq), wq.permute(0, 3, 1, 2), stride=s, padding=p)
    assert _rel(y, _nhwc(ref)) < 1e-2
    yf = y.float().reshape(-1, Kc)
    sums = part[:T].sum(0)
    torch.testing.assert_close(sums[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(sums[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
    y8 = G.conv_fwd_fp8(x8, w8, (s, s), (p, p), ascale=(1.0 / s_x, 1.0 / s_w))
    assert _rel(y, y8.float()) < 1e-2


@pytest.mark.gpu
def test_bn_backward_apply_e5m2_copy_and_amax():
    """The BN backward-apply pass's OCP e5m2 copy of dz (delayed scale from the slot) dequantises
    to dz within e5m2 rounding, and the slot's amax lanes receive max |dz|."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(5)
    M, C = 4096, 256
    g = (torch.randn(M, C, device="cuda") * 1e-3).bfloat16()
    y = torch.randn(M, C, device="cuda").bfloat16()
    st = K.BNState(C, "cuda")
    st.mean.copy_(y.float().mean(0))
    st.rstd.copy_(torch.rsqrt(y.float().var(0, unbiased=False) + 1e-5))
    gamma = torch.rand(C, device="cuda") + 0.5
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    part = torch.stack([g.float().sum(0), (g.float() * y.float()).sum(0)]).unsqueeze(0).contiguous()
    slot = torch.zeros(K.FP8_SLOT, device="cuda")
    slot[2] = 2.0 ** 16
    slot[3] = 2.0 ** -16
    q8 = torch.empty(M * C, dtype=torch.uint8, device="cuda")
    dz = K.bn_backward_from_partial(g, y, gamma, st, dg, db, part, 1, q8=q8, q8_slot=slot)
    back = K.dequant_fp8(q8, slot[2:3], e5m2=True).float().view(M, C)
    assert _rel(back, dz.float()) < 0.08
    assert abs(float(slot[8:72].max()) - float(dz.float().abs().max())) <= 1e-6 + 1e-2 * float(dz.float().abs().max())


@pytest.mark.parametrize("M,N,K,splits,beta", [(1024, 1024, 8192, 4, 0), (4096, 1024, 4096, 2, 1),
                                               (1024, 4096, 4096, 1, 0), (1032, 1160, 8192, 3, 0)])
def test_weight_gradient_with_fused_bias_rowsum_vs_fp32(M, N, K, splits, beta):
    """gemm_wgrad_bias: dW (+)= dy^T.x on the 256-wide ping-pong kernel AND the bias gradient
    colsum(dy) from the same dy tiles in LDS (gemm256_kernel RS) vs fp32 torch; the last shape
    has a partial 256-row tile (M = 1032) and a non-multiple-of-256 N. Deterministic: two runs
    agree bitwise."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(0)
    dy = (torch.randn(K, M, device="cuda") * 0.5).bfloat16()
    x = torch.randn(K, N, device="cuda").bfloat16()
    assert G.wgrad_bias_ok(M, N, K, splits)
    out0 = torch.randn(M, N, device="cuda")
    out = out0.clone()
    bias = torch.full((M,), 7.0, device="cuda")
    G.gemm_wgrad_bias(dy, x, out, bias, splits=splits, beta=beta)
    ref = dy.float().t() @ x.float() + (out0 if beta else 0)
    rel = float((out - ref).norm() / ref.norm())
    assert rel < 2e-3, rel
    bref = dy.float().sum(0)
    torch.testing.assert_close(bias, bref, rtol=1e-4, atol=1e-3)
    out2 = out0.clone()
    bias2 = torch.zeros(M, device="cuda")
    G.gemm_wgrad_bias(dy, x, out2, bias2, splits=splits, beta=beta)
    assert torch.equal(out, out2) and torch.equal(bias, bias2)
    # the plain split-K path computes the same weight gradient
    out3 = out0.clone()
    G.gemm(dy, x, trans_a=True, out=out3, splits=splits, beta=beta)
    torch.testing.assert_close(out, out3, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("four_wave", [True, False])
@pytest.mark.parametrize("cfg", [(2, 16, 16, 256, 256, 1), (1, 16, 16, 128, 128, 1), (4, 8, 8, 512, 512, 1),
                                 (2, 16, 16, 128, 256, 2), (3, 16, 8, 256, 512, 1), (2, 14, 14, 256, 256, 1),
                                 (16, 8, 8, 512, 512, 1), (8, 16, 16, 256, 256, 2)])
def test_conv_wgrad_fp8_vs_fp32_oracle(monkeypatch, cfg, four_wave):
    """fp8 weight gradient (e5m2 dy x e4m3 im2col(x), both MN-major through ds_read_b64_tr_b8, block-
    scaled MFMA, split-K) of a 3x3 conv vs the fp32 weight gradient of the DEQUANTISED operands
    (tight: only the summation order differs) and vs the bf16 weight gradient (fp8 rounding: loose).
    four_wave: the 4-wave transposed-read kernel's fp8 form (gemm4t8_kernel, 32x32x64 MFMA, split-K
    summed in the launch; partial 256-column tiles at N = 1152 / 2304), else the 8-wave kernel."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    monkeypatch.setattr(G, "_WGRAD4T8", four_wave)
    N, H, W, C, Kc, s = cfg
    torch.manual_seed(17 + C)
    x = torch.randn(N, H, W, C, device="cuda").relu().bfloat16()
    P = (H + 2 - 3) // s + 1
    Q = (W + 2 - 3) // s + 1
    dy = (torch.randn(N, P, Q, Kc, device="cuda") * 1e-3).bfloat16()
    s_x = torch.tensor([448.0 / float(x.float().abs().max())], device="cuda")
    s_dy = torch.tensor([57344.0 * 0.5 / float(dy.float().abs().max())], device="cuda")
    x8 = K.quant_fp8(x, s_x)
    dy8 = K.quant_fp8(dy, s_dy, e5m2=True)
    inv = (1.0 / s_dy, 1.0 / s_x)
    wshape = (Kc, 3, 3, C)
    assert G.conv_wgrad_fp8_ok(x8.shape, wshape, (s, s), (1, 1)) == (N * P * Q % 128 == 0)
    if N * P * Q % 128:
        return
    for splits in (1, 3):
        dw = G.conv_wgrad_fp8(x8, dy8, wshape, (s, s), (1, 1), ascale=inv, splits=splits)
        # exact decodes (fp8 values are bf16-representable at unit scale), scaled in fp32
        one = torch.ones(1, device="cuda")
        xq = K.dequant_fp8(x8, one).float() * inv[1]
        dyq = K.dequant_fp8(dy8, one, e5m2=True).float() * inv[0]
        wv = torch.zeros(Kc, C, 3, 3, device="cuda", requires_grad=True)
        y = F.conv2d(xq.permute(0, 3, 1, 2), wv, stride=s, padding=1)
        y.backward(dyq.permute(0, 3, 1, 2))
        ref = wv.grad.permute(0, 2, 3, 1)
        assert _rel(dw, ref) < 1e-4, splits
    ref_bf = G.conv_wgrad(x, dy, wshape, (s, s), (1, 1))
    assert _rel(dw, ref_bf) < 0.1


@pytest.mark.gpu
def test_persistent_gemm_tile_queue_matches_fp32_and_replays():
    """The persistent 256-row GEMM (> one round of tiles, elementwise epilogue) with its per-XCD
    tile queue: bias + GELU + aux epilogue vs fp32, repeated launches (the queue resets itself)
    bitwise equal, and hipGraph replays of the same launch bitwise equal too."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(31)
    # 264 tiles > 256 CUs, 16 K-tiles: the ping-pong schedule's persistent kernel with a dynamic tail
    M, N, K = 33 * 256, 8 * 256, 1024
    a = (torch.randn(M, K, device="cuda") / 8).bfloat16()
    b = (torch.randn(N, K, device="cuda") / 8).bfloat16()
    bias = torch.randn(N, device="cuda")
    aux = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    y = G.gemm(a, b, trans_b=True, bias=bias, act=G.ACT_GELU, aux=aux, tile=(256, 256))
    pre = a.float() @ b.float().t() + bias
    ref = torch.nn.functional.gelu(pre, approximate="tanh")
    assert _rel(aux, pre) < 5e-3
    assert _rel(y, ref) < 5e-3
    for _ in range(3):
        y2 = G.gemm(a, b, trans_b=True, bias=bias, act=G.ACT_GELU, aux=aux, tile=(256, 256))
        assert torch.equal(y2, y)
    out = torch.empty_like(y)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        G.gemm(a, b, trans_b=True, bias=bias, act=G.ACT_GELU, aux=aux, out=out, tile=(256, 256))  # warm (allocates the queue)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            G.gemm(a, b, trans_b=True, bias=bias, act=G.ACT_GELU, aux=aux, out=out, tile=(256, 256))
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, y)
