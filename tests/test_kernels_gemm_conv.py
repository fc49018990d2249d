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
