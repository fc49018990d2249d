"""The 4-wave 256x256 AGPR-accumulator GEMM (gemm4w.hip) vs a PyTorch fp32 reference.

Pins the kernel that carries BERT's dense layers (tf.layers.dense MatMul,
/root/reference/distribute_training.py:54,61): the plain store, the bias, bias + GELU + pre-activation
(aux) copy, dGELU and accumulate (beta) epilogues, at BERT-Large shapes and at edge shapes
(M and N not multiples of 256, rows past M / N read as zeros by the buffer loads) and at ResNet-50
1x1-conv GEMM shapes."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


SHAPES = [(256, 256, 128), (512, 512, 128), (1000, 264, 384), (300, 1000, 1024), (4096, 4096, 1024),
          (2048, 1024, 4096), (65, 8, 128),
          # ResNet-50 b256 1x1 convs as GEMMs (pixels x Cout x Cin): stage-4 c3, stage-5 c1
          (12544, 1024, 256), (3136, 512, 2048)]


@pytest.fixture(params=[3, 30, 0], ids=["asm_sched3", "persistent", "compiler_sched"])
def sched(request):
    from tensorflow_train_distributed_amd.ops import gemm as G
    old = G.set_g4_sched(request.param)
    yield request.param
    G.set_g4_sched(old)


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm4w_plain_vs_fp32(M, N, K, sched):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(M + N + K)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    ref = a.float() @ b.float().t()
    out = G.gemm4w(a, b)
    assert _rel(out, ref) < 8e-3
    # asymmetric check of the output layout: a = I picks rows of b
    if M == N == 256:
        eye = torch.eye(256, K, device="cuda").bfloat16()
        assert torch.equal(G.gemm4w(eye, b), (eye.float() @ b.float().t()).bfloat16())


@pytest.mark.parametrize("M,N,K", [(1000, 264, 384), (4096, 4096, 1024)])
def test_gemm4w_epilogues_vs_fp32(M, N, K, sched):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(7)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() * 0.1
    bias = torch.randn(N, device="cuda")
    acc = a.float() @ b.float().t()
    # bias
    assert _rel(G.gemm4w(a, b, bias=bias), acc + bias) < 8e-3
    # bias + GELU with the pre-activation copy
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = G.gemm4w(a, b, bias=bias, act=G.ACT_GELU, aux=pre)
    assert _rel(pre, acc + bias) < 8e-3
    assert _rel(y, F.gelu(acc + bias, approximate="tanh")) < 1e-2
    # dGELU: out = acc * gelu'(residual)
    r = torch.randn(M, N, device="cuda").bfloat16()
    rr = r.float().requires_grad_(True)
    g = torch.autograd.grad(F.gelu(rr, approximate="tanh"), rr, torch.ones_like(rr))[0]
    assert _rel(G.gemm4w(a, b, act=G.ACT_DGELU, residual=r), acc * g) < 1e-2
    # beta: out = acc + out
    old = torch.randn(M, N, device="cuda").bfloat16()
    o = old.clone()
    G.gemm4w(a, b, out=o, beta=1)
    assert _rel(o, acc + old.float()) < 8e-3


def test_gemm4w_strided_operands(sched):
    """Column slices of a fused buffer as operands (row stride = leading dimension)."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(3)
    big = (torch.rand(512, 3 * 256, device="cuda") * 2 - 1).bfloat16()
    a = big[:, 256:512]
    b = (torch.rand(384, 256, device="cuda") * 2 - 1).bfloat16()
    out = G.gemm4w(a, b)
    assert _rel(out, a.float() @ b.float().t()) < 8e-3


@pytest.mark.parametrize("N,H,C,K,R,stride", [
    (8, 14, 256, 256, 3, 1),    # stage-4 3x3
    (8, 28, 128, 128, 3, 2),    # stage-3 block-1 3x3 stride 2
    (8, 14, 512, 512, 3, 2),    # stage-5 block-1 3x3 stride 2
    (8, 7, 512, 512, 3, 1),     # stage-5 3x3
    (8, 14, 256, 1024, 1, 1),   # stage-4 c3 (dense operand)
    (8, 7, 2048, 512, 1, 1),    # stage-5 c1
    (8, 28, 512, 1024, 1, 2),   # stage-4 projection (1x1 stride 2: gathered)
    (3, 9, 64, 72, 3, 1),       # C = 64, odd spatial size, M and K not multiples of 256
])
def test_conv_fwd4w_vs_fp32(N, H, C, K, R, stride):
    """Forward conv on the 4-wave kernel (im2col gather through the operand DMA, zeros for the
    padding taps) vs F.conv2d in fp32, and its BN partial sums vs the stored output's."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(N + H + C + K + R + stride)
    pad = R // 2
    x = (torch.rand(N, H, H, C, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(K, R, R, C, device="cuda") * 2 - 1) * (1.0 / (R * R * C) ** 0.5)).bfloat16()
    y, part, T = G.conv_fwd4w(x, w, (stride, stride), (pad, pad))
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=stride, padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 8e-3
    M = y.numel() // K
    assert T == 2 * -(-M // 256)
    yf = y.float().reshape(M, K)
    s = part.sum(0)
    assert _rel(s[0], yf.sum(0)) < 1e-4
    assert _rel(s[1], (yf * yf).sum(0)) < 1e-4
    # no statistics requested: same output bits
    y2, p2, _ = G.conv_fwd4w(x, w, (stride, stride), (pad, pad), stat=False)
    assert p2 is None and torch.equal(y, y2)


@pytest.mark.parametrize("N,H,C,K,R", [
    (8, 14, 256, 256, 3),   # stage-4 c2 data gradient
    (8, 7, 512, 512, 3),    # stage-5 c2
    (3, 9, 72, 64, 3),      # K = 64 channels of dy, C = 72, odd spatial size
])
def test_conv_dgrad4w_feed_vs_fp32(N, H, C, K, R):
    """3x3 unit-stride data gradient on the 4-wave kernel (dy gathered with reversed taps) with the
    feeding-BN epilogue: g = dx * ReLU bits stored, partial sums (sum g, sum g * y), vs fp32."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(N + H + C + K)
    pad = R // 2
    dy = (torch.rand(N, H, H, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(K, R, R, C, device="cuda") * 2 - 1) * (1.0 / (R * R * K) ** 0.5)).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()  # [C][R][S][K]
    y = (torch.rand(N, H, H, C, device="cuda") * 2 - 1).bfloat16()
    M = N * H * H
    mask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda")
    old = G._DGRAD4W
    G._DGRAD4W = 2
    try:
        out, part, T = G.conv_dgrad(dy, wt, (N, H, H, C), (1, 1), (pad, pad), bn_stat=(y, mask))
        kinds = []
        saved, G._LOG = G._LOG, []
        try:
            G.conv_dgrad(dy, wt, (N, H, H, C), (1, 1), (pad, pad), bn_stat=(y, mask))
            kinds = [e_[0] for e_ in G.gemm_log()]
        finally:
            G._LOG = saved
    finally:
        G._DGRAD4W = old
    assert any(k_.startswith("dgrad4w") for k_ in kinds), kinds
    dx = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                    padding=pad).permute(0, 2, 3, 1).reshape(M, C)
    bits = ((mask.view(-1, 1).int() >> torch.arange(8, device="cuda")) & 1).reshape(M, C).float()
    ref = dx * bits
    got = out.float().reshape(M, C)
    assert _rel(got, ref) < 8e-3
    assert torch.all(got[bits == 0] == 0)
    assert T == 2 * -(-M // 256)
    s = part.sum(0)
    yf = y.float().reshape(M, C)
    assert _rel(s[0], got.sum(0)) < 1e-4
    assert _rel(s[1], (got * yf).sum(0)) < 1e-4
