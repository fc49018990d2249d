"""The 4-wave transposed-read weight-gradient GEMM (gemm4t.hip) vs a PyTorch fp32 reference.

Pins the kernel that carries BERT's dense-layer weight gradients (the kernel gradients of
tf.layers.dense, /root/reference/distribute_training.py:54,61, formed by compute_gradients at
:152): dW = dy^T . x on MN-major operands with the split-K sum inside the launch, the fused bias
gradient (column sums of dy), accumulate (beta) and alpha, at BERT-Large shapes and edge shapes
(M, N not multiples of 256; row-strided operands), and the 128-row tile form taken by outputs of at
most 128 rows (ResNet stage-2/3 convs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K,splits", [
    (256, 256, 128, 1), (256, 256, 1024, 4), (512, 768, 2048, 3), (264, 1000, 384, 2), (1000, 264, 640, 5),
    (1024, 1024, 8192, 16), (3072, 1024, 8192, 4), (4096, 1024, 4096, 3), (8, 16, 128, 1),
    # <= 128 output rows: the 128-row tile form (gemm4t.hip g4t_bm)
    (128, 512, 4096, 8), (64, 576, 2048, 4), (128, 1152, 1024, 3), (120, 264, 640, 2), (128, 256, 128, 1)])
def test_gemm4t_vs_fp32(M, N, K, splits):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(M + N + K + splits)
    dy = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
    x = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    ref = dy.float().t() @ x.float()
    out = G.gemm4t(dy, x, splits=splits)
    assert _rel(out, ref) < 1e-5
    # the counters are left zeroed: a second launch on the same stream gives the same bits
    out2 = G.gemm4t(dy, x, splits=splits)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M,N,K,splits", [(1024, 4096, 4096, 3), (264, 1000, 384, 2), (3072, 1024, 2048, 1)])
def test_gemm4t_bias_beta_alpha(M, N, K, splits):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(11)
    dy = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
    x = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    ref = dy.float().t() @ x.float()
    old = torch.randn(M, N, device="cuda")
    out = old.clone()
    bias = torch.full((M,), 123.0, device="cuda")
    G.gemm4t(dy, x, out, bias, splits=splits, beta=1, alpha=0.5)
    assert _rel(out, 0.5 * ref + old) < 1e-5
    assert _rel(bias, dy.float().sum(0)) < 1e-5


def test_gemm4t_strided_operands():
    """Column slices of fused buffers (row stride = leading dimension), as the fused QKV gradient."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(5)
    big = (torch.rand(2048, 3 * 256, device="cuda") * 2 - 1).bfloat16()
    dy = big[:, 256:512]
    x = (torch.rand(2048, 384, device="cuda") * 2 - 1).bfloat16()
    bias = torch.empty(256, device="cuda")
    out = G.gemm4t(dy, x, None, bias, splits=4)
    assert _rel(out, dy.float().t() @ x.float()) < 1e-5
    assert _rel(bias, dy.float().sum(0)) < 1e-5


def test_wgrad_bias_entry_takes_gemm4t():
    """ops.gemm.gemm_wgrad_bias (the BERT engine's call) routes to the 4-wave kernel and agrees."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(9)
    K, M, N = 4096, 1024, 1024
    dy = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
    x = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    out = torch.empty(M, N, device="cuda")
    bias = torch.empty(M, device="cuda")
    splits = G.gemm_wgrad_splits(M, N, K, big_wgs=192)
    assert G.wgrad_bias_ok(M, N, K, splits)
    G.gemm_wgrad_bias(dy, x, out, bias, splits=splits)
    assert _rel(out, dy.float().t() @ x.float()) < 1e-5
    assert _rel(bias, dy.float().sum(0)) < 1e-5


@pytest.mark.parametrize("beta", [0, 1])
def test_conv_wgrad_1x1_takes_gemm4t(beta):
    """ops.gemm.conv_wgrad of a unit-stride 1x1 conv with >= 256 input and output channels (the
    ResNet-50 stage 3/4 weight gradients) runs on the 4-wave transposed-read kernel."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(13)
    x = (torch.rand(8, 16, 16, 256, device="cuda") * 2 - 1).bfloat16()
    dy = (torch.rand(8, 16, 16, 512, device="cuda") * 2 - 1).bfloat16()
    ref = dy.reshape(-1, 512).float().t() @ x.reshape(-1, 256).float()
    out = torch.randn(512, 1, 1, 256, device="cuda")
    old = out.clone()
    G.conv_wgrad(x, dy, (512, 1, 1, 256), out=out, beta=beta, splits=4)
    want = ref + (old.view(512, 256) if beta else 0)
    assert _rel(out.view(512, 256), want) < 1e-5


# --- convolution weight gradients on the 4-wave kernel with the im2col gather of x -------------
# (the kernel gradients of the ResNet-50 convs; b1024 stage shapes: stage 4/5 3x3, strided 3x3 /
# 1x1 projections, unit-stride 1x1), vs torch.nn.grad.conv2d_weight in fp32 on the same bf16 data

def _conv_wgrad_ref(x, dy, w_shape, stride, pad):
    xf = x.float().permute(0, 3, 1, 2)
    dyf = dy.float().permute(0, 3, 1, 2)
    K, R, S, C = w_shape
    dw = torch.nn.grad.conv2d_weight(xf, (K, C, R, S), dyf, stride=stride, padding=pad)
    return dw.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("N,H,C,K,R,stride,splits", [
    (1024, 14, 256, 256, 3, 1, None),    # stage 4 c2 (3x3, pad 1)
    (1024, 14, 512, 512, 3, 2, None),    # stage 5 block-1 c2 (3x3 stride 2)
    (1024, 7, 512, 512, 3, 1, None),     # stage 5 c2
    (1024, 14, 1024, 2048, 1, 2, None),  # stage 5 projection (1x1 stride 2)
    (1024, 28, 512, 1024, 1, 2, None),   # stage 4 projection
    (1024, 14, 256, 1024, 1, 1, None),   # stage 4 c3 (unit-stride 1x1: dense operands)
    (64, 9, 64, 256, 3, 1, 3),           # odd spatial size, C = 64 (four taps per 256 columns)
    (16, 12, 128, 264, 3, 2, 1),         # K not a multiple of 256, one split (576 pixels)
    (4, 8, 8, 256, 3, 1, 2),             # C = 8 (256 pixels): 32 taps of 8 channels per 256 columns
    # 128-row tiles (<= 128 output channels): stage-3 c2 / block-1 c2 / c1, stage-2 c2 (batch 64)
    (64, 28, 128, 128, 3, 1, None),
    (64, 56, 128, 128, 3, 2, None),
    (64, 28, 512, 128, 1, 1, None),
    (64, 56, 64, 64, 3, 1, None),
])
def test_conv_wgrad4t_vs_fp32(N, H, C, K, R, stride, splits):
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(N + H + C + K + R + stride)
    pad = R // 2
    x = (torch.rand(N, H, H, C, device="cuda") * 2 - 1).bfloat16()
    P = (H + 2 * pad - R) // stride + 1
    dy = (torch.rand(N, P, P, K, device="cuda") * 2 - 1).bfloat16()
    w_shape = (K, R, R, C)
    ref = _conv_wgrad_ref(x, dy, w_shape, stride, pad)
    out = G.conv_wgrad4t(x, dy, w_shape, (stride, stride), (pad, pad), splits=splits)
    assert _rel(out, ref) < 1e-5
    # deterministic (fixed split order), counters left zeroed for the next launch
    out2 = G.conv_wgrad4t(x, dy, w_shape, (stride, stride), (pad, pad), splits=splits)
    assert torch.equal(out, out2)
    # accumulate
    old = torch.randn_like(ref)
    acc = old.clone()
    G.conv_wgrad4t(x, dy, w_shape, (stride, stride), (pad, pad), out=acc, beta=1, splits=splits)
    assert _rel(acc, ref + old) < 1e-5


def test_conv_wgrad_dispatches_to_4wave_kernel():
    """ops.gemm.conv_wgrad routes a stage-4 3x3 weight gradient to the 4-wave kernel (launch log)."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    x = (torch.rand(64, 14, 14, 256, device="cuda") * 2 - 1).bfloat16()
    dy = (torch.rand(64, 14, 14, 256, device="cuda") * 2 - 1).bfloat16()
    saved, G._LOG = G._LOG, []
    try:
        out = G.conv_wgrad(x, dy, (256, 3, 3, 256), (1, 1), (1, 1))
        kinds = [e[0] for e in G.gemm_log()]
    finally:
        G._LOG = saved
    assert any(k.startswith("wgrad4t_3x3") for k in kinds), kinds
    assert _rel(out, _conv_wgrad_ref(x, dy, (256, 3, 3, 256), 1, 1)) < 1e-5
