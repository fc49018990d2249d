"""Halo-tiled 3x3 conv kernel (csrc/kernels/conv3_halo.hip) vs an fp32 PyTorch conv oracle and
vs the kernels it replaces (bn_apply / bn_bwd_apply + the tiled implicit-GEMM engine):

* plain forward (+ per-tile BN statistics) matches the fp32 convolution of the same bf16 input;
* BN-forward prologue: the written activation and ReLU bits are bit-identical to ttdk_bn_apply,
  the output matches the convolution of that activation;
* data gradient (flipped transposed filter) matches conv_dgrad; with the BN-backward prologue
  the written dz matches ttdk_bn_bwd_apply and the ReLU-masked output + BN-backward sums match
  conv_dgrad(bn_stat=...) on the same dz.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

NIMG, H, W, C, N = 3, 56, 56, 64, 64


def _ops():
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    return G, K


def _rand(shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(shape, generator=g, device="cuda") * scale).to(torch.bfloat16)


def _conv_ref(x, w):
    """fp32 NHWC 3x3/s1/p1 conv: x [N,H,W,C], w [K,3,3,C] -> [N,H,W,K]."""
    return F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max())


def test_conv3_plain_forward_and_stats():
    G, _ = _ops()
    x = _rand((NIMG, H, W, C), seed=1)
    w = _rand((N, 3, 3, C), scale=(9 * C) ** -0.5, seed=2)
    out, partial, T = G.conv3_halo(x, w, stat=True)
    torch.cuda.synchronize()
    assert T == NIMG * H * W // G.conv3_rows(H, W, C, N)
    assert _rel(out, _conv_ref(x, w)) < 1e-2
    o = out.float().reshape(-1, N)
    torch.testing.assert_close(partial[:, 0].sum(0), o.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(partial[:, 1].sum(0), (o * o).sum(0), rtol=1e-3, atol=1e-1)


def test_conv3_bn_forward_prologue_matches_apply():
    G, K = _ops()
    y = _rand((NIMG, H, W, C), seed=3)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.2
    w = _rand((N, 3, 3, C), scale=(9 * C) ** -0.5, seed=4)
    want = torch.empty_like(y)
    want_mask = torch.zeros(y.numel() // 8, dtype=torch.uint8, device="cuda")
    K.bn_apply(y.view(-1, C), sc, sh, relu=True, out=want.view(-1, C), mask=want_mask)
    side = torch.empty_like(y)
    side_mask = torch.zeros_like(want_mask)
    out, partial, T = G.conv3_halo(y, w, prologue=("bn_fwd", sc, sh, side, side_mask), stat=True)
    torch.cuda.synchronize()
    assert torch.equal(side, want)
    assert torch.equal(side_mask, want_mask)
    assert _rel(out, _conv_ref(want, w)) < 1e-2
    torch.testing.assert_close(partial[:, 0].sum(0), out.float().reshape(-1, N).sum(0), rtol=1e-3, atol=1e-1)


def test_conv3_dgrad_matches_conv_dgrad():
    G, K = _ops()
    dz = _rand((NIMG, H, W, N), seed=5)
    w = _rand((N, 3, 3, C), scale=(9 * C) ** -0.5, seed=6)
    wt = K.krsc_to_crsk(w)  # [C, 3, 3, N]
    got = G.conv3_halo(dz, wt, flip=True)
    ref = G.conv_dgrad(dz, wt, (NIMG, H, W, C), (1, 1), (1, 1))
    torch.cuda.synchronize()
    # exact oracle: dx = conv_transpose(dz, w)
    oracle = F.conv_transpose2d(dz.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    assert _rel(got, oracle.permute(0, 2, 3, 1)) < 1e-2
    assert _rel(got, ref) < 1e-2


def test_conv3_bn_backward_prologue_and_stat_epilogue():
    from tensorflow_train_distributed_amd.ops import _lib
    G, K = _ops()
    g = _rand((NIMG, H, W, N), seed=7)
    y = _rand((NIMG, H, W, N), seed=8)
    coef = torch.randn(3, N, device="cuda") * torch.tensor([[1.0], [0.1], [0.05]], device="cuda")
    w = _rand((N, 3, 3, C), scale=(9 * C) ** -0.5, seed=9)
    wt = K.krsc_to_crsk(w)
    M = NIMG * H * W
    want_dz = torch.empty_like(g)
    _lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, None, y.data_ptr(), coef.data_ptr(), want_dz.data_ptr(),
              M * N, N, _lib.stream())
    fy = _rand((NIMG, H, W, C), seed=10)
    fmask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda")
    ref, rpart, rT = G.conv_dgrad(want_dz, wt, (NIMG, H, W, C), (1, 1), (1, 1), bn_stat=(fy, fmask))
    side = torch.empty_like(g)
    out, part, T = G.conv3_halo(g, wt, flip=True, prologue=("bn_bwd", y, None, coef, side), bn_stat=(fy, fmask))
    torch.cuda.synchronize()
    torch.testing.assert_close(side.float(), want_dz.float(), rtol=8e-3, atol=1e-5)
    assert _rel(out, ref) < 2e-2
    torch.testing.assert_close(part.sum(0), rpart.sum(0), rtol=2e-2, atol=2.0)


# ---- stage-3 streamed-filter variant (28 x 28, 128 -> 128): tiles of 8 rows of the flattened
# (image, row) sequence, so tiles straddle images and NIMG = 3 ends in a partial tile
S3 = (3, 28, 28, 128, 128)


@pytest.fixture
def s3_on():
    from tensorflow_train_distributed_amd.ops import gemm as G
    old = G.set_conv3_s3(True)
    yield
    G.set_conv3_s3(old)


def test_conv3_stage3_streamed_forward_bn_prologue_and_stats(s3_on):
    G, K = _ops()
    nimg, h, w_, c, n = S3
    assert G.conv3_rows(h, w_, c, n) == 8 * w_
    y = _rand((nimg, h, w_, c), seed=11)
    sc = torch.rand(c, device="cuda") + 0.5
    sh = torch.randn(c, device="cuda") * 0.2
    w = _rand((n, 3, 3, c), scale=(9 * c) ** -0.5, seed=12)
    want = torch.empty_like(y)
    want_mask = torch.zeros(y.numel() // 8, dtype=torch.uint8, device="cuda")
    K.bn_apply(y.view(-1, c), sc, sh, relu=True, out=want.view(-1, c), mask=want_mask)
    side = torch.empty_like(y)
    side_mask = torch.zeros_like(want_mask)
    out, partial, T = G.conv3_halo(y, w, prologue=("bn_fwd", sc, sh, side, side_mask), stat=True)
    torch.cuda.synchronize()
    assert T == -(-nimg * h // 8)
    assert torch.equal(side, want) and torch.equal(side_mask, want_mask)
    ref = _conv_ref(want, w)
    assert _rel(out, ref) < 1e-2
    o = out.float().reshape(-1, n)
    torch.testing.assert_close(partial[:, 0].sum(0), o.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(partial[:, 1].sum(0), (o * o).sum(0), rtol=1e-3, atol=1e-1)
    # plain forward on the same kernel family
    out0 = G.conv3_halo(want, w)
    torch.cuda.synchronize()
    assert _rel(out0, ref) < 1e-2


def test_conv3_stage3_streamed_dgrad_with_bn_stat_epilogue(s3_on):
    G, K = _ops()
    nimg, h, w_, c, n = S3
    dz = _rand((nimg, h, w_, n), seed=13)
    w = _rand((n, 3, 3, c), scale=(9 * c) ** -0.5, seed=14)
    wt = K.krsc_to_crsk(w)
    oracle = F.conv_transpose2d(dz.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    got = G.conv3_halo(dz, wt, flip=True)
    torch.cuda.synchronize()
    assert _rel(got, oracle.permute(0, 2, 3, 1)) < 1e-2
    M = nimg * h * w_
    fy = _rand((nimg, h, w_, c), seed=15)
    fmask = torch.randint(0, 256, (M * c // 8,), dtype=torch.uint8, device="cuda")
    ref, rpart, _ = G.conv_dgrad(dz, wt, (nimg, h, w_, c), (1, 1), (1, 1), bn_stat=(fy, fmask))
    out, part, T = G.conv3_halo(dz, wt, flip=True, bn_stat=(fy, fmask))
    torch.cuda.synchronize()
    assert _rel(out, ref) < 2e-2
    torch.testing.assert_close(part.sum(0), rpart.sum(0), rtol=2e-2, atol=2.0)
