"""Streaming pointwise-conv kernel (csrc/kernels/pw_gemm.hip) vs fp32 PyTorch references and
vs the kernels it replaces (bn_apply / bn_bwd_apply + the tiled GEMM engine):

* plain GEMM (+ per-tile BN statistics) for every (K, N) tile configuration, ragged M;
* BN-forward prologue: the stored unit output and ReLU bits are bit-identical to ttdk_bn_apply
  (with residual and with the projection-shortcut residual BN), the product matches A' . w^T;
* BN-backward prologue: dz matches ttdk_bn_bwd_apply (same expression, up to fma contraction); with the dgrad-style epilogue
  (accumulate into the shortcut gradient, ReLU-masked gradient + BN-backward sums of the next
  unit, second statistics source) the outputs match conv_dgrad on the same dz.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    return G, K


def _rand(shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(shape, generator=g, device="cuda") * scale).to(torch.bfloat16)


CASES = [(64, 256), (64, 128), (64, 64), (128, 512), (128, 128), (128, 64), (256, 64), (256, 512), (512, 128)]


@pytest.mark.parametrize("K,N", CASES)
def test_pw_plain_and_stats(K, N):
    G, _ = _ops()
    M = 8 * 56 * 56 + 77  # ragged last tile
    x = _rand((M, K), seed=1)
    w = _rand((N, K), scale=K ** -0.5, seed=2)
    out, partial, T = G.pw_conv(x, w, stat=True)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().T
    assert T == -(-M // G.pw_rows(N, K))
    err = (out.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, err
    o = out.float()
    torch.testing.assert_close(partial[:, 0].sum(0), o.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(partial[:, 1].sum(0), (o * o).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("K,N,proj", [(64, 256, False), (256, 64, True), (128, 512, False), (512, 128, True)])
def test_pw_bn_forward_prologue_matches_apply(K, N, proj):
    G, Kk = _ops()
    M = 4 * 28 * 28 + 5
    y = _rand((M, K), seed=3)
    res = _rand((M, K), seed=4)
    sc = torch.rand(K, device="cuda") + 0.5
    sh = torch.randn(K, device="cuda") * 0.2
    rsc = torch.rand(K, device="cuda") + 0.5 if proj else None
    rsh = torch.randn(K, device="cuda") * 0.2 if proj else None
    w = _rand((N, K), scale=K ** -0.5, seed=5)
    want = torch.empty_like(y)
    want_mask = torch.zeros(M * K // 8, dtype=torch.uint8, device="cuda")
    Kk.bn_apply(y, sc, sh, residual=res, residual_bn=(rsc, rsh) if proj else None, relu=True, out=want,
                mask=want_mask)
    side = torch.empty_like(y)
    side_mask = torch.zeros_like(want_mask)
    out, partial, T = G.pw_conv(y, w, prologue=("bn_fwd", sc, sh, res, rsc, rsh, side, side_mask), stat=True)
    torch.cuda.synchronize()
    assert torch.equal(side, want)
    assert torch.equal(side_mask, want_mask)
    ref = want.float() @ w.float().T
    assert (out.float() - ref).abs().max() / ref.abs().max() < 1e-2
    torch.testing.assert_close(partial[:, 0].sum(0), out.float().sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("K,N,second", [(64, 256, False), (256, 64, True), (128, 512, True)])
def test_pw_bn_backward_prologue_matches_dgrad_path(K, N, second):
    from tensorflow_train_distributed_amd.ops import _lib
    G, Kk = _ops()
    Nimg, H, W = 4, 28, 28
    M = Nimg * H * W
    g = _rand((M, K), seed=6)
    y = _rand((M, K), seed=7)
    bits = torch.randint(0, 256, (M * K // 8,), dtype=torch.uint8, device="cuda")
    coef = torch.randn(3, K, device="cuda") * torch.tensor([[1.0], [0.1], [0.05]], device="cuda")
    w = _rand((K, N), scale=K ** -0.5, seed=8)  # forward conv weight [Kout=K][Cin=N]
    wt = w.t().contiguous()                      # dgrad B operand [C=N][K]
    want_dz = torch.empty_like(g)
    _lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, bits.data_ptr(), y.data_ptr(), coef.data_ptr(),
              want_dz.data_ptr(), M * K, K, _lib.stream())
    # the consuming unit (this dgrad's output feeds its BN backward): y2 + ReLU bits, + a shortcut grad
    y2 = _rand((Nimg, H, W, N), seed=9)
    bits2 = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device="cuda")
    y3 = _rand((Nimg, H, W, N), seed=10) if second else None
    acc0 = _rand((Nimg, H, W, N), seed=11)
    ref_out = acc0.clone()
    r = G.conv_dgrad(want_dz.view(Nimg, H, W, K), wt.view(N, 1, 1, K), (Nimg, H, W, N), out=ref_out, beta=1,
                     bn_stat=(y2, bits2), bn_stat2=y3)
    side = torch.empty_like(g)
    out = acc0.clone()
    got = G.pw_conv(g.view(Nimg, H, W, K), wt, prologue=("bn_bwd", y, bits, coef, side), out=out, beta=1,
                    bn_stat=(y2, bits2), bn_stat2=y3)
    torch.cuda.synchronize()
    # same expression as ttdk_bn_bwd_apply; fma contraction may differ by one bf16 rounding step
    torch.testing.assert_close(side.float(), want_dz.float(), rtol=8e-3, atol=1e-5)
    rel = (out.float() - ref_out.float()).abs().max() / ref_out.float().abs().max()
    assert rel < 2e-2, rel
    for a, b in zip((got[1],) + ((got[3],) if second else ()), (r[1],) + ((r[3],) if second else ())):
        torch.testing.assert_close(a.sum(0), b.sum(0), rtol=2e-2, atol=2.0)


@pytest.mark.parametrize("K,N,dgrad_epi", [(256, 64, True), (64, 256, True), (256, 64, False), (64, 256, False),
                                            (64, 64, False), (64, 64, True)])
def test_pw_bn_backward_prologue_fused_weight_gradient(K, N, dgrad_epi):
    """wgrad=(x, dw): the weight gradient formed from the dz tile in LDS (dz never stored) equals
    the fp32 dz^T . x of the dz the unfused kernel stores, and the data gradient / statistics
    are the unfused kernel's, bit for bit (same kernel body)."""
    G, _ = _ops()
    Nimg, H, W = 6, 28, 28
    M = Nimg * H * W - 37  # ragged last tile
    g = _rand((M, K), seed=12)
    y = _rand((M, K), seed=13)
    bits = torch.randint(0, 256, (M * K // 8,), dtype=torch.uint8, device="cuda")
    coef = torch.randn(3, K, device="cuda") * torch.tensor([[1.0], [0.1], [0.05]], device="cuda")
    wt = _rand((N, K), scale=K ** -0.5, seed=14)  # dgrad B operand [C=N][K]
    x = _rand((M, N), seed=15)                   # the conv input
    assert G.pw_wgrad_fusable(M, N, K, dgrad_epi)
    kw = {}
    if dgrad_epi:
        kw = dict(beta=1, bn_stat=(_rand((M, N), seed=16), torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8,
                                                                          device="cuda")))
    acc0 = _rand((M, N), seed=17)
    side = torch.empty_like(g)
    out_a = acc0.clone()
    ra = G.pw_conv(g, wt, prologue=("bn_bwd", y, bits, coef, side), out=out_a, **kw)
    out_b = acc0.clone()
    dw = torch.full((K, N), float("nan"), device="cuda")
    rb = G.pw_conv(g, wt, prologue=("bn_bwd", y, bits, coef, None), out=out_b, wgrad=(x, dw), **kw)
    dw2 = torch.ones((K, N), device="cuda")
    G.pw_conv(g, wt, prologue=("bn_bwd", y, bits, coef, None), out=acc0.clone(), wgrad=(x, dw2, 1), **kw)
    dw3 = torch.empty((K, N), device="cuda")  # capped persistent grid (side-stream launches)
    out_c = acc0.clone()
    G.pw_conv(g, wt, prologue=("bn_bwd", y, bits, coef, None), out=out_c, wgrad=(x, dw3), max_wgs=64, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out_a, out_b) and torch.equal(out_a, out_c)
    torch.testing.assert_close(dw3, dw, rtol=1e-4, atol=1e-4 * float(dw.abs().max()))
    if dgrad_epi:
        assert torch.equal(ra[1], rb[1])
    ref = side.float().t() @ x.float()
    rel = (dw - ref).abs().max() / ref.abs().max()
    assert rel < 1e-3, rel
    torch.testing.assert_close(dw2, ref + 1.0, rtol=1e-3, atol=1e-3 * float(ref.abs().max()))
