"""Numerics of BN / pooling / xent / element-wise / fp8 / optimizer kernels vs PyTorch fp32."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_batchnorm_fwd_bwd_relu_residual():
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(0)
    M, C = 3000, 96
    y = (torch.randn(M, C, device="cuda") * 2 + 1).bfloat16()
    res = torch.randn(M, C, device="cuda").bfloat16()
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda")
    rm = torch.zeros(C, device="cuda")
    rv = torch.ones(C, device="cuda")
    partial, T = K.bn_stats_partial(y)
    sums = K.bn_reduce_partials(partial, T, C)
    st = K.BNState(C, "cuda")
    K.bn_fwd_finalize(sums, M, gamma, beta, 1e-5, 0.9, rm, rv, st)
    out = K.bn_apply(y, st.scale, st.shift, residual=res, relu=True)
    yr = y.float().requires_grad_(True)
    g_r = gamma.clone().requires_grad_(True)
    b_r = beta.clone().requires_grad_(True)
    ref = torch.relu(F.batch_norm(yr, None, None, g_r, b_r, training=True, eps=1e-5) + res.float())
    assert _rel(out, ref) < 1e-2
    torch.testing.assert_close(rm, 0.1 * y.float().mean(0), rtol=1e-3, atol=1e-3)
    dout = torch.randn(M, C, device="cuda").bfloat16()
    ref.backward(dout.float())
    dg = torch.empty(C, device="cuda")
    db = torch.empty(C, device="cuda")
    g_sc = torch.empty_like(dout)
    dz = K.bn_backward(dout, out, y, gamma, st, dg, db, g_out=g_sc)
    assert _rel(dz, yr.grad) < 2e-2
    assert _rel(dg, g_r.grad) < 1e-2
    assert _rel(db, b_r.grad) < 1e-2
    assert _rel(g_sc, dout.float() * (out.float() > 0)) < 1e-6
    # bit-mask ReLU path (what the ResNet engine uses): identical results without re-reading out
    mask = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda")
    out2 = K.bn_apply(y, st.scale, st.shift, residual=res, relu=True, mask=mask)
    assert torch.equal(out2, out)
    bits = ((mask[:, None].int() >> torch.arange(8, device="cuda")) & 1).reshape(M, C)
    assert torch.equal(bits.bool(), out.float() > 0)
    dg2, db2, g_sc2 = torch.empty_like(dg), torch.empty_like(db), torch.empty_like(dout)
    dz2 = K.bn_backward(dout, None, y, gamma, st, dg2, db2, g_out=g_sc2, mask=mask)
    assert torch.equal(dz2, dz) and torch.equal(g_sc2, g_sc)
    torch.testing.assert_close(dg2, dg) and torch.testing.assert_close(db2, db)


@pytest.mark.parametrize("C", [96, 4096])
def test_bn_apply_with_residual_bn_affine(C):
    """Projection-shortcut fusion: act(y*s + h + (r*rs + rh)) in one pass against the fp32
    reference and against applying the residual's BN as its own pass first."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(3)
    M = 2000
    y = torch.randn(M, C, device="cuda").bfloat16()
    r = (torch.randn(M, C, device="cuda") * 3 + 1).bfloat16()
    s, h = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    rs, rh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    out = K.bn_apply(y, s, h, residual=r, residual_bn=(rs, rh), relu=True)
    ref = torch.relu(y.float() * s + h + r.float() * rs + rh)
    assert _rel(out, ref) < 1e-2
    unfused = K.bn_apply(y, s, h, residual=K.bn_apply(r, rs, rh), relu=True)
    # the unfused path rounds the normalised residual to bf16 once more: fused is never worse
    assert float((out.float() - ref).abs().max()) <= float((unfused.float() - ref).abs().max()) + 1e-6


@pytest.mark.parametrize("M,C", [(3000, 96), (200000, 40), (50000, 2048), (600000, 256)])
def test_bn_fused_reduce_finalize_matches_unfused(M, C):
    """Slice reduction + finalize (two launches, no atomics) == the memset/atomic-reduce/finalize
    sequence, for fwd and bwd, called repeatedly."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(M + C)
    y = (torch.randn(M, C, device="cuda") * 2 + 1).bfloat16()
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda")
    partial, T = K.bn_stats_partial(y)
    ref = K.BNState(C, "cuda")
    rm0, rv0 = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    K.bn_fwd_finalize(K.bn_reduce_partials(partial, T, C), M, gamma, beta, 1e-5, 0.9, rm0, rv0, ref)
    for _ in range(3):
        st = K.BNState(C, "cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        K.bn_fwd_stats(partial, T, M, gamma, beta, 1e-5, 0.9, rm, rv, st)
        for a, b in ((st.mean, ref.mean), (st.rstd, ref.rstd), (st.scale, ref.scale), (st.shift, ref.shift),
                     (rm, rm0), (rv, rv0)):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    dout = torch.randn(M, C, device="cuda").bfloat16()
    yr = y.float().requires_grad_(True)
    g_r = gamma.clone().requires_grad_(True)
    F.batch_norm(yr, None, None, g_r, None, training=True, eps=1e-5).backward(dout.float())
    dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    dz = K.bn_backward(dout, None, y, gamma, st, dg, db)
    assert _rel(dz, yr.grad) < 2e-2 and _rel(dg, g_r.grad) < 1e-2
    torch.testing.assert_close(db, dout.float().sum(0), rtol=1e-3, atol=1e-2)


def test_maxpool_avgpool():
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(1)
    x = torch.randn(2, 17, 17, 64, device="cuda").bfloat16()
    y, arg = K.maxpool_fwd(x, 3, 2, 1)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.float(), yr.permute(0, 2, 3, 1))
    dy = torch.randn_like(y)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    dx = K.maxpool_bwd(dy, arg, x.shape, 3, 2, 1)
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    p = K.avgpool_fwd(x)
    assert _rel(p, x.float().mean((1, 2))) < 1e-2
    dp = torch.randn(2, 64, device="cuda").bfloat16()
    dxa = K.avgpool_bwd(dp, x.shape)
    assert _rel(dxa, (dp.float() / (17 * 17))[:, None, None, :].expand(x.shape)) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sparse_xent_in_top_k(dtype):
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(2)
    z = torch.randn(37, 1000, device="cuda").to(dtype)
    lab = torch.randint(0, 1000, (37,), device="cuda")
    lab[0] = z[0].float().argmax()
    z[1, 5] = z[1].float().max() + 1
    z[1, 7] = z[1, 5]  # tie on the max: strictly-greater rule -> label 5 is top-1
    lab[1] = 5
    sums, dl, rows, corr = K.sparse_xent(z, lab, want_rows=True)
    zr = z.float().requires_grad_(True)
    loss = F.cross_entropy(zr, lab, reduction="none")
    loss.mean().backward()
    assert _rel(rows, loss) < 1e-3
    assert _rel(dl, zr.grad) < 1e-2
    greater = (z.float() > z.float().gather(1, lab[:, None])).sum(1)
    assert torch.equal(corr.bool(), greater < 1)
    assert abs(float(sums[0]) - float(loss.mean())) < 1e-3
    assert abs(float(sums[1]) - float((greater < 1).float().mean())) < 1e-6
    assert bool(corr[1])


def test_bias_act_dropout():
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(3)
    x = torch.randn(512, 200, device="cuda")
    b = torch.randn(200, device="cuda")
    for act, fn in [(K.ACT_ELU, F.elu), (K.ACT_RELU, F.relu), (K.ACT_GELU, lambda t: F.gelu(t, approximate="tanh"))]:
        y = K.bias_act_dropout(x, b, act)
        assert _rel(y, fn(x + b)) < 1e-5
        xr = x.clone().requires_grad_(True)
        fn(xr + b).backward(torch.ones_like(x))
        dx = K.bias_act_dropout_bwd(torch.ones_like(x), x, b, act)
        assert _rel(dx, xr.grad) < 1e-4
    y = K.bias_act_dropout(torch.ones(1 << 20, 8, device="cuda"), None, K.ACT_NONE, rate=0.25, seed=7, offset=3)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.75) < 0.005
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1 / 0.75))
    g = K.bias_act_dropout_bwd(torch.ones_like(y), torch.ones_like(y), None, K.ACT_NONE, rate=0.25, seed=7, offset=3)
    assert torch.equal(g, y)


def test_fp8_roundtrip():
    from tensorflow_train_distributed_amd.ops import kernels as K
    x = (torch.randn(4096, device="cuda") * 3).bfloat16()
    am = K.amax(x)
    assert abs(float(am) - float(x.float().abs().max())) < 1e-6
    scale = (448.0 / am).float()
    q = K.quant_fp8(x, scale)
    xd = K.dequant_fp8(q, scale)
    assert _rel(xd, x) < 0.05
    ref = (x.float() * scale).to(torch.float8_e4m3fn)
    assert torch.equal(q, ref.view(torch.uint8))


def test_flat_optimizers_match_cpu():
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec, FlatSGD, FlatAdam, FlatLAMB, Schedule
    torch.manual_seed(4)
    specs = [ParamSpec("a/kernel", (300, 70), lambda t, g: t.normal_(generator=g)),
             ParamSpec("a/bias", (70,), lambda t, g: t.normal_(generator=g), weight_decay=False),
             ParamSpec("b/kernel", (40000,), lambda t, g: t.normal_(generator=g))]
    for idx, make in enumerate([lambda p: FlatSGD(p, Schedule(kind=1, base_lr=0.1, decay_steps=2, decay_rate=0.5, staircase=True),
                                   momentum=0.9, weight_decay=0.01),
                 lambda p: FlatSGD(p, Schedule(base_lr=0.05)),
                 lambda p: FlatAdam(p, Schedule(base_lr=1e-3), weight_decay=0.01, max_grad_norm=1.0),
                 lambda p: FlatAdam(p, Schedule(base_lr=1e-3), weight_decay=0.01, decoupled=True),
                 lambda p: FlatLAMB(p, Schedule(kind=2, base_lr=1e-2, warmup_steps=2, total_steps=10),
                                    weight_decay=0.01)]):
        pc = FlatParams(specs, "cpu", compute_dtype=None, seed=5)
        pg = FlatParams(specs, "cuda", seed=5)
        oc, og = make(pc), make(pg)
        valid = torch.zeros(pc.numel, dtype=torch.bool)
        for sp in specs:
            o = pc.offsets[sp.name]
            valid[o:o + int(torch.tensor(sp.shape).prod())] = True
        for it in range(4):
            gr = torch.randn(pc.numel) * valid  # padding between variables never carries gradient
            pc.grad.copy_(gr)
            pg.grad.copy_(gr)
            oc.step()
            og.step()
        d = (pg.master.cpu() - pc.master).abs()
        assert _rel(pg.master.cpu(), pc.master) < 1e-5, (idx, int(d.argmax()), float(d.max()))
        assert _rel(pg.compute.float().cpu(), pc.master) < 1e-2


def test_colsum_and_dgrad_accumulate():
    from tensorflow_train_distributed_amd.ops import kernels as K
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(6)
    x = torch.randn(1000, 100, device="cuda").bfloat16()
    assert _rel(K.colsum(x), x.float().sum(0)) < 1e-4
    # many row slices: vector bf16 path + parallel fold (C % 4 == 0), scalar paths, accumulate
    for rows, C, dt in ((20000, 1024, torch.bfloat16), (5000, 100, torch.float32), (3000, 90, torch.bfloat16),
                        (40000, 3072, torch.bfloat16)):
        x = torch.randn(rows, C, device="cuda").to(dt)
        ref = x.double().sum(0)
        got = K.colsum(x)
        assert float((got.double() - ref).abs().max()) < 1e-3 * float(ref.abs().max()) + 1e-2, (rows, C)
        again = K.colsum(x)
        assert torch.equal(got, again), (rows, C)  # fixed-order folds
        base = torch.randn(C, device="cuda")
        acc = base.clone()
        K.colsum(x, out=acc, beta=1)
        assert float((acc.double() - ref - base.double()).abs().max()) < 1e-3 * float(ref.abs().max()) + 1e-2
    dy = torch.randn(2, 8, 8, 64, device="cuda").bfloat16()
    w = (torch.randn(64, 3, 3, 32, device="cuda") / 24).bfloat16()
    base = torch.randn(2, 8, 8, 32, device="cuda").bfloat16()
    ref = G.conv_dgrad(dy, w.permute(3, 1, 2, 0).contiguous(), (2, 8, 8, 32), (1, 1), (1, 1)).float() + base.float()
    out = base.clone()
    G.conv_dgrad(dy, w.permute(3, 1, 2, 0).contiguous(), (2, 8, 8, 32), (1, 1), (1, 1), out=out, beta=1)
    assert _rel(out, ref) < 1e-2


@pytest.mark.parametrize("shape", [(2, 16, 16, 64), (3, 14, 10, 128)])
def test_sampled_projection_dgrad_then_stride2_beta(shape):
    """The stride-2 1x1 projection dgrad with sampled_only=True leaves the pixels it does not
    sample unwritten (here: NaN garbage); the unit-stride dgrad that accumulates into it with
    beta_s2 reads only the sampled (even h, w) pixels, so the sum equals the zero-filled path."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    torch.manual_seed(7)
    N, H, W, C = shape
    K = 2 * C
    dy_p = torch.randn(N, H // 2, W // 2, K, device="cuda").bfloat16()
    w_p = (torch.randn(K, 1, 1, C, device="cuda") / 16).bfloat16()
    dy_1 = torch.randn(N, H, W, 96, device="cuda").bfloat16()
    w_1 = (torch.randn(96, 1, 1, C, device="cuda") / 10).bfloat16()
    wt_p = w_p.permute(3, 1, 2, 0).contiguous()
    wt_1 = w_1.permute(3, 1, 2, 0).contiguous()
    ref = G.conv_dgrad(dy_p, wt_p, (N, H, W, C), (2, 2), (0, 0))  # zero-filled
    ref = G.conv_dgrad(dy_1, wt_1, (N, H, W, C), out=ref, beta=1).float()
    out = torch.full((N, H, W, C), float("nan"), device="cuda", dtype=torch.bfloat16)
    G.conv_dgrad(dy_p, wt_p, (N, H, W, C), (2, 2), (0, 0), out=out, sampled_only=True)
    assert torch.isnan(out[:, 1::2].float()).all()  # unsampled rows untouched
    G.conv_dgrad(dy_1, wt_1, (N, H, W, C), out=out, beta=1, beta_s2=(H, W))
    assert not torch.isnan(out.float()).any()
    assert torch.equal(out.float(), ref)
    full = F.conv_transpose2d(dy_p.float().permute(0, 3, 1, 2), w_p.float().permute(0, 3, 1, 2), stride=2,
                              output_padding=(H % 2 == 0 and 1 or 0, W % 2 == 0 and 1 or 0))
    full = full + F.conv2d(dy_1.float().permute(0, 3, 1, 2), w_1.float().permute(3, 0, 1, 2))
    assert _rel(out.permute(0, 3, 1, 2), full) < 1e-2


@pytest.mark.parametrize("shape", [(4, 16, 16, 64), (2, 12, 10, 32), (3, 8, 8, 256)])
def test_stem_fused_bn_relu_maxpool_and_backward_stats(shape):
    """Fused BN+ReLU+maxpool (stem) equals bn_apply followed by maxpool_fwd bit for bit; the
    fused pooling backward equals maxpool_bwd * relu mask with exact BN partial sums."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(5)
    N, H, W, C = shape
    y = torch.randn(shape, device="cuda").bfloat16()
    scale = torch.rand(C, device="cuda") + 0.5
    shift = torch.randn(C, device="cuda") * 0.3
    mask_ref = torch.empty(N * H * W * C // 8, dtype=torch.uint8, device="cuda")
    act = K.bn_apply(y.view(-1, C), scale, shift, relu=True, mask=mask_ref).view(shape)
    pooled_ref, arg_ref = K.maxpool_fwd(act, 3, 2, 1)
    assert K.stem_pool_fusable(shape)
    pooled, arg, mask = K.bn_relu_maxpool(y, scale, shift)
    assert torch.equal(pooled, pooled_ref)
    assert torch.equal(arg, arg_ref)
    assert torch.equal(mask, mask_ref)
    dy = torch.randn_like(pooled)
    dx_ref = K.maxpool_bwd(dy, arg_ref, shape, 3, 2, 1).float()
    bits = ((mask_ref[:, None] >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).view(shape).float()
    g_ref = dx_ref * bits
    g, partial, T = K.maxpool_bwd_bnstat(dy, arg, mask, y)
    assert partial.shape[0] == T
    torch.testing.assert_close(g.float(), g_ref, rtol=1e-2, atol=1e-2)
    sums = partial.sum(0)
    gf = g.float().view(-1, C)
    torch.testing.assert_close(sums[0], gf.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sums[1], (gf * y.float().view(-1, C)).sum(0), rtol=1e-4, atol=1e-3)


def test_pad_channels_rgb_fast_path():
    from tensorflow_train_distributed_amd.ops import kernels as K
    x = torch.randn(3, 17, 16, 3, device="cuda").bfloat16()  # rows % 8 == 0 -> vector path
    y = K.pad_channels(x, 8)
    assert torch.equal(y[..., :3], x) and bool((y[..., 3:] == 0).all())
    x2 = torch.randn(3, 5, 3, 3, device="cuda").bfloat16()  # 45 rows -> generic path
    y2 = K.pad_channels(x2, 8)
    assert torch.equal(y2[..., :3], x2) and bool((y2[..., 3:] == 0).all())


def test_bf16_rounding_matches_torch_bitwise():
    """f2bf / pack_bf16x2 / pack8 (common.h: every kernel's fp32 -> bf16 store) against torch's
    round-to-nearest-even conversion, bitwise, on 2^24 random bit patterns (every exponent,
    denormals included) plus the edge classes: exact ties (low half 0x8000) with even and odd
    kept mantissas, one ulp either side of a tie, +-0, +-inf, the largest finite values (which
    round to inf), the smallest denormals, and NaNs (any NaN must stay a NaN)."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    g = torch.Generator().manual_seed(7)
    rnd = torch.randint(-2**31, 2**31 - 1, (1 << 24,), generator=g, dtype=torch.int64)
    hi = torch.randint(0, 1 << 16, (1 << 16,), generator=g, dtype=torch.int64) << 16
    ties = torch.cat([hi | 0x8000, hi | 0x7fff, hi | 0x8001, hi | 0x0001, hi | 0xffff])
    edges = torch.tensor([0x00000000, 0x80000000, 0x7f800000, 0xff800000, 0x7f7fffff, 0xff7fffff, 0x7f7f8000,
                          0x7f7f7fff, 0x00000001, 0x80000001, 0x00008000, 0x00018000, 0x007fffff, 0x00800000,
                          0x7fc00000, 0xffc00000, 0x7f800001, 0x7fbfffff, 0x3f808000, 0x3f818000, 0x3f80ffff,
                          0xbf808000, 0x3f800000, 0x00007fff], dtype=torch.int64)
    bits = torch.cat([rnd & 0xffffffff, ties, edges])
    bits = bits[: bits.numel() // 8 * 8]
    x_cpu = (bits.to(torch.int64) & 0xffffffff).to(torch.int64)
    x_cpu = torch.where(x_cpu >= 2**31, x_cpu - 2**32, x_cpu).to(torch.int32).view(torch.float32)
    ref = x_cpu.to(torch.bfloat16).view(torch.int16)
    one, pair, eight = K.bf16_round_probe(x_cpu.cuda())
    torch.cuda.synchronize()
    isnan = torch.isnan(x_cpu)
    for name, got in (("f2bf", one), ("pack_bf16x2", pair), ("pack8", eight)):
        got = got.cpu()
        bad = (got != ref) & ~isnan
        assert int(bad.sum()) == 0, (name, int(bad.sum()), hex(int(x_cpu.view(torch.int32)[bad][0]) & 0xffffffff),
                                     hex(int(got[bad][0]) & 0xffff), hex(int(ref[bad][0]) & 0xffff))
        gn = got[isnan].to(torch.int32) & 0xffff
        # a NaN stays a NaN (its sign and payload are not specified: torch's CPU conversion returns
        # the canonical 0x7fc0, the hardware conversion a quiet NaN of its own)
        assert bool(((gn & 0x7f80) == 0x7f80).all() and ((gn & 0x007f) != 0).all()), (name, "NaN not kept")
    # the GPU's own torch conversion agrees too (what torch-side reference code computes on device)
    dev_ref = x_cpu.cuda().to(torch.bfloat16).view(torch.int16).cpu()
    assert int(((dev_ref != ref) & ~isnan).sum()) == 0


def test_transpose_batch_matches_torch():
    """Many [A][C] -> [C][A] transposes in one launch (ops.kernels.TransposeBatch, BERT's weight
    copies) bit for bit against torch, and a rebuilt pointer table after a destination moves."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(0)
    shapes = [(3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096), (128, 256)]
    src = [torch.randn(a, c, device="cuda").to(torch.bfloat16) for a, c in shapes]
    dst = [torch.empty(c, a, device="cuda", dtype=torch.bfloat16) for a, c in shapes]
    tb = K.TransposeBatch(list(zip(src, dst)))
    tb.run()
    for s_, d_ in zip(src, dst):
        assert torch.equal(d_, s_.t())
    dst[2] = torch.empty_like(dst[2])
    src[0].mul_(2)
    tb.run(list(zip(src, dst)))
    for s_, d_ in zip(src, dst):
        assert torch.equal(d_, s_.t())
    with pytest.raises(ValueError):
        K.TransposeBatch([(torch.zeros(100, 128, device="cuda", dtype=torch.bfloat16),
                           torch.zeros(128, 100, device="cuda", dtype=torch.bfloat16))])


@pytest.mark.parametrize("A,B,C", [(1024, 1, 4096), (4096, 1, 1024), (3072, 1, 1024), (136, 1, 264), (1000, 1, 24),
                                   (13, 1, 40), (64, 9, 128)])
def test_weight_transpose_matches_torch(A, B, C):
    """[A][B][C] -> [C][B][A] bf16: the 128 x 128 LDS-staged tile kernel (B == 1, multiples of
    128), the 8 x 8 register-block kernel (B == 1, multiples of 8) and the LDS-tile kernel
    (everything else) against torch's permute, bit for bit."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    w = torch.randn(A, 1, B, C, device="cuda").to(torch.bfloat16)
    out = K.krsc_to_crsk(w)
    assert torch.equal(out.view(C, B, A), w.view(A, B, C).permute(2, 1, 0))
