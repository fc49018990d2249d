"""ResNet-50 GPU engine (hand-written kernels) vs the fp32 PyTorch reference of the same net."""
import pytest
import torch

from tensorflow_train_distributed_amd.models.resnet import ResNet, resnet50


def test_resnet50_reference_cpu_step():
    torch.manual_seed(0)
    m = resnet50(num_classes=10, device="cpu")
    n_trainable = sum(int(torch.tensor(s.shape).prod()) for s in m.params.specs if s.trainable)
    assert n_trainable - 64 * 7 * 7 * 5 == 23528522  # ResNet-50 with a 10-way head (stem padded 3->8 ch)
    x = torch.randn(2, 32, 32, 3)
    y = torch.randint(0, 10, (2,))
    s = m.reference_forward_backward(x, y)
    assert torch.isfinite(s).all()
    g = m.params.grad
    assert float(g.abs().sum()) > 0
    # padded stem input channels get no gradient
    assert float(m.params.g["conv1_conv/kernel"][..., 3:].abs().sum()) == 0.0


@pytest.mark.gpu
def test_resnet50_engine_matches_reference():
    # A shallow ResNet with every block type of ResNet-50 (identity, projection+stride-2,
    # strided 3x3): a deep random-init net amplifies bf16 rounding chaotically (~1.3x per block
    # measured at batch 8), which would test conditioning, not the engine.
    torch.manual_seed(0)
    m = ResNet(((64, 2, 1), (128, 1, 2), (256, 1, 2), (512, 1, 2)), num_classes=100, device="cuda", seed=3)
    x = torch.randn(16, 64, 64, 3, device="cuda").bfloat16()
    y = torch.randint(0, 100, (16,), device="cuda")
    sums = m.forward_backward(x, y)
    g_engine = m.params.grad.clone()
    mm_engine = m.params.var["conv2_block1_1_bn/moving_mean"].clone()
    # reference on the same (bf16-rounded) weights
    leaves = {n: m.params.c[n].float().detach().clone().requires_grad_(m.params.spec(n).trainable)
              for n in m.params.names()}
    loss, acc, _ = m.reference_loss(x.float(), y, leaves, bf16_activations=True)
    loss.backward()
    assert abs(float(sums[0]) - float(loss)) < 0.05 * float(loss)
    names = [n for n in m.params.names() if m.params.spec(n).trainable]
    report = []
    for n in names:
        a = g_engine[m.params.offsets[n]:m.params.offsets[n] + leaves[n].numel()]
        b = leaves[n].grad.flatten()
        report.append((n, float((a - b).norm() / (b.norm() + 1e-20)), float(a.norm()), float(b.norm())))
    bad = [r for r in report if r[1] > 0.15]
    print("\n".join("%-40s rel=%.4f |e|=%.4g |r|=%.4g" % r for r in report[:40]))
    ge = torch.cat([g_engine[m.params.offsets[n]:m.params.offsets[n] + leaves[n].numel()] for n in names])
    gr = torch.cat([leaves[n].grad.flatten() for n in names])
    cos = float(torch.dot(ge, gr) / (ge.norm() * gr.norm()))
    rels = sorted(r[1] for r in report)
    print("cosine %.5f, per-variable rel median %.4f p90 %.4f max %.4f" % (cos, rels[len(rels) // 2], rels[int(0.9 * len(rels))], rels[-1]))
    # (measured 0.966: the bf16 forward drift flips near-zero ReLU masks of this 5-stage net;
    # per-unit numerics are pinned by test_convbn_unit_backward_oracle)
    assert cos > 0.96, (cos, bad[:8])
    # End to end, the bf16 forward drifts ~1-2% from the fp32 oracle by the last stage, so
    # ReLU masks differ on near-zero activations; per-unit exactness is checked by
    # test_convbn_unit_backward_oracle with shared masks. Here: direction + head exactness.
    for n in ["predictions/kernel", "predictions/bias"]:
        a = m.params.g[n].flatten()
        b = leaves[n].grad.flatten()
        rel = float((a - b).norm() / b.norm())
        assert rel < 0.05, (n, rel)
    assert float(mm_engine.abs().sum()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["c1", "c2", "c3", "cd", "stem"])
def test_convbn_unit_backward_oracle(which):
    """Each conv+BN(+ReLU) unit's backward vs an fp32 oracle built from the engine's own saved
    forward tensors (so ReLU masks are identical and only rounding differs)."""
    import torch.nn.functional as F
    from torch.nn.grad import conv2d_input, conv2d_weight
    torch.manual_seed(1)
    m = ResNet(((64, 1, 1), (128, 1, 2)), num_classes=10, device="cuda", seed=2)
    P = m.params
    if which == "stem":
        c = m.stem
        x = torch.randn(4, 32, 32, 8, device="cuda").bfloat16()
        x[..., 3:] = 0
    else:
        c = m.blocks[1][which]
        x = torch.randn(4, 16, 16, c.cin_store, device="cuda").bfloat16()
    relu = which != "cd"
    out, ctx = m._convbn_fwd(c, x, relu)
    dout = torch.randn_like(out)
    m._grad_hook = None
    dx, _ = m._convbn_bwd(c, dout, ctx, need_dx=which != "stem")
    _, y, mask, st = ctx
    g = dout.float() * (out.float() > 0) if relu else dout.float()
    if relu:  # the saved bit mask is exactly [out > 0]
        bits = ((mask[:, None].int() >> torch.arange(8, device="cuda")) & 1).reshape(out.shape)
        assert torch.equal(bits.bool(), out > 0)
    yf = y.float()
    xhat = (yf - st.mean) * st.rstd
    gamma = P.var[c.name + "_bn/gamma"]
    M = yf[..., 0].numel()
    dbeta = g.sum((0, 1, 2))
    dgamma = (g * xhat).sum((0, 1, 2))
    dz = gamma * st.rstd * (g - dbeta / M - xhat * dgamma / M)

    def rel(a, b):
        return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-20))

    assert rel(P.g[c.name + "_bn/beta"], dbeta) < 1e-3
    assert rel(P.g[c.name + "_bn/gamma"], dgamma) < 1e-2
    dzb = dz.to(torch.bfloat16).float().permute(0, 3, 1, 2)
    wf = P.c[c.name + "_conv/kernel"].float().permute(0, 3, 1, 2)
    xf = x.float().permute(0, 3, 1, 2)
    dw = conv2d_weight(xf, wf.shape, dzb, stride=c.stride, padding=c.pad).permute(0, 2, 3, 1)
    assert rel(P.g[c.name + "_conv/kernel"], dw) < 2e-2
    if dx is not None:
        dxr = conv2d_input(xf.shape, wf, dzb, stride=c.stride, padding=c.pad).permute(0, 2, 3, 1)
        assert rel(dx, dxr) < 2e-2


@pytest.mark.gpu
def test_resnet_step_hipgraph_replay_matches_eager():
    """A whole training step (fwd, bwd, in-graph LR schedule, momentum update) captured into a
    hipGraph and replayed must reproduce the eager steps (up to float-atomic summation order in
    the BN-statistics / bias reductions)."""
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    from tensorflow_train_distributed_amd.utils.graphs import capture

    def make():
        m = ResNet(((64, 1, 1), (128, 1, 2)), num_classes=10, device="cuda", seed=5)
        o = FlatSGD(m.params, Schedule(kind=2, base_lr=0.1, warmup_steps=2, end_lr=0.0, power=2.0,
                                       total_steps=100), momentum=0.9, weight_decay=5e-5)
        return m, o

    torch.manual_seed(0)
    x = torch.randn(8, 32, 32, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (8,), device="cuda", dtype=torch.int32)
    m1, o1 = make()
    m2, o2 = make()

    def step(m, o):
        s = m.forward_backward(x, y)
        o.step()
        return s

    eager = [step(m1, o1).clone() for _ in range(4)]
    graph, out = capture(lambda: step(m2, o2), warmup=1)  # warmup = step 1, capture records (no run)
    replays = [graph.replay().clone() for _ in range(3)]  # steps 2..4
    torch.cuda.synchronize()
    for a, b in zip(eager[1:], replays):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-3)
    d = (m1.params.master - m2.params.master).abs().max()
    assert float(d) < 1e-3 * float(m1.params.master.abs().max()), float(d)
    assert int(o1.step_t) == int(o2.step_t) == 4


@pytest.mark.gpu
def test_resnet_step_segmented_capture_matches_eager():
    """The bench's capture: the two-stream step recorded as per-stream linear graph segments
    (event record / wait nodes at every fork and join) and replayed on the eager streams must
    reproduce the eager steps."""
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    from tensorflow_train_distributed_amd.utils import graphs

    def make():
        m = ResNet(((64, 1, 1), (128, 2, 2)), num_classes=10, device="cuda", seed=5)
        o = FlatSGD(m.params, Schedule(kind=2, base_lr=0.1, warmup_steps=2, end_lr=0.0, power=2.0,
                                       total_steps=100), momentum=0.9, weight_decay=5e-5)
        return m, o

    torch.manual_seed(0)
    x = torch.randn(16, 32, 32, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (16,), device="cuda", dtype=torch.int32)
    m1, o1 = make()
    m2, o2 = make()
    assert m2.wgrad_stream and m2.cd_side

    def step(m, o):
        s = m.forward_backward(x, y)
        o.step()
        return s

    eager = [step(m1, o1).clone() for _ in range(5)]
    main = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    seg = graphs.capture_segmented(lambda: step(m2, o2), main=main, warmup=1)  # warmup = step 1
    assert seg.info["streams"] == 2 and seg.info["segments"] >= 4, seg.info
    replays = [seg.replay().clone() for _ in range(4)]  # steps 2..5
    torch.cuda.synchronize()
    for a, b in zip(eager[1:], replays):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-3)
    d = (m1.params.master - m2.params.master).abs().max()
    assert float(d) < 1e-3 * float(m1.params.master.abs().max()), float(d)
    assert int(o1.step_t) == int(o2.step_t) == 5


@pytest.mark.gpu
@pytest.mark.parametrize("fp8_1x1,min_cos", [(False, 0.9), (True, 0.8)])
def test_resnet_fp8_forward_path_tracks_bf16_and_trains_with_lamb(monkeypatch, fp8_1x1, min_cos):
    """precision="fp8": the 3x3 convs with 128-multiple input channels run the fp8 block-scaled
    MFMA forward with delayed activation scaling, and the unit-stride 3x3 data gradients the fp8
    MFMA with e5m2 gradients (delayed scaling; step 1 calibrates both); the step must track the
    bf16 engine and train with LAMB. fp8_1x1 (TTD_FP8_1X1, the default): the 1x1 convs with >= 128
    channels in and out too — forward, data and weight gradients — which puts e5m2 rounding on
    every data gradient of this 16-image, 64..256-channel net (gradient cosine vs bf16 0.85 here;
    at ResNet-50 b1024 the loss tracks bf16 to 0.0 % over 120 LAMB steps,
    profiles/r6_fp8_1x1_ab.txt)."""
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, Schedule
    monkeypatch.setenv("TTD_FP8_1X1", "1" if fp8_1x1 else "0")
    torch.manual_seed(0)
    stages = ((64, 2, 1), (128, 2, 2), (256, 1, 2))
    x = torch.randn(16, 64, 64, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (16,), device="cuda", dtype=torch.int32)
    ref = ResNet(stages, num_classes=10, device="cuda", seed=7)
    f8 = ResNet(stages, num_classes=10, device="cuda", seed=7, precision="fp8")
    assert sum(f8._fp8_conv(c) for c in f8.conv_list()) >= 3
    assert len(f8._g8) >= 1  # a unit-stride 3x3 data gradient on the fp8 MFMA (e5m2 gradients) from step 2
    assert any(c.k == 1 and f8._fp8_conv(c) for c in f8.conv_list()) == fp8_1x1
    assert any(c.k == 1 and c.name in f8._g8 for c in f8.conv_list()) == fp8_1x1
    s_ref = ref.forward_backward(x, y).clone()
    f8.forward_backward(x, y)  # step 1 calibrates the delayed activation scales
    s8 = f8.forward_backward(x, y).clone()
    assert abs(float(s8[0]) - float(s_ref[0])) < 0.05 * float(s_ref[0])
    a, b = f8.params.grad, ref.params.grad
    cos = float(torch.dot(a, b) / (a.norm() * b.norm()))
    assert cos > min_cos, cos
    opt = FlatLAMB(f8.params, Schedule(kind=0, base_lr=0.02), weight_decay=1e-4)
    losses = []
    for _ in range(12):
        losses.append(float(f8.forward_backward(x, y)[0]))
        opt.step()
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.gpu
def test_resnet_fp8_only_input_without_weight_prep():
    """precision="fp8" with the per-step filter preparation off (TTD_WPREP=0 equivalent): the fp8
    data gradient of the unit-stride 3x3 convs is then off, but their forward still stores only
    the fp8 copy of the input (TTD_FP8_ONLY_INPUT), so the backward must take the fp8 weight
    gradient from a freshly quantised dz instead of asking for the unstored bf16 input (ADVICE r4:
    this raised from step 2 on). Several steps run; losses stay finite and track the default."""
    torch.manual_seed(0)
    stages = ((64, 2, 1), (128, 2, 2), (256, 1, 2))
    x = torch.randn(16, 64, 64, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (16,), device="cuda", dtype=torch.int32)
    ref = ResNet(stages, num_classes=10, device="cuda", seed=7, precision="fp8")
    f8 = ResNet(stages, num_classes=10, device="cuda", seed=7, precision="fp8")
    f8.wprep = False
    for _ in range(3):
        lr_ = float(ref.forward_backward(x, y)[0])
        l8 = float(f8.forward_backward(x, y)[0])
        assert l8 == l8 and abs(l8 - lr_) < 0.05 * abs(lr_), (l8, lr_)
    assert f8._x_unstored, "the fp8-only input path was not exercised"
    a, b = f8.params.grad, ref.params.grad
    assert float(torch.dot(a, b) / (a.norm() * b.norm())) > 0.95


@pytest.mark.gpu
@pytest.mark.parametrize("flag,size,batch", [("fuse_pw", 64, 16), ("fuse_c3", 224, 4)])
def test_resnet_streaming_pointwise_fusions_match_unfused_engine(flag, size, batch):
    """The BN-prologue fusions on the streaming pointwise kernel (c2 apply -> c3 conv, c3 apply ->
    next c1 conv, c3 BN backward -> c3 dgrad) evaluate the same per-element expressions as the
    unfused engine; only accumulation order and fma contraction differ. A deep random-init net
    amplifies such rounding chaotically (tools/debug_pw_ab.py: both engines sit at the same
    distance from the fp32 oracle), so this compares both engines with the oracle on the shallow
    net of the test above (stage 2 with two blocks: every fusion site is exercised). fuse_c3: the
    halo 3x3 kernel with c1's BN apply / c2's BN backward as prologue (224-pixel input, so
    stage 2 runs at its 56x56 shape)."""
    torch.manual_seed(0)
    stages = ((64, 2, 1), (128, 1, 2), (256, 1, 2), (512, 1, 2))
    x = torch.randn(batch, size, size, 3, device="cuda").bfloat16()
    y = torch.randint(0, 100, (batch,), device="cuda")
    res = {}
    for fuse in (True, False):
        m = ResNet(stages, num_classes=100, device="cuda", seed=3)
        setattr(m, flag, fuse)
        sums = m.forward_backward(x, y)
        torch.cuda.synchronize()
        g = m.params.grad.clone()
        leaves = {n: m.params.c[n].float().detach().clone().requires_grad_(m.params.spec(n).trainable)
                  for n in m.params.names()}
        loss, _, _ = m.reference_loss(x.float(), y, leaves, bf16_activations=True)
        loss.backward()
        names = [n for n in m.params.names() if m.params.spec(n).trainable]
        a = torch.cat([g[m.params.offsets[n]:m.params.offsets[n] + leaves[n].numel()] for n in names])
        b = torch.cat([leaves[n].grad.flatten() for n in names])
        res[fuse] = (float(sums[0]), float(loss), float(torch.dot(a, b) / (a.norm() * b.norm())), g)
    (lf, rf, cf, gf), (lu, ru, cu, gu) = res[True], res[False]
    assert abs(lf - lu) < 5e-3 * abs(lu), (lf, lu)
    assert cf > 0.95 and cf > cu - 0.01, (cf, cu)
    # engine-vs-engine agreement is bounded by the same bf16 chaos (both are checked against the
    # fp32 oracle above, which is the correctness criterion)
    assert float(torch.dot(gf, gu) / (gf.norm() * gu.norm())) > 0.96


@pytest.mark.gpu
def test_packed_rgb_input_skips_padding_and_matches_padded():
    """At 224 x 224 the dedicated stem kernels read the packed [N,224,224,3] images (no
    channel-padding pass): the step must equal, bitwise, the one fed the 8-channel padded copy."""
    from tensorflow_train_distributed_amd.ops import kernels as K
    torch.manual_seed(0)
    m = ResNet(((64, 1, 1), (128, 1, 2)), num_classes=10, device="cuda", seed=5)
    x = torch.randn(2, 224, 224, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (2,), device="cuda")
    assert m._stem_packed_ok(tuple(x.shape))
    s8 = m.forward_backward(K.pad_channels(x.contiguous(), m.in_store), y).clone()
    g8 = m.params.grad.clone()
    s3 = m.forward_backward(x, y).clone()
    g3 = m.params.grad.clone()
    assert torch.equal(s3, s8)
    assert torch.equal(g3, g8)
    assert float(m.params.g["conv1_conv/kernel"][..., 3:].abs().sum()) == 0.0


@pytest.mark.gpu
def test_gradient_ready_hooks_fire_in_flat_layout_order():
    """The bucketed all-reduce launches every bucket up to the variable a hook names, so the
    engine's hooks must come in flat-layout order even with branches on the side stream (the
    projection backward runs there, concurrent with c3 -> c2)."""
    torch.manual_seed(0)
    m = ResNet(((64, 2, 1), (128, 1, 2)), num_classes=10, device="cuda", seed=5)
    x = torch.randn(4, 32, 32, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (4,), device="cuda")
    names = []
    m.forward_backward(x, y, grad_hook=names.append)
    torch.cuda.synchronize()
    off = [m.params.offsets[n] for n in names]
    assert off == sorted(off), names
    convs = [c.name for c in m.conv_list()]
    assert sorted(n.split("_bn/")[0] for n in names if n.endswith("_bn/moving_variance")) == sorted(convs)
