"""`ttd.nn` / `ttd.layers` / `ttd.initializers` / `ttd.regularizers`: TF naming and
semantics on CPU, and the HIP autograd path vs the fp32 CPU path on the GPU."""
import math

import numpy as np
import pytest
import torch

import tensorflow_train_distributed_amd as ttd
from tensorflow_train_distributed_amd import initializers as I
from tensorflow_train_distributed_amd import layers as L
from tensorflow_train_distributed_amd import nn as N
from tensorflow_train_distributed_amd import regularizers as R


@pytest.fixture(autouse=True)
def fresh():
    ttd.train.reset_default_graph()
    L.reset_naming(0)
    yield


def test_variance_scaling_matches_reference_init():
    g = torch.Generator().manual_seed(0)
    w = I.variance_scaling_initializer()((784, 200), g)
    sigma = math.sqrt(1.3 * 2 / 784)  # 0.0576
    assert abs(sigma - 0.0576) < 1e-3
    assert float(w.abs().max()) <= 2 * sigma + 1e-6
    assert abs(float(w.std()) - sigma * 0.8796) < 0.003
    u = I.GlorotUniform()((100, 50), g)
    assert float(u.abs().max()) <= math.sqrt(6 / 150) + 1e-6


def test_regularizers():
    w = torch.tensor([[1.0, -2.0], [3.0, -4.0]])
    assert float(R.l1_regularizer(0.01)(w)) == pytest.approx(0.1)
    assert float(R.L2(0.5)(w)) == pytest.approx(15.0)


def test_tf_layers_dense_naming_collections_and_unapplied_regularizer():
    x = torch.randn(4, 784)
    h = L.dense(x, 200, activation=N.elu, kernel_initializer=I.variance_scaling_initializer(),
                kernel_regularizer=R.l1_regularizer(0.01), name="hidden1")
    h = L.dense(h, 10, name="output")
    assert h.shape == (4, 10)
    names = [n for n, _ in ttd.train.get_collection("trainable_variables")]
    assert names == ["hidden1/kernel", "hidden1/bias", "output/kernel", "output/bias"]
    regs = ttd.train.get_collection("regularization_losses")
    assert len(regs) == 1  # built (Q1) ...
    k = dict(ttd.train.get_collection("variables"))["hidden1/kernel"]
    assert float(regs[0]) == pytest.approx(0.01 * float(k.abs().sum()), rel=1e-5)
    # auto naming like tf.layers
    a, b = L.Dense(3), L.Dense(3)
    a(torch.randn(2, 5))
    b(torch.randn(2, 5))
    assert [n for n, _ in a.named_variables()] == ["dense/kernel", "dense/bias"]
    assert [n for n, _ in b.named_variables()] == ["dense_1/kernel", "dense_1/bias"]


def _mlp():
    return L.Sequential([
        L.Dense(200, "elu", kernel_initializer=I.variance_scaling_initializer(), name="hidden1"),
        L.Dropout(0.0),
        L.Dense(100, "elu", kernel_initializer=I.variance_scaling_initializer(), name="hidden2"),
        L.Dense(50, "elu", kernel_initializer=I.variance_scaling_initializer(), name="hidden3"),
        L.Dense(25, "elu", kernel_initializer=I.variance_scaling_initializer(), name="hidden4"),
        L.Dense(10, name="output"),
    ])


def test_sequential_mlp_to_flat_trains_with_flat_optimizer():
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    torch.manual_seed(0)
    m = _mlp()
    x = torch.randn(64, 784)
    y = torch.randint(0, 10, (64,))
    m(x)
    fp = m.to_flat("cpu")
    assert fp.numel >= 183685 and sum(int(np.prod(s.shape)) for s in fp.specs) == 183685
    opt = FlatSGD(fp, Schedule(kind=0, base_lr=0.1))
    losses = []
    for _ in range(20):
        fp.zero_grad()
        loss = N.sparse_softmax_cross_entropy_with_logits(labels=y, logits=m(x)).mean()
        loss.backward()
        assert float(fp.g["output/kernel"].abs().sum()) > 0  # grads land in the flat buffer
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.5
    # the module reads the optimizer-updated master weights
    assert m.layer_list[0].kernel.data_ptr() == fp.var["hidden1/kernel"].data_ptr()


def test_conv2d_same_padding_and_attention_cpu():
    x = torch.randn(2, 9, 9, 5)
    k = torch.randn(3, 3, 5, 4)
    y = N.conv2d(x, k, (2, 2), "SAME")
    assert y.shape == (2, 5, 5, 4)
    layer = L.Conv2D(6, 3, strides=1, padding="valid")
    assert layer(x).shape == (2, 7, 7, 6)
    assert [n for n, _ in layer.named_variables()] == ["conv2d/kernel", "conv2d/bias"]
    q = torch.randn(2, 128, 128)
    o = N.attention(q, q, q, num_heads=2, seqlen=torch.tensor([128, 70]))
    assert o.shape == q.shape and torch.isfinite(o).all()
    zt = torch.tensor([[1.0, 2.0, 2.0], [3.0, float("nan"), 0.0]])
    assert N.in_top_k(zt, torch.tensor([1, 1]), 1).tolist() == [True, False]


# ------------------------------------------------------------------ GPU: HIP path vs CPU path
gpu = pytest.mark.gpu


@gpu
@pytest.mark.parametrize("act", [None, "relu", "gelu", "tanh", "elu"])
def test_gpu_dense_matches_cpu(act):
    torch.manual_seed(1)
    # bf16-representable operands: the GPU computes in bf16, so rounding the inputs would
    # move pre-activations across ReLU/ELU kinks and compare masks, not kernels
    x = torch.randn(300, 200).bfloat16().float()
    w = (torch.randn(200, 104) * 0.1).bfloat16().float()
    b = torch.randn(104) * 0.1
    xc, wc, bc = [t.clone().requires_grad_(True) for t in (x, w, b)]
    yc = N.dense(xc, wc, bc, activation=act)
    dy = torch.randn_like(yc)
    yc.backward(dy)
    xg, wg, bg = [t.cuda().requires_grad_(True) for t in (x, w, b)]
    yg = N.dense(xg, wg, bg, activation=act)
    yg.backward(dy.cuda())
    torch.testing.assert_close(yg.cpu(), yc.detach(), atol=5e-2, rtol=5e-2)
    for a, c in ((xg, xc), (wg, wc), (bg, bc)):
        rel = float((a.grad.cpu() - c.grad).norm() / c.grad.norm())
        assert rel < 2e-2, rel


@gpu
def test_gpu_conv_layernorm_dropout_xent_attention():
    torch.manual_seed(2)
    # conv (channel padding 3 -> 8 inside)
    x = torch.randn(2, 16, 16, 3)
    k = torch.randn(3, 3, 3, 16) * 0.2
    xc, kc = x.clone().requires_grad_(True), k.clone().requires_grad_(True)
    yc = N.conv2d(xc, kc, (1, 1), "SAME")
    yc.sum().backward()
    xg, kg = x.cuda().requires_grad_(True), k.cuda().requires_grad_(True)
    yg = N.conv2d(xg, kg, (1, 1), "SAME")
    yg.sum().backward()
    torch.testing.assert_close(yg.cpu(), yc.detach(), atol=5e-2, rtol=5e-2)
    assert float((kg.grad.cpu() - kc.grad).norm() / kc.grad.norm()) < 2e-2
    # layer norm
    h = torch.randn(64, 512)
    g, bb = torch.rand(512) + 0.5, torch.randn(512) * 0.1
    hc = h.clone().requires_grad_(True)
    N.layer_norm(hc, g, bb).pow(2).sum().backward()
    hg = h.cuda().requires_grad_(True)
    N.layer_norm(hg, g.cuda(), bb.cuda()).pow(2).sum().backward()
    assert float((hg.grad.cpu() - hc.grad).norm() / hc.grad.norm()) < 3e-2
    # dropout keeps ~1-rate and scales
    d = N.dropout(torch.ones(1 << 20, device="cuda"), 0.25)
    keep = float((d > 0).float().mean())
    assert abs(keep - 0.75) < 0.005 and abs(float(d.max()) - 1 / 0.75) < 1e-5
    # xent
    z = torch.randn(32, 10)
    lab = torch.randint(0, 10, (32,))
    zc = z.clone().requires_grad_(True)
    N.sparse_softmax_cross_entropy_with_logits(labels=lab, logits=zc).mean().backward()
    zg = z.cuda().requires_grad_(True)
    lg = N.sparse_softmax_cross_entropy_with_logits(labels=lab.cuda().int(), logits=zg)
    lg.mean().backward()
    torch.testing.assert_close(zg.grad.cpu(), zc.grad, atol=1e-5, rtol=1e-3)
    # attention (no dropout)
    q = torch.randn(2, 128, 128)
    qc = q.clone().requires_grad_(True)
    N.attention(qc, qc, qc, 2).sum().backward()
    qg = q.cuda().requires_grad_(True)
    og = N.attention(qg, qg, qg, 2)
    og.sum().backward()
    assert float((qg.grad.cpu() - qc.grad).norm() / qc.grad.norm()) < 3e-2


@gpu
def test_gpu_sequential_training_with_flat_adam():
    from tensorflow_train_distributed_amd.train.flat import FlatAdam, Schedule
    torch.manual_seed(3)
    m = _mlp()
    x = torch.randn(128, 784, device="cuda")
    y = torch.randint(0, 10, (128,), device="cuda", dtype=torch.int32)
    m(x)
    fp = m.to_flat("cuda")
    opt = FlatAdam(fp, Schedule(kind=0, base_lr=1e-3))
    losses = []
    for _ in range(30):
        fp.zero_grad()
        loss = N.sparse_softmax_cross_entropy_with_logits(labels=y, logits=m(x)).mean()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.5, losses


def test_weight_prep_table_layout_cpu():
    """WeightPrep (one launch for every data-gradient filter operand): the sub-pixel phase
    entries follow ops.gemm's phase order and partition the taps, the output views tile the
    buffer without overlap, and tile_begin is the running tile count (checked without a GPU)."""
    import numpy as np
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    src = torch.zeros(10_000_000, dtype=torch.bfloat16)
    wp = K.WeightPrep(src)
    shapes = {"a": (256, 1, 1, 64), "b": (128, 3, 3, 128), "c": (512, 3, 3, 256)}
    off = 0
    for n, s in shapes.items():
        wp.add(n, off, s)
        if s[1] == 3:
            wp.add(n + "/phases", off, s, sub=(2, 1, 1, 28, 28))
        off += int(np.prod(s))
    wp.build()
    rows = wp._tab.numpy().view(K.WeightPrep._DT)
    tiles = 0
    for r in rows:
        assert r["tile_begin"] == tiles
        tiles += r["Tr"] * r["Ts"] * (-(-r["K"] // 32)) * (-(-r["C"] // 32))
    assert tiles == wp._tiles
    for n, s in shapes.items():
        Kc, R, S, C = s
        assert tuple(wp.crsk(n).shape) == (C, R, S, Kc)
        if R == 3:
            ph = wp.phases(n + "/phases")
            assert ph.numel() == C * R * S * Kc  # the phases partition the 9 taps
            want = [(T1, T2) for (T1, _) in G._phases(2, 1, 3, 28) for (T2, _) in G._phases(2, 1, 3, 28)]
            got = [(int(r["Tr"]), int(r["Ts"])) for r in rows if r["s"] == 2 and r["K"] == Kc and r["C"] == C]
            assert got == want
    ends = sorted((v[1], v[1] + (int(np.prod(v[2])) if v[0] == "crsk" else v[2])) for v in wp._views.values())
    for (a0, a1), (b0, b1) in zip(ends, ends[1:]):
        assert a1 <= b0
    assert ends[-1][1] == wp.buf.numel()
