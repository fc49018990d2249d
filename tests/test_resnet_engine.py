"""ResNet-50 GPU engine (hand-written kernels) vs the fp32 PyTorch reference of the same net."""
import pytest
import torch

from tensorflow_train_distributed_amd.models.resnet import resnet50


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
    torch.manual_seed(0)
    m = resnet50(num_classes=100, device="cuda", seed=3)
    x = torch.randn(8, 64, 64, 3, device="cuda").bfloat16()
    y = torch.randint(0, 100, (8,), device="cuda")
    sums = m.forward_backward(x, y)
    g_engine = m.params.grad.clone()
    mm_engine = m.params.var["conv2_block1_1_bn/moving_mean"].clone()
    # reference on the same (bf16-rounded) weights
    leaves = {n: m.params.c[n].float().detach().clone().requires_grad_(m.params.spec(n).trainable)
              for n in m.params.names()}
    loss, acc, _ = m.reference_loss(x.float(), y, leaves)
    loss.backward()
    assert abs(float(sums[0]) - float(loss)) < 0.05 * float(loss)
    names = [n for n in m.params.names() if m.params.spec(n).trainable]
    ge = torch.cat([g_engine[m.params.offsets[n]:m.params.offsets[n] + leaves[n].numel()] for n in names])
    gr = torch.cat([leaves[n].grad.flatten() for n in names])
    cos = float(torch.dot(ge, gr) / (ge.norm() * gr.norm()))
    assert cos > 0.98, cos
    for n in ["predictions/kernel", "conv5_block3_3_conv/kernel", "conv2_block1_1_conv/kernel", "conv1_conv/kernel"]:
        a = m.params.g[n].flatten()
        b = leaves[n].grad.flatten()
        rel = float((a - b).norm() / b.norm())
        assert rel < 0.15, (n, rel)
    assert float(mm_engine.abs().sum()) > 0
