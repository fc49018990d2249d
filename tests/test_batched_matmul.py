"""Batched MatMul (tf.matmul on rank > 2 operands): ttd.nn.matmul runs ONE strided-batched GEMM
launch per product (ops.gemm.gemm_batched, batch index on the grid's z), forward and backward,
checked against a PyTorch fp32 torch.matmul oracle. Reference op: the dense MatMul of
/root/reference/distribute_training.py:54,61 generalised to batched operands (BASELINE.json:5)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


SHAPES = [((8, 512, 64), (8, 64, 512)), ((16, 512, 512), (16, 512, 64)), ((3, 2, 37, 40), (3, 2, 40, 29))]


@pytest.mark.parametrize("sa,sb", SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_batched_matmul_forward_backward_vs_fp32(sa, sb, dtype):
    import tensorflow_train_distributed_amd as ttd
    torch.manual_seed(0)
    a = torch.randn(sa, device="cuda").to(dtype).requires_grad_(True)
    b = torch.randn(sb, device="cuda").to(dtype).requires_grad_(True)
    y = ttd.nn.matmul(a, b)
    a32 = a.detach().float().requires_grad_(True)
    b32 = b.detach().float().requires_grad_(True)
    r = torch.matmul(a32, b32)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert y.shape == r.shape and _rel(y, r) < tol
    g = torch.randn_like(r)
    y.backward(g.to(y.dtype))
    r.backward(g.to(y.dtype).float())
    assert _rel(a.grad, a32.grad) < tol * 2 and _rel(b.grad, b32.grad) < tol * 2


def test_batched_matmul_is_one_launch_per_product():
    import tensorflow_train_distributed_amd as ttd
    from torch.profiler import ProfilerActivity, profile
    a = torch.randn(16, 512, 512, device="cuda").bfloat16().requires_grad_(True)
    b = torch.randn(16, 512, 64, device="cuda").bfloat16().requires_grad_(True)
    ttd.nn.matmul(a, b).float().sum().backward()  # warm-up (library load)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        y = ttd.nn.matmul(a, b)
        y.float().sum().backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA" and "gemm" in e.name]
    # forward + dA + dB: three GEMM kernels, not 3 x 16
    assert len(names) == 3, names
