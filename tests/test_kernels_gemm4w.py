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
