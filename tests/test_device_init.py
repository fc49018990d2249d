"""Device-side Philox initialisation (csrc/kernels/init.hip): distribution moments, the +-2
sigma truncation, determinism in (seed, offset), and FlatParams(device_init=True) for the
ResNet engine (reference: tf.truncated_normal_initializer is a device op,
/root/reference/distribute_training.py:49)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_init_random_distributions():
    from tensorflow_train_distributed_amd.ops import kernels as K
    n = 1 << 22
    t = torch.empty(n, device="cuda")
    K.init_random_(t, K.INIT_TRUNCATED, 0.5, 2.0, seed=7, offset=3)
    x = t.cpu().double()
    assert float(x.min()) >= 0.5 - 4.0 - 1e-5 and float(x.max()) <= 0.5 + 4.0 + 1e-5
    # variance of a +-2 sigma truncated standard normal: 0.7737
    assert abs(float(x.mean()) - 0.5) < 0.01
    assert abs(float(x.std()) - 2.0 * math.sqrt(0.7737413)) < 0.01
    again = torch.empty(n, device="cuda")
    K.init_random_(again, K.INIT_TRUNCATED, 0.5, 2.0, seed=7, offset=3)
    assert torch.equal(t, again)
    K.init_random_(again, K.INIT_TRUNCATED, 0.5, 2.0, seed=7, offset=4)
    assert not torch.equal(t, again)
    K.init_random_(t, K.INIT_NORMAL, 0.0, 1.0, seed=1)
    x = t.cpu().double()
    assert abs(float(x.mean())) < 0.01 and abs(float(x.std()) - 1.0) < 0.01 and float(x.abs().max()) > 4.0
    K.init_random_(t, K.INIT_UNIFORM, -1.0, 3.0, seed=2)
    x = t.cpu().double()
    assert float(x.min()) >= -1.0 and float(x.max()) < 3.0 and abs(float(x.mean()) - 1.0) < 0.01
    K.init_random_(t, K.INIT_CONSTANT, 0.25)
    assert bool((t == 0.25).all())


def test_resnet_params_initialised_on_device():
    from tensorflow_train_distributed_amd.models.resnet import ResNet
    m = ResNet(((64, 1, 1), (128, 1, 2), (256, 1, 2), (512, 1, 2)), num_classes=10, device="cuda", seed=3)
    P = m.params
    w = P.var["conv2_block1_2_conv/kernel"]
    std = math.sqrt(2.0 / (9 * 64)) / 0.87962566103423978
    assert float(w.abs().max()) <= 2 * std + 1e-6
    assert abs(float(w.float().std()) - std * math.sqrt(0.7737413)) < 0.05 * std
    assert bool((P.var["conv2_block1_2_bn/gamma"] == 1).all()) and bool((P.var["conv2_block1_2_bn/beta"] == 0).all())
    m2 = ResNet(((64, 1, 1), (128, 1, 2), (256, 1, 2), (512, 1, 2)), num_classes=10, device="cuda", seed=3)
    assert torch.equal(m2.params.master, P.master)
