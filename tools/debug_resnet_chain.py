"""Chained forward: engine vs bf16-faithful fp32 reference, error growth per block (debug aid)."""
import torch
import torch.nn.functional as F
from tensorflow_train_distributed_amd.models.resnet import resnet50
from tensorflow_train_distributed_amd.ops import kernels as K

torch.manual_seed(0)
m = resnet50(num_classes=100, device="cuda", seed=3)
P = m.params
x = torch.randn(8, 64, 64, 3, device="cuda").bfloat16()

def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-20))

def rnd(t):
    return t.to(torch.bfloat16).float()

def ref_convbn(c, t, relu, res=None):
    w = P.c[c.name + "_conv/kernel"].float()[..., :t.shape[1]].permute(0, 3, 1, 2)
    y = rnd(F.conv2d(t, w, stride=c.stride, padding=c.pad))
    y = F.batch_norm(y, None, None, P.var[c.name + "_bn/gamma"], P.var[c.name + "_bn/beta"], training=True, eps=1e-5)
    if res is not None:
        y = y + res
    return rnd(F.relu(y) if relu else y)

xin = K.pad_channels(x, 8)
o, _ = m._convbn_fwd(m.stem, xin, True)
r = ref_convbn(m.stem, x.float().permute(0, 3, 1, 2), True)
print("stem", rel(o, r.permute(0, 2, 3, 1)))
h, _ = K.maxpool_fwd(o, 3, 2, 1)
hr = F.max_pool2d(r, 3, 2, 1)
print("pool", rel(h, hr.permute(0, 2, 3, 1)), "std", float(hr.std()))
for i, blk in enumerate(m.blocks):
    o1, _ = m._convbn_fwd(blk["c1"], h, True)
    o2, _ = m._convbn_fwd(blk["c2"], o1, True)
    sc = m._convbn_fwd(blk["cd"], h, False)[0] if blk["cd"] is not None else h
    h, _ = m._convbn_fwd(blk["c3"], o2, True, residual=sc)
    r1 = ref_convbn(blk["c1"], hr, True)
    r2 = ref_convbn(blk["c2"], r1, True)
    rs = ref_convbn(blk["cd"], hr, False) if blk["cd"] is not None else hr
    hr = ref_convbn(blk["c3"], r2, True, rs)
    print("block %2d err %.4f std %.3f" % (i, rel(h, hr.permute(0, 2, 3, 1)), float(hr.std())))
