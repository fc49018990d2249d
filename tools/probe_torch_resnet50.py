"""Probe: time a plain-PyTorch (MIOpen/hipBLASLt) ResNet-50 bf16 training step on one MI355X.

Used only as an external yardstick for our own HIP kernels (not part of the framework path).
"""
import time, json, sys
import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, mid, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, mid, 1, bias=False); self.b1 = nn.BatchNorm2d(mid)
        self.c2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False); self.b2 = nn.BatchNorm2d(mid)
        self.c3 = nn.Conv2d(mid, cout, 1, bias=False); self.b3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        sc = x if self.down is None else self.down(x)
        return F.relu(y + sc)


class ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False); self.bn1 = nn.BatchNorm2d(64)
        layers = []
        cin = 64
        for mid, n, s in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
            for i in range(n):
                layers.append(Bottleneck(cin, mid, mid * 4, s if i == 0 else 1)); cin = mid * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, 1000)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.max_pool2d(x, 3, 2, 1)
        x = self.layers(x)
        x = x.mean((2, 3))
        return self.fc(x)


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda")
    m = ResNet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(bs, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (bs,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    n = 20
    t0 = time.time()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / n
    print(json.dumps({"probe": "torch_resnet50_bf16_autocast_channels_last", "bs": bs,
                      "ms_per_step": dt * 1e3, "img_per_s": bs / dt}), flush=True)


if __name__ == "__main__":
    main()
