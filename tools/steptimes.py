import sys, time, torch
sys.path.insert(0, '.')
import bench
from types import SimpleNamespace
args = SimpleNamespace(batch=512, precision=sys.argv[1], optimizer='momentum', bucket_mb=32.0, image_size=224)
dev = torch.device('cuda', 0)
step, B, info = bench.build_resnet(args, dev, 0, 1)
ts = []
for i in range(12):
    torch.cuda.synchronize(); t0 = time.perf_counter(); s = step(); torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
print(sys.argv[1], ['%.1f' % t for t in ts], 'loss %.3f' % float(s[0]), flush=True)
