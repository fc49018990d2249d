"""Run one ResNet-50 training step with the GEMM launch log on, then match the launch log
against a rocprofv3 kernel trace (gemm_kernel dispatches in order) to report per-layer
time, achieved TFLOP/s and the HBM-bound floor. Usage (on the GPU box):

  TTD_GEMM_LOG=1 rocprofv3 --kernel-trace -d gpurun_out/p -o run --output-format csv -- \
      python3 tools/gemm_shapes_profile.py run --batch 256
  python3 tools/gemm_shapes_profile.py report gpurun_out/p/run_kernel_trace.csv gpurun_out/gemm_log.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(batch):
    import torch
    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.ops import gemm as G
    dev = torch.device("cuda")
    m = resnet50(device=dev)
    x = torch.randn(batch, 224, 224, 3, device=dev).bfloat16()
    y = torch.randint(0, 1000, (batch,), device=dev)
    for _ in range(2):
        m.forward_backward(x, y)
    torch.cuda.synchronize()
    G.gemm_log(reset=True)
    m.forward_backward(x, y)
    torch.cuda.synchronize()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(G.gemm_log(), open("gpurun_out/gemm_log.json", "w"))


def report(trace_csv, log_json):
    import csv
    log = json.load(open(log_json))
    rows = [r for r in csv.DictReader(open(trace_csv))
            if "gemm_kernel" in r["Kernel_Name"] or "gemm256_kernel" in r["Kernel_Name"]]
    # the last len(log) gemm dispatches belong to the logged step
    rows = rows[-len(log):]
    agg = {}
    tot = 0.0
    for (kind, M, N, K, splits), r in zip(log, rows):
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += t
        fl = 2.0 * M * N * K
        kn = r["Kernel_Name"]
        kern = ("big" + kn.split("gemm256_kernel<")[1].split(",")[0]) if "gemm256" in kn else \
            ("4w" + kn.split("gemm_kernel<")[1].split(",")[0] + "x" + kn.split("gemm_kernel<")[1].split(",")[1].strip())
        key = (kind, M, N, K, kern)
        a = agg.setdefault(key, [0, 0.0, fl])
        a[0] += 1
        a[1] += t
    print("total gemm us %.1f" % tot)
    print("%-16s %8s %6s %6s %5s %9s %8s %8s" % ("kind", "M", "N", "K", "n", "us(each)", "TF/s", "kernel"))
    for (kind, M, N, K, kern), (n, t, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-16s %8d %6d %6d %5d %9.1f %8.1f %8s" % (kind, M, N, K, n, t / n, fl / (t / n) / 1e6, kern))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 256)
    else:
        report(sys.argv[2], sys.argv[3])
