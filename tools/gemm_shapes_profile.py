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
    # streaming pointwise (pw_*), halo 3x3 (c3_*) and stem launches are logged too but dispatch
    # their own kernels, not gemm_kernel / gemm256_kernel: leave them out of the pairing
    log = [e for e in json.load(open(log_json)) if not e[0].startswith(("pw_", "c3_", "stem_"))]
    rows = [r for r in csv.DictReader(open(trace_csv))
            if "gemm_kernel" in r["Kernel_Name"] or "gemm256_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
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


def _bytes(kind, M, N, K):
    """HBM bytes a GEMM must move at least (bf16 operands read once, output written once)."""
    R = int(kind.split("_")[1].split("x")[0]) if "x" in kind.split("_")[1] else 1
    s = int(kind.split("_s")[1][0]) if "_s" in kind else 1
    if kind.startswith("fwd"):
        return 2 * (M * s * s * K // (R * R) + M * N + N * K)
    if kind.startswith("dgrad"):
        return 2 * (M // (s * s) * K // (R * R) + M * N + N * K)
    if kind.startswith("wgrad"):
        return 2 * K * (M + N // (R * R)) + 4 * M * N
    return 2 * (M * K + N * K + M * N)


def report_seq(trace_csv, log_json):
    """Every dispatch of the logged step in launch order (single-stream runs:
    TTD_WGRAD_STREAM=0), GEMMs annotated with their shape, TF/s and HBM-bound floor."""
    import csv
    log = json.load(open(log_json))
    allrows = list(csv.DictReader(open(trace_csv)))
    allrows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gi = [i for i, r in enumerate(allrows) if "gemm_kernel" in r["Kernel_Name"] or "gemm256_kernel" in r["Kernel_Name"]]
    gi = gi[-len(log):]
    first = gi[0]
    # include the non-GEMM dispatches that precede the first GEMM of the step (stem prologue)
    while first > 0 and "pad3to8" not in allrows[first]["Kernel_Name"]:
        first -= 1
    # the launch log and the dispatch order can differ by a swap (a unit's wgrad and dgrad):
    # match each dispatch to the next log entry of the same family (wgrad kernels read both
    # operands M/N-major: MN*/Op*MN/OpWgrad*)
    def fam_k(name):
        return "wgrad" if ("MNDense" in name or "MNConvGather" in name or "OpDenseMN" in name or "OpWgrad" in name) \
            else "other"
    pending = list(log)
    gmap = {}
    for i in gi:
        f = fam_k(allrows[i]["Kernel_Name"])
        j = next((j for j, e in enumerate(pending[:4]) if (e[0].startswith("wgrad") or e[0] == "gemm_tn") == (f == "wgrad")), 0)
        gmap[i] = pending.pop(j)
    tot = floor = 0.0
    cat = {}
    for i in range(first, len(allrows)):
        r = allrows[i]
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = r["Kernel_Name"].replace("void ", "").replace("ttdk::(anonymous namespace)::", "")
        n = n.replace("(anonymous namespace)::", "")
        n = n.split("(")[0] if not n.startswith("big::") else n.split(">(")[0] + ">"
        tot += t
        if i in gmap:
            kind, M, N, K, sp = gmap[i]
            b = _bytes(kind, M, N, K)
            fl = 2.0 * M * N * K
            fb = max(b / 6.0e6, fl / 1.6e9)  # us at 6.0 TB/s or 1.6 PF/s
            floor += fb
            key = kind.split("_")[0]
            c = cat.setdefault(key, [0.0, 0.0])
            c[0] += t
            c[1] += fb
            print("%8.1f us  floor %7.1f  %-22s M=%-8d N=%-5d K=%-8d %6.0f TF/s %5.2f TB/s  %s" % (
                t, fb, kind, M, N, K, fl / t / 1e6, b / t / 1e6, n[:60]))
        else:
            key = n[:40]
            c = cat.setdefault(key, [0.0, 0.0])
            c[0] += t
            print("%8.1f us  %s grid=%s" % (t, n[:90], r.get("Grid_Size_X", r.get("Grid_Size", ""))))
    print("step kernels %.1f us; GEMM floor (6.0 TB/s | 1.6 PF/s) %.1f us" % (tot, floor))
    for k, (t, fb) in sorted(cat.items(), key=lambda kv: -kv[1][0])[:25]:
        print("  %-42s %9.1f us  floor %9.1f" % (k, t, fb))


if __name__ == "__main__":
    if sys.argv[1] == "seq":
        report_seq(sys.argv[2], sys.argv[3])
        sys.exit(0)
    if sys.argv[1] == "run":
        run(int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 256)
    else:
        report(sys.argv[2], sys.argv[3])
