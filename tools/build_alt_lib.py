#!/usr/bin/env python3
"""Build an alternate libttd_hip.so with extra hipcc flags on chosen sources, for A/B runs
through TTD_HIP_LIB_OVERRIDE (the in-tree library is left alone).

    python tools/build_alt_lib.py --out tensorflow_train_distributed_amd/lib/alt/libttd_hip_noslp.so \\
        --flags=-fno-slp-vectorize --files attention conv_dgrad conv_fwd conv_wgrad gemm_conv pw_gemm
"""
import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--flags", default="", help="extra hipcc flags (space separated)")
    ap.add_argument("--files", nargs="*", default=None, help="source stems that get the flags (default: all)")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    from tensorflow_train_distributed_amd import _native
    srcs = _native.hip_sources()
    objdir = os.path.join(os.path.dirname(os.path.abspath(a.out)), "obj_" + os.path.basename(a.out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=" + _native.HIP_ARCH, "-O3", "-std=c++17", "-fPIC",
            "-fvisibility=hidden", "-munsafe-fp-atomics", "-Wno-unused-result"]
    extra = a.flags.split()

    def build(src):
        stem = os.path.basename(src)[:-4]
        obj = os.path.join(objdir, stem + ".o")
        cmd = base + (extra if a.files is None or stem in a.files else []) + ["-c", src, "-o", obj]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if p.returncode:
            raise RuntimeError(" ".join(cmd) + "\n" + p.stdout)
        return obj

    with ThreadPoolExecutor(a.jobs) as ex:
        objs = list(ex.map(build, srcs))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=" + _native.HIP_ARCH, "-shared", "-fPIC", "-o", a.out,
                    *objs, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    print("built", a.out)


if __name__ == "__main__":
    main()
