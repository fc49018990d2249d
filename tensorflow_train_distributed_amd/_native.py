"""Build and load the framework's native libraries.

Two shared objects are built IN-TREE under ``tensorflow_train_distributed_amd/lib``:

* ``libttd_rt.so``  - host runtime (C++17, g++): crc32c, TFRecord/Event IO, TensorBundle V2
  checkpoint IO, the parameter-server transport/variable store/accumulators/token queue and
  the prefetching batch loader. Exported through a flat C ABI (``ttd_*``).
* ``libttd_hip.so`` - the hand-written CDNA4 (gfx950) HIP kernels: MFMA GEMM / implicit-GEMM
  convolution, BatchNorm/LayerNorm, softmax/cross-entropy, pooling, embedding, fused
  optimizers, fp8 casts, attention. Also a flat C ABI (``ttdk_*``); every launcher takes an
  explicit ``hipStream_t`` so PyTorch's current stream (and hipGraph capture) is honoured.

Both are loaded with :mod:`ctypes`; nothing here depends on Python or PyTorch headers, so a
clean build takes seconds (rt) to about a minute (hip, parallel per-file compile).
"""
from __future__ import annotations

import ctypes
import fcntl
import glob
import hashlib
import os
import shutil
import subprocess
import threading
from concurrent.futures import ThreadPoolExecutor

_PKG = os.path.dirname(os.path.abspath(__file__))
_CSRC = os.path.join(_PKG, "csrc")
_LIBDIR = os.path.join(_PKG, "lib")
_OBJDIR = os.path.join(_LIBDIR, "obj")

RT_LIB = os.path.join(_LIBDIR, "libttd_rt.so")
# kernel-side headers the host runtime also compiles (the collective engine's call plan)
_RT_SHARED = [os.path.join(_CSRC, "kernels", "collective_plan.h")]
HIP_LIB = os.path.join(_LIBDIR, "libttd_hip.so")

HIP_ARCH = os.environ.get("TTD_HIP_ARCH", "gfx950")

_lock = threading.Lock()
_rt = None
_hip = None


class NativeBuildError(RuntimeError):
    pass


def _newest_mtime(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _run(cmd):
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise NativeBuildError("command failed: %s\n%s" % (" ".join(cmd), p.stdout))
    return p.stdout


def _jobs():
    try:
        n = int(os.environ.get("MAX_JOBS", "0"))
    except ValueError:
        n = 0
    return max(1, min(n or (os.cpu_count() or 4), 16))


def _build_objects(srcs, headers, compile_cmd, ext):
    os.makedirs(_OBJDIR, exist_ok=True)
    hdr_m = _newest_mtime(headers)
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(_OBJDIR, os.path.basename(s) + ext)
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_m):
            todo.append((s, o))
    if todo:
        with ThreadPoolExecutor(_jobs()) as ex:
            list(ex.map(lambda so: _run(compile_cmd(*so)), todo))
    return objs, bool(todo)


def build_rt(force: bool = False) -> str:
    """Compile libttd_rt.so with g++ (host only)."""
    srcs = sorted(glob.glob(os.path.join(_CSRC, "runtime", "*.cc")))
    hdrs = glob.glob(os.path.join(_CSRC, "runtime", "*.h")) + _RT_SHARED
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-fvisibility=hidden"]
    san = os.environ.get("TTD_RT_SANITIZE")  # e.g. "thread" or "address" (host-only builds)
    if san:
        flags += ["-fsanitize=" + san, "-g", "-O1"]
    if force:
        shutil.rmtree(_OBJDIR, ignore_errors=True)
    objs, changed = _build_objects(
        srcs, hdrs, lambda s, o: [cxx, *flags, "-c", s, "-o", o], ".rt.o")
    if changed or not os.path.exists(RT_LIB) or os.path.getmtime(RT_LIB) < _newest_mtime(objs):
        _run([cxx, *flags, "-shared", "-o", RT_LIB, *objs])
    return RT_LIB


def hip_sources():
    return sorted(glob.glob(os.path.join(_CSRC, "kernels", "*.hip")))


# Per-file extra flags. attention.hip: no SLP vectorisation — -O3 packs adjacent f32 multiplies /
# FMAs of the softmax into v_pk_*_f32, which beside MFMAs cost more issue cycles than the scalar
# pair (cdna_hip_programming.md, attention prefill pitfalls).
_FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"]}


def build_hip(force: bool = False) -> str:
    """Cross-compile every HIP kernel for gfx950 into libttd_hip.so (no GPU needed)."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    srcs = hip_sources()
    hdrs = glob.glob(os.path.join(_CSRC, "kernels", "*.h"))
    flags = ["--offload-arch=" + HIP_ARCH, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
             "-munsafe-fp-atomics", "-Wno-unused-result"]
    if force:
        shutil.rmtree(_OBJDIR, ignore_errors=True)
    objs, changed = _build_objects(
        srcs, hdrs, lambda s, o: [hipcc, *flags, *_FILE_FLAGS.get(os.path.basename(s), []), "-c", s, "-o", o],
        ".hip.o")
    if changed or not os.path.exists(HIP_LIB) or os.path.getmtime(HIP_LIB) < _newest_mtime(objs):
        # librccl.so.1: the native collective engine (collective.hip). At run time the soname
        # resolves to the RCCL torch already loaded, so the process holds one RCCL.
        _run([hipcc, "--offload-arch=" + HIP_ARCH, "-shared", "-fPIC", "-o", HIP_LIB, *objs,
              "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    return HIP_LIB


def _src_hash(kind):
    pats = {"rt": ("runtime", "*.cc", "*.h"), "hip": ("kernels", "*.hip", "*.h")}[kind]
    h = hashlib.sha1()
    files = []
    for pat in pats[1:]:
        files += sorted(glob.glob(os.path.join(_CSRC, pats[0], pat)))
    if kind == "rt":
        files += _RT_SHARED
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(HIP_ARCH.encode())
    if kind == "hip":
        h.update(repr(sorted(_FILE_FLAGS.items())).encode())
    return h.hexdigest()


def _ensure(kind, lib, builder, force=False):
    """Build `lib` unless its stamp matches the current source hash (mtime-independent, so
    a snapshot copied to another machine does not rebuild). Serialised across processes."""
    os.makedirs(_LIBDIR, exist_ok=True)
    stamp = lib + ".stamp"
    want = _src_hash(kind)
    with open(os.path.join(_LIBDIR, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            have = open(stamp).read().strip() if os.path.exists(stamp) else ""
            if force or have != want or not os.path.exists(lib):
                builder(force)
                with open(stamp, "w") as fh:
                    fh.write(want)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return lib


def build(force: bool = False):
    _ensure("rt", RT_LIB, build_rt, force)
    _ensure("hip", HIP_LIB, build_hip, force)


def rt() -> ctypes.CDLL:
    """The host runtime library (built on first use if missing or stale)."""
    global _rt
    if _rt is None:
        with _lock:
            if _rt is None:
                _ensure("rt", RT_LIB, build_rt)
                lib = ctypes.CDLL(RT_LIB)
                lib.ttd_last_error.restype = ctypes.c_char_p
                _rt = lib
    return _rt


def hip() -> ctypes.CDLL:
    """The gfx950 kernel library. Raises loudly if it cannot be built or loaded."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                alt = os.environ.get("TTD_HIP_LIB_OVERRIDE")  # A/B runs against another build
                if alt:
                    _hip = ctypes.CDLL(alt)
                else:
                    _ensure("hip", HIP_LIB, build_hip)
                    _hip = ctypes.CDLL(HIP_LIB)
    return _hip


def rt_error() -> str:
    return rt().ttd_last_error().decode("utf-8", "replace")
