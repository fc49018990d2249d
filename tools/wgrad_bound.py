#!/usr/bin/env python3
"""Diagnostic only (never a benchmark number): the ResNet-50 bench step with side-stream weight-
gradient GEMMs (ops.gemm.conv_wgrad) replaced by no-ops, to bound how much of the step the side
stream's CU occupancy costs the main-stream chain. Same arguments as bench.py.

TTD_WGRAD_SKIP selects which weight gradients are skipped (default all):
  all | c3small (3x3, Cout < 256) | c3big (3x3, Cout >= 256) | p1 (1x1 stride 1) | p2 (1x1 stride 2)
(comma-separated). Per class, the wall-time difference prices that class's side-stream cost.

    TTD_WGRAD_SKIP=c3small python tools/wgrad_bound.py --steps 20 --warmup 5
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

_real = G.conv_wgrad
_skip = set(os.environ.get("TTD_WGRAD_SKIP", "all").split(","))


def _cls(wshape, stride):
    K, R, S, C = wshape
    if R == 3:
        return "c3big" if K >= 256 else "c3small"
    return "p2" if tuple(stride) != (1, 1) else "p1"


def _wgrad(x, dz, wshape, stride, pad, **kw):
    if "all" in _skip or _cls(wshape, stride) in _skip:
        return None
    return _real(x, dz, wshape, stride, pad, **kw)


G.conv_wgrad = _wgrad
import bench  # noqa: E402

if __name__ == "__main__":
    sys.exit(bench.main())
