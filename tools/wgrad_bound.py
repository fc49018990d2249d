#!/usr/bin/env python3
"""Diagnostic only (never a benchmark number): the ResNet-50 bench step with the side-stream
weight-gradient GEMMs (ops.gemm.conv_wgrad) replaced by no-ops, to bound how much of the step
the side stream's CU occupancy costs the main-stream chain. Same arguments as bench.py.

    python tools/wgrad_bound.py --steps 20 --warmup 5
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

G.conv_wgrad = lambda *a, **k: None
import bench  # noqa: E402

if __name__ == "__main__":
    sys.exit(bench.main())
