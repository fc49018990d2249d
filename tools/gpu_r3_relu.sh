#!/bin/bash
# ReLU as one v_maximum3_f32 (no canonicalising v_max before it) in every GEMM / BN / pool epilogue
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_relu.log 2>&1; rc=$?; tail -2 gpurun_out/t_relu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py > gpurun_out/b_relu1.log 2>&1 && tail -1 gpurun_out/b_relu1.log | cut -c1-170 &&
timeout -k 10 200 python bench.py > gpurun_out/b_relu2.log 2>&1 && tail -1 gpurun_out/b_relu2.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_relu.log 2>&1 && tail -1 gpurun_out/bert_relu.log | cut -c1-170
