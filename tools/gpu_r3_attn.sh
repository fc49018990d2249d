#!/bin/bash
# fused attention backward: tests, standalone bench, BERT A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_transformer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1; rc=$?; tail -15 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/attn_bench.py 32 > gpurun_out/attn_b32.txt 2>&1 && cat gpurun_out/attn_b32.txt &&
timeout -k 10 120 python tools/attn_bench.py 128 > gpurun_out/attn_b128.txt 2>&1 && cat gpurun_out/attn_b128.txt &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_f1.log 2>&1 && tail -1 gpurun_out/bert_f1.log | cut -c1-200 &&
TTD_ATTN_FUSED_BWD=0 timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_f0.log 2>&1 && tail -1 gpurun_out/bert_f0.log | cut -c1-200
