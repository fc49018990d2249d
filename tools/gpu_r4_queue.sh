#!/bin/bash
# persistent GEMM with a per-XCD tile queue: numerics + BERT A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gemm_conv.py tests/test_bert.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_t.log 2>&1; rc=$?; tail -2 gpurun_out/q_t.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do for q in 0 1; do
TTD_PERS_QUEUE=$q timeout -k 10 200 python bench.py --model bert > gpurun_out/q.log 2>&1 && bash tools/bench_val.sh "queue=$q" gpurun_out/q.log || exit 1
done; done
