#!/bin/bash
# LayerNorm backward with one-iteration-ahead row prefetch: numerics, standalone A/B, BERT A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_transformer.py tests/test_bert.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lnpf_t.log 2>&1; rc=$?; tail -2 gpurun_out/lnpf_t.log; [ $rc -eq 0 ] || exit 1
for p in 0 1 0 1; do TTD_LN_BWD_PREFETCH=$p timeout -k 10 100 python tools/ln_bench.py > gpurun_out/lnpf.log 2>&1 && echo "pf=$p $(tail -1 gpurun_out/lnpf.log | cut -c1-190)" || exit 1; done
for r in 1 2; do for p in 0 1; do
TTD_LN_BWD_PREFETCH=$p timeout -k 10 200 python bench.py --model bert > gpurun_out/lnpf_b.log 2>&1 && bash tools/bench_val.sh "pf=$p" gpurun_out/lnpf_b.log || exit 1
done; done
