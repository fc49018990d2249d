#!/bin/bash
# fp8 + LAMB vs bf16 + LAMB on one box (end of session)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/f8e.log 2>&1 && bash tools/bench_val.sh "fp8+lamb" gpurun_out/f8e.log || exit 1
timeout -k 10 200 python bench.py --optimizer lamb > gpurun_out/bfe.log 2>&1 && bash tools/bench_val.sh "bf16+lamb" gpurun_out/bfe.log || exit 1
done
