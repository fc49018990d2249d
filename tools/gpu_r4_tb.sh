#!/bin/bash
# 4-wave weight-gradient split target sweep (ResNet-50 b1024 bf16)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for t in 256 512 1024; do
TTD_WGRAD_TARGET_BLOCKS=$t timeout -k 10 150 python bench.py > gpurun_out/tb.log 2>&1 && bash tools/bench_val.sh "tb=$t" gpurun_out/tb.log || exit 1
done; done
