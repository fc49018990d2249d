#!/bin/bash
# diagnostic: what the split-K fold passes cost the ResNet-50 / BERT steps (TTD_DIAG_SKIP_FOLD=1 skips them: wrong gradients)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for f in 0 1; do
TTD_DIAG_SKIP_FOLD=$f timeout -k 10 150 python bench.py > gpurun_out/df_$f.log 2>&1 && bash tools/bench_val.sh "resnet skip=$f" gpurun_out/df_$f.log || exit 1
done; done
for f in 0 1; do
TTD_DIAG_SKIP_FOLD=$f timeout -k 10 200 python bench.py --model bert > gpurun_out/dfb_$f.log 2>&1 && bash tools/bench_val.sh "bert skip=$f" gpurun_out/dfb_$f.log || exit 1
done
