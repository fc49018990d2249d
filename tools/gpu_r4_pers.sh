#!/bin/bash
# BERT: persistent (static tile partition) vs one-tile-per-workgroup main-stream GEMMs in the two-stream step
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for p in 1 0; do
TTD_BIG_PERS=$p timeout -k 10 200 python bench.py --model bert > gpurun_out/pers.log 2>&1 && bash tools/bench_val.sh "pers=$p" gpurun_out/pers.log || exit 1
done; done
