#!/bin/bash
# re-check binary ResNet knobs after the DMA / WGS changes (one box, interleaved with the default)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { timeout -k 10 150 env $1 python bench.py > gpurun_out/kn.log 2>&1 && bash tools/bench_val.sh "$1" gpurun_out/kn.log; }
for r in 1 2; do
run TTD_X=0 || exit 1
run TTD_BIG_PP=0 || exit 1
run TTD_WGRAD_GATHER_X3=0 || exit 1
run TTD_MAIN_PRIO=0 || exit 1
run TTD_PW_FOLD_SIDE=0 || exit 1
done
