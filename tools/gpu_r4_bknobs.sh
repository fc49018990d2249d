#!/bin/bash
# BERT-Large knob re-check after the LN-backward prefetch / tile queue (2 interleaved rounds, one box)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
for cfg in "192 256" "160 256" "256 256" "192 512"; do
set -- $cfg
TTD_BERT_WGRAD_WGS=$1 TTD_LN_BWD_BLOCKS=$2 timeout -k 10 200 python bench.py --model bert > gpurun_out/bk.log 2>&1 && bash tools/bench_val.sh "wgs=$1 ln=$2" gpurun_out/bk.log || exit 1
done; done
