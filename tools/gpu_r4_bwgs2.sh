#!/bin/bash
# BERT weight-gradient workgroup target with the hipBLASLt plain GEMMs on the main stream
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for w in 192 160 224; do
TTD_BERT_WGRAD_WGS=$w timeout -k 10 200 python bench.py --model bert > gpurun_out/bw.log 2>&1 && bash tools/bench_val.sh "wgs=$w" gpurun_out/bw.log || exit 1
done; done
