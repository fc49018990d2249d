#!/bin/bash
# BERT weight-gradient workgroup target sweep
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for w in ${WGS_LIST:-128 160 192 256}; do
TTD_BERT_WGRAD_WGS=$w timeout -k 10 200 python bench.py --model bert > gpurun_out/bwgs_${w}_$r.log 2>&1 && echo "wgs=$w $(tail -1 gpurun_out/bwgs_${w}_$r.log | cut -c100-128)" || exit 1
done; done
