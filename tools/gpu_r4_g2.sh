#!/bin/bash
# hipGraph defaults: ResNet default (graph), BERT eager vs graph A/B, MLP default
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/r4_d1.log 2>&1 && tail -1 gpurun_out/r4_d1.log | cut -c1-700 &&
timeout -k 10 120 python bench.py --model mlp > gpurun_out/r4_mlp.log 2>&1; tail -2 gpurun_out/r4_mlp.log | cut -c1-400
for i in 1 2; do
timeout -k 10 240 python bench.py --model bert --graph 0 > gpurun_out/r4_bge$i.log 2>&1 && tail -1 gpurun_out/r4_bge$i.log | cut -c1-160 &&
timeout -k 10 240 python bench.py --model bert --graph 1 > gpurun_out/r4_bgg$i.log 2>&1 && tail -1 gpurun_out/r4_bgg$i.log | cut -c1-160 || exit 1
done
