#!/bin/bash
# Multi-rank rehearsal on one GPU: bench.py self-launching 2 and 4 ranks that share the GPU, gradient
# all-reduce over gloo (RCCL refuses two ranks on one device); the JSON line carries replicas_in_sync.
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 2 > gpurun_out/mr2.log 2>&1; rc=$?; tail -1 gpurun_out/mr2.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/mr2.log; exit 1; }
TTD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --batch 256 --steps 4 --warmup 2 > gpurun_out/mr4.log 2>&1; rc=$?; tail -1 gpurun_out/mr4.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/mr4.log; exit 1; }
