#!/bin/bash
# two-rank rehearsal on one GPU (gloo) of the BERT bench's N>1 path
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --model bert --gpus 2 --steps 3 --warmup 2 --batch 16 > gpurun_out/n2b.log 2>&1; rc=$?
grep -v "^\s*$" gpurun_out/n2b.log | tail -3 | cut -c1-300; exit $rc
