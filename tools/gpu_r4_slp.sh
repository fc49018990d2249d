#!/bin/bash
# A/B: the in-tree build vs the MFMA-bearing sources built with -fno-slp-vectorize
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=$PWD/tensorflow_train_distributed_amd/lib/alt/libttd_hip_noslp.so
for i in 1 2; do
timeout -k 10 200 python bench.py > gpurun_out/r4_sa$i.log 2>&1 && tail -1 gpurun_out/r4_sa$i.log | cut -c1-150 &&
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 200 python bench.py > gpurun_out/r4_sb$i.log 2>&1 && tail -1 gpurun_out/r4_sb$i.log | cut -c1-150 || exit 1
done
timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_sba.log 2>&1 && tail -1 gpurun_out/r4_sba.log | cut -c1-150 &&
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_sbb.log 2>&1 && tail -1 gpurun_out/r4_sbb.log | cut -c1-150
