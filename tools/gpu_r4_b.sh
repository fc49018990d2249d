#!/bin/bash
# no-SLP A/B (ResNet x2, BERT), fp8 loss tracking (200 steps), full GPU suite
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=$PWD/tensorflow_train_distributed_amd/lib/alt/libttd_hip_noslp.so
for i in 1 2; do
timeout -k 10 200 python bench.py > gpurun_out/r4_sa$i.log 2>&1 && tail -1 gpurun_out/r4_sa$i.log | cut -c1-150 &&
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 200 python bench.py > gpurun_out/r4_sb$i.log 2>&1 && tail -1 gpurun_out/r4_sb$i.log | cut -c1-150 || exit 1
done
timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_sba.log 2>&1 && tail -1 gpurun_out/r4_sba.log | cut -c1-150 &&
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_sbb.log 2>&1 && tail -1 gpurun_out/r4_sbb.log | cut -c1-150 || exit 1
timeout -k 10 300 python tools/fp8_tracking.py --steps 200 --out gpurun_out/r4_fp8_tracking.json > gpurun_out/r4_fp8t.log 2>&1; tail -2 gpurun_out/r4_fp8t.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4_tall.log 2>&1; rc=$?; tail -5 gpurun_out/r4_tall.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1; tail -1 gpurun_out/r4_smoke.log
