#!/bin/bash
# stage-3 halo kernel tests + A/B, no-SLP A/B, fp8 loss tracking
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_CONV3_S3=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_conv3.py > gpurun_out/r4_c3s_t.log 2>&1; rc=$?; tail -4 gpurun_out/r4_c3s_t.log; [ $rc -eq 0 ] || exit 1
TTD_CONV3_S3=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet_engine.py > gpurun_out/r4_c3s_re.log 2>&1; rc=$?; tail -2 gpurun_out/r4_c3s_re.log; [ $rc -eq 0 ] || exit 1
ALT=$PWD/tensorflow_train_distributed_amd/lib/alt/libttd_hip_noslp.so
for i in 1 2; do
TTD_CONV3_S3=0 timeout -k 10 200 python bench.py > gpurun_out/r4_c3a$i.log 2>&1 && tail -1 gpurun_out/r4_c3a$i.log | cut -c1-120 &&
TTD_CONV3_S3=1 timeout -k 10 200 python bench.py > gpurun_out/r4_c3b$i.log 2>&1 && tail -1 gpurun_out/r4_c3b$i.log | cut -c1-120 &&
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 200 python bench.py > gpurun_out/r4_sb$i.log 2>&1 && tail -1 gpurun_out/r4_sb$i.log | cut -c1-120 || exit 1
done
timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_sba.log 2>&1 && tail -1 gpurun_out/r4_sba.log | cut -c1-120 &&
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_sbb.log 2>&1 && tail -1 gpurun_out/r4_sbb.log | cut -c1-120 || exit 1
timeout -k 10 300 python tools/fp8_tracking.py --steps 200 --out gpurun_out/r4_fp8_tracking.json > gpurun_out/r4_fp8t.log 2>&1; tail -1 gpurun_out/r4_fp8t.log
