#!/bin/bash
# stage-3 streamed-filter halo conv: kernel tests, engine tests, A/B in the step
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_CONV3_S3=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_conv3.py > gpurun_out/r4_c3s_t.log 2>&1; rc=$?; tail -12 gpurun_out/r4_c3s_t.log; [ $rc -eq 0 ] || exit 1
TTD_CONV3_S3=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet_engine.py > gpurun_out/r4_c3s_re.log 2>&1; rc=$?; tail -3 gpurun_out/r4_c3s_re.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
TTD_CONV3_S3=0 timeout -k 10 200 python bench.py > gpurun_out/r4_c3a$i.log 2>&1 && tail -1 gpurun_out/r4_c3a$i.log | cut -c1-150 &&
TTD_CONV3_S3=1 timeout -k 10 200 python bench.py > gpurun_out/r4_c3b$i.log 2>&1 && tail -1 gpurun_out/r4_c3b$i.log | cut -c1-150 || exit 1
done
