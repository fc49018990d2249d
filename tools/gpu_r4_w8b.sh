#!/bin/bash
# fp8 weight gradients + fp8-only stored inputs / dz: engine tests, A/B, 200-step loss tracking
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_engine.py tests/test_kernels_misc.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/w8b_e.log 2>&1; rc=$?; tail -2 gpurun_out/w8b_e.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
TTD_FP8_ONLY_INPUT=0 timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/w8b_0_$i.log 2>&1 && tail -1 gpurun_out/w8b_0_$i.log | cut -c95-175 || exit 1
timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/w8b_1_$i.log 2>&1 && tail -1 gpurun_out/w8b_1_$i.log | cut -c95-175 || exit 1
done
timeout -k 10 200 python bench.py --optimizer lamb > gpurun_out/w8b_bf.log 2>&1 && tail -1 gpurun_out/w8b_bf.log | cut -c95-175 &&
timeout -k 10 400 python tools/fp8_tracking.py --steps 200 --out gpurun_out/w8b_track.json > gpurun_out/w8b_track.log 2>&1 && tail -1 gpurun_out/w8b_track.log
