#!/bin/bash
# fp8 weight gradients in the ResNet fp8 + LAMB step: engine tests, A/B, short loss tracking
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/w8_e.log 2>&1; rc=$?; tail -2 gpurun_out/w8_e.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
TTD_FP8_WGRAD=0 timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/w8_0_$i.log 2>&1 && tail -1 gpurun_out/w8_0_$i.log | cut -c95-175 || exit 1
TTD_FP8_WGRAD=1 timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/w8_1_$i.log 2>&1 && tail -1 gpurun_out/w8_1_$i.log | cut -c95-175 || exit 1
done
timeout -k 10 200 python bench.py --optimizer lamb > gpurun_out/w8_bf.log 2>&1 && tail -1 gpurun_out/w8_bf.log | cut -c95-175
