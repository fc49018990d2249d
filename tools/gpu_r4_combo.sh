#!/bin/bash
# fp8 wgrad for strided 3x3 convs: engine tests + fp8 A/B, then the ResNet knob re-check
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cb_e.log 2>&1; rc=$?; tail -2 gpurun_out/cb_e.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
TTD_FP8_WGRAD=0 timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/cb_0.log 2>&1 && echo "fp8 wgrad off $(tail -1 gpurun_out/cb_0.log | cut -c100-135)" || exit 1
timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/cb_1.log 2>&1 && echo "fp8 wgrad on  $(tail -1 gpurun_out/cb_1.log | cut -c100-135)" || exit 1
done
timeout -k 10 200 python bench.py --optimizer lamb > gpurun_out/cb_bl.log 2>&1 && echo "bf16 lamb $(tail -1 gpurun_out/cb_bl.log | cut -c100-135)" || exit 1
bash tools/gpu_r4_knobs.sh
