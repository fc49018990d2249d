#!/bin/bash
# pw fused-wgrad slab fold on the side stream: kernel tests + ResNet A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_pw.py tests/test_resnet_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fo_t.log 2>&1; rc=$?; tail -3 gpurun_out/fo_t.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
TTD_PW_FOLD_SIDE=0 timeout -k 10 150 python bench.py > gpurun_out/fo_0_$i.log 2>&1 && tail -1 gpurun_out/fo_0_$i.log | cut -c100-175 || exit 1
TTD_PW_FOLD_SIDE=1 timeout -k 10 150 python bench.py > gpurun_out/fo_1_$i.log 2>&1 && tail -1 gpurun_out/fo_1_$i.log | cut -c100-175 || exit 1
done
