#!/bin/bash
# wgrad+bias kernel (uniform turn counter): test, BERT A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gemm_conv.py -k "fused_bias_rowsum" > gpurun_out/r4_C_t.log 2>&1; rc=$?; tail -2 gpurun_out/r4_C_t.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
TTD_BERT_BIAS_WGRAD=0 timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_Cb0$i.log 2>&1 && tail -1 gpurun_out/r4_Cb0$i.log | cut -c1-120 &&
timeout -k 10 240 python bench.py --model bert > gpurun_out/r4_Cb1$i.log 2>&1 && tail -1 gpurun_out/r4_Cb1$i.log | cut -c1-120 || exit 1
done
timeout -k 10 200 python bench.py > gpurun_out/r4_Cr.log 2>&1 && tail -1 gpurun_out/r4_Cr.log | cut -c1-120
