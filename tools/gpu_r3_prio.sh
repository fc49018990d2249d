#!/bin/bash
# persistent GEMM variants at the BERT shapes: MFMA-cluster priority schemes (TTD_PERS_PRIO 0/1/2)
# and the 4-wave 128x128-per-wave kernel (TTD_GEMM4W=1, numerics vs the 8-wave kernel first)
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_GEMM4W=1 timeout -k 10 120 python tools/one_gemm.py 65536 4096 1024 0 1 5 > gpurun_out/g4w_one.txt 2>&1; cat gpurun_out/g4w_one.txt
TTD_GEMM4W=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gemm_conv.py -x -q -m gpu --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/t_g4w.log 2>&1; tail -3 gpurun_out/t_g4w.log
TTD_GEMM4W=1 timeout -k 10 300 python tools/gemm_bench.py --tokens 65536 --only bert > gpurun_out/gemm_g4w.txt 2>&1; echo "gemm4w"; cut -c1-17,60-90 gpurun_out/gemm_g4w.txt | grep bert | head -5
for pr in 0 1 2 0 1 2; do
TTD_PERS_PRIO=$pr timeout -k 10 300 python tools/gemm_bench.py --tokens 65536 --only bert > gpurun_out/gemm_prio$pr.txt 2>&1 || exit 1
echo "prio $pr"; cut -c1-17,60-90 gpurun_out/gemm_prio$pr.txt | grep bert | head -5
done
