#!/bin/bash
# persistent GEMM: counted wait at the tile transition — tests, GEMM bench A/B, BERT A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gemm_conv.py tests/test_bert.py -x -q -m gpu --timeout 120 --timeout-method thread -k "persistent or bert or gemm" > gpurun_out/t_pers.log 2>&1; rc=$?; tail -3 gpurun_out/t_pers.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/gemm_bench.py --tokens 65536 --only bert > gpurun_out/gemm_pers1.txt 2>&1 && cat gpurun_out/gemm_pers1.txt &&
TTD_PERS_STORE_WAIT=1 timeout -k 10 300 python tools/gemm_bench.py --tokens 65536 --only bert > gpurun_out/gemm_pers0.txt 2>&1 && cat gpurun_out/gemm_pers0.txt &&
for i in 1 2; do
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_p1_$i.log 2>&1 && tail -1 gpurun_out/bert_p1_$i.log | cut -c1-160 &&
TTD_PERS_STORE_WAIT=1 timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_p0_$i.log 2>&1 && tail -1 gpurun_out/bert_p0_$i.log | cut -c1-160 || exit 1
done
