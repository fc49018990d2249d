#!/bin/bash
# attention dK/dV + fused backward: dropout hash halves picked by one v_perm_b32 per element
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_transformer.py tests/test_bert.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_ap.log 2>&1; rc=$?; tail -2 gpurun_out/t_ap.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/attn_bench.py 128 > gpurun_out/attn_ap.txt 2>&1 && grep -v amdgpu gpurun_out/attn_ap.txt &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_ap1.log 2>&1 && tail -1 gpurun_out/bert_ap1.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_ap2.log 2>&1 && tail -1 gpurun_out/bert_ap2.log | cut -c1-170
