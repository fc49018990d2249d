#!/bin/bash
# attention VALU trims (one cvt_pk per bf16 pair, permlane row reductions, DPP lane swap, scalar
# tile-row offsets) + forward occupancy A/B (TTD_ATTN_FWD_OCC=2/4): full GPU suite (the bf16 pair
# pack is shared by every kernel), standalone attention, BERT and ResNet benches
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_av.log 2>&1; rc=$?; tail -3 gpurun_out/t_av.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/attn_bench.py 128 > gpurun_out/attn_av2.txt 2>&1 && grep -v amdgpu gpurun_out/attn_av2.txt &&
TTD_ATTN_FWD_OCC=4 timeout -k 10 120 python tools/attn_bench.py 128 > gpurun_out/attn_av4.txt 2>&1 && grep -v amdgpu gpurun_out/attn_av4.txt &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_av2.log 2>&1 && tail -1 gpurun_out/bert_av2.log | cut -c1-170 &&
TTD_ATTN_FWD_OCC=4 timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_av4.log 2>&1 && tail -1 gpurun_out/bert_av4.log | cut -c1-170 &&
timeout -k 10 200 python bench.py > gpurun_out/b_av.log 2>&1 && tail -1 gpurun_out/b_av.log | cut -c1-170
