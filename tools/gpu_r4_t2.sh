#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_engine.py tests/test_kernels_misc.py tests/test_kernels_gemm_conv.py -k "bf16_rounding or rccl or segmented or bucket or watchdog or probe or version or persistent or fused_bias_rowsum or splitk or layouts" > gpurun_out/r4_t2.log 2>&1; rc=$?; tail -30 gpurun_out/r4_t2.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/graph_prio_probe2.py > gpurun_out/r4_gprio.log 2>&1; tail -6 gpurun_out/r4_gprio.log
timeout -k 10 200 python bench.py --graph 1 > gpurun_out/r4_bg1.log 2>&1 && tail -1 gpurun_out/r4_bg1.log | cut -c1-300 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/r4_bb1.log 2>&1 && tail -1 gpurun_out/r4_bb1.log | cut -c1-250 &&
TTD_BERT_BIAS_WGRAD=0 timeout -k 10 200 python bench.py --model bert > gpurun_out/r4_bb0.log 2>&1 && tail -1 gpurun_out/r4_bb0.log | cut -c1-250
