#!/bin/bash
# asm DMA in the mixed-layout GEMMs + LN-backward occupancy: numerics, LN A/B, BERT bench + profile
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gemm_conv.py tests/test_bert.py tests/test_kernels_transformer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/mx_t.log 2>&1; rc=$?; tail -3 gpurun_out/mx_t.log; [ $rc -eq 0 ] || exit 1
for nb in 256 512 1024; do TTD_LN_BWD_BLOCKS=$nb timeout -k 10 100 python tools/ln_bench.py > gpurun_out/mx_ln_$nb.log 2>&1 && echo "nb=$nb $(tail -1 gpurun_out/mx_ln_$nb.log | cut -c1-200)" || exit 1; done
timeout -k 10 240 python bench.py --model bert > gpurun_out/mx_b.log 2>&1 && tail -1 gpurun_out/mx_b.log | cut -c100-190 &&
TTD_LN_BWD_BLOCKS=256 timeout -k 10 240 python bench.py --model bert > gpurun_out/mx_b256.log 2>&1 && tail -1 gpurun_out/mx_b256.log | cut -c100-190 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mx_pb -o run --output-format csv -- python3 bench.py --model bert --steps 3 --warmup 2 > gpurun_out/mx_pb.log 2>&1 && python3 tools/kstats.py gpurun_out/mx_pb/run_kernel_stats.csv "BERT-Large b128 r4 (hipGraph replay)" 6 > gpurun_out/mx_kstats_bert.md && python3 tools/trace_step.py gpurun_out/mx_pb/run_kernel_trace.csv --start embed_fwd --streams > gpurun_out/mx_streams_bert.txt && head -30 gpurun_out/mx_streams_bert.txt
