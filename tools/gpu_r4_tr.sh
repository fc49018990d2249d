#!/bin/bash
# 2-D weight transpose kernel: numerics + BERT-Large bench and per-stream profile
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_misc.py -x -q -m gpu --timeout 120 --timeout-method thread -k transpose > gpurun_out/tr_t.log 2>&1; rc=$?; tail -3 gpurun_out/tr_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python bench.py --model bert > gpurun_out/tr_b.log 2>&1 && tail -1 gpurun_out/tr_b.log | cut -c1-160 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_pb -o run --output-format csv -- python3 bench.py --model bert --steps 3 --warmup 2 > gpurun_out/tr_pb.log 2>&1 && python3 tools/kstats.py gpurun_out/tr_pb/run_kernel_stats.csv "BERT-Large b128 r4 (hipGraph replay)" 6 > gpurun_out/tr_kstats_bert.md && python3 tools/trace_step.py gpurun_out/tr_pb/run_kernel_trace.csv --start embed_fwd --streams > gpurun_out/tr_streams_bert.txt && head -30 gpurun_out/tr_streams_bert.txt
