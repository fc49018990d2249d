#!/bin/bash
# BERT-Large b128 kernel stats + per-stream step trace (current code)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/evb -o run --output-format csv -- python3 bench.py --model bert --steps 3 --warmup 2 > gpurun_out/evb.log 2>&1 && python3 tools/kstats.py gpurun_out/evb/run_kernel_stats.csv "BERT-Large b128 r4 s3 (hipGraph replay)" 6 > gpurun_out/evb_kstats.md && python3 tools/trace_step.py gpurun_out/evb/run_kernel_trace.csv --start embed_fwd --streams > gpurun_out/evb_streams.txt && head -3 gpurun_out/evb_streams.txt || exit 1
rm -f gpurun_out/evb/run_kernel_trace.csv
