#!/bin/bash
# kernel-trace profiles: BERT-Large b128 (per-stream step breakdown) and ResNet-50 fp8 + LAMB
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/bert -o run --output-format csv -- python3 bench.py --model bert --steps 3 --warmup 2 > gpurun_out/prof2/bert.log 2>&1 || { tail -5 gpurun_out/prof2/bert.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof2/bert/run_kernel_stats.csv "BERT-Large b128 r3 session 2" 6 > gpurun_out/prof2/kstats_bert.md
python3 tools/trace_step.py gpurun_out/prof2/bert/run_kernel_trace.csv --start embed_fwd_kernel --streams > gpurun_out/prof2/streams_bert.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/fp8 -o run --output-format csv -- python3 bench.py --precision fp8 --optimizer lamb --steps 3 --warmup 2 > gpurun_out/prof2/fp8.log 2>&1 || { tail -5 gpurun_out/prof2/fp8.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof2/fp8/run_kernel_stats.csv "ResNet-50 b1024 fp8 + LAMB r3 session 2" 6 > gpurun_out/prof2/kstats_fp8.md
python3 tools/trace_step.py gpurun_out/prof2/fp8/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/prof2/streams_fp8.txt
rm -f gpurun_out/prof2/*/run_kernel_trace.csv
head -20 gpurun_out/prof2/kstats_bert.md; head -5 gpurun_out/prof2/streams_bert.txt; grep "^stream" gpurun_out/prof2/streams_bert.txt; head -16 gpurun_out/prof2/kstats_fp8.md
