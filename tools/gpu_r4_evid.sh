#!/bin/bash
# evidence refresh: BERT wgrad PMC, ResNet bf16 / fp8+LAMB kernel stats + per-stream traces, fp8 tracking
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_wgrad.sh 4096 1024 65536 > gpurun_out/ev_pmcw1.txt 2>&1; tail -22 gpurun_out/ev_pmcw1.txt | grep -i "util\|wait\|us \|TF/s" ; 
bash tools/pmc_wgrad.sh 1024 4096 65536 > gpurun_out/ev_pmcw2.txt 2>&1; grep -i "util\|wait_any\|TF/s" gpurun_out/ev_pmcw2.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_pr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/ev_pr.log 2>&1 && python3 tools/kstats.py gpurun_out/ev_pr/run_kernel_stats.csv "ResNet-50 b1024 r4 s2 (hipGraph replay)" 6 > gpurun_out/ev_kstats_resnet.md && python3 tools/trace_step.py gpurun_out/ev_pr/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/ev_streams_resnet.txt && head -3 gpurun_out/ev_streams_resnet.txt || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_pf -o run --output-format csv -- python3 bench.py --precision fp8 --optimizer lamb --steps 3 --warmup 2 > gpurun_out/ev_pf.log 2>&1 && python3 tools/kstats.py gpurun_out/ev_pf/run_kernel_stats.csv "ResNet-50 fp8 + LAMB b1024 r4 s2" 6 > gpurun_out/ev_kstats_fp8.md && python3 tools/trace_step.py gpurun_out/ev_pf/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/ev_streams_fp8.txt && head -3 gpurun_out/ev_streams_fp8.txt || exit 1
timeout -k 10 400 python tools/fp8_tracking.py --steps 200 --out gpurun_out/ev_track.json > gpurun_out/ev_track.log 2>&1 && tail -1 gpurun_out/ev_track.log
