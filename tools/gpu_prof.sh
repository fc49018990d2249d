#!/bin/bash
# One profiled bench step set + summaries (replaces the per-experiment gpu_r*_*.sh launchers).
# usage: bash tools/gpu_prof.sh TAG MODEL [extra bench.py args...]   (env vars pass through)
#   MODEL: resnet50 | bert. Writes gpurun_out/TAG/{run_kernel_trace.csv,...},
#   gpurun_out/TAG_kstats.md (per-kernel totals), TAG_streams.txt (per-stream step breakdown),
#   TAG_solo.txt (where the step runs on the main stream alone).
export TMPDIR=/tmp
TAG=$1; MODEL=$2; shift 2
START=stem_fwd; [ "$MODEL" = bert ] && START=embed_fwd
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- \
  python3 bench.py --model $MODEL --steps 3 --warmup 2 "$@" > gpurun_out/$TAG.log 2>&1 || { tail -20 gpurun_out/$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/$TAG/run_kernel_stats.csv "$TAG" 5 > gpurun_out/${TAG}_kstats.md
python3 tools/trace_step.py gpurun_out/$TAG/run_kernel_trace.csv --start $START --streams > gpurun_out/${TAG}_streams.txt
python3 tools/solo_time.py gpurun_out/$TAG/run_kernel_trace.csv --start $START > gpurun_out/${TAG}_solo.txt
tail -1 gpurun_out/$TAG.log | cut -c1-160
head -12 gpurun_out/${TAG}_streams.txt
head -8 gpurun_out/${TAG}_solo.txt
