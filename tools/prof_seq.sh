#!/bin/bash
# Single-stream per-dispatch profile of one ResNet-50 step in launch order (GEMMs annotated with
# shape, TF/s, HBM floor). Usage: bash tools/prof_seq.sh <tag> [batch]
tag=${1:-seq}; B=${2:-1024}
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_WGRAD_STREAM=0 TTD_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pseq_$tag -o run --output-format csv -- python3 tools/gemm_shapes_profile.py run --batch $B > gpurun_out/pseq_$tag.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/pseq_$tag.log; exit 1; }
python3 tools/gemm_shapes_profile.py seq gpurun_out/pseq_$tag/run_kernel_trace.csv gpurun_out/gemm_log.json > gpurun_out/seq_$tag.txt
tail -30 gpurun_out/seq_$tag.txt
