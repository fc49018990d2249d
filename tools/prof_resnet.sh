#!/bin/bash
# Per-layer GEMM + kernel-stats profile of one ResNet-50 step. Usage: bash tools/prof_resnet.sh <tag> [batch]
tag=${1:-cur}; B=${2:-512}
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 tools/gemm_shapes_profile.py run --batch $B > gpurun_out/prof_$tag.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/prof_$tag.log; exit 1; }
python3 tools/gemm_shapes_profile.py report gpurun_out/prof_$tag/run_kernel_trace.csv gpurun_out/gemm_log.json > gpurun_out/gemm_report_$tag.txt
head -70 gpurun_out/gemm_report_$tag.txt
python3 tools/kstats.py gpurun_out/prof_$tag/run_kernel_stats.csv "ResNet-50 b$B $tag" 3 > gpurun_out/kstats_$tag.md
