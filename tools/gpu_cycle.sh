#!/bin/bash
# One GPU iteration: tests, bench, per-GEMM-shape profile. Usage: bash tools/gpu_cycle.sh [tag]
tag=${1:-cur}
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/t_$tag.log 2>&1
echo "pytest_rc=$?"; tail -3 gpurun_out/t_$tag.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || { echo bench_failed; tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
TTD_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 tools/gemm_shapes_profile.py run --batch 256 > gpurun_out/prof_$tag.log 2>&1 || { echo prof_failed; exit 1; }
python3 tools/gemm_shapes_profile.py report gpurun_out/prof_$tag/run_kernel_trace.csv gpurun_out/gemm_log.json > gpurun_out/gemm_report_$tag.txt
head -25 gpurun_out/gemm_report_$tag.txt
python3 - "$tag" <<'PY'
import csv, sys
tag = sys.argv[1]
rows = list(csv.DictReader(open('gpurun_out/prof_%s/run_kernel_stats.csv' % tag)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('kernel total ms (3 steps): %.2f' % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%7.2f ms %5.1f%% n=%4s %s' % (float(r['TotalDurationNs']) / 1e6, 100 * float(r['TotalDurationNs']) / tot, r['Calls'], r['Name'][:90]))
PY
