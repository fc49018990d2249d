#!/bin/bash
# HBM bytes per ResNet-50 step: FETCH_SIZE and WRITE_SIZE passes (separate runs: TCC counter budget)
# + a kernel-trace run for per-kernel time / achieved TB/s. usage: bash tools/pmc_bytes.sh <tag> [extra bench args]
# (TTD_WGRAD_STREAM=0 in the environment: one stream, so each kernel's time is its own)
tag=${1:-cur}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/pmc_${tag}_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_${tag}_$c.log; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/pmc_${tag}_trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/pmc_${tag}_trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/pmc_bytes.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE gpurun_out/pmc_${tag}_trace > gpurun_out/pmc_bytes_$tag.txt
head -60 gpurun_out/pmc_bytes_$tag.txt
