#!/bin/bash
# HBM bytes per ResNet-50 step: FETCH_SIZE and WRITE_SIZE passes (separate runs: TCC counter budget)
# usage: bash tools/pmc_bytes.sh <tag> [extra bench args]
tag=${1:-cur}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/pmc_${tag}_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_${tag}_$c.log; exit 1; }
done
python3 tools/pmc_bytes.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE > gpurun_out/pmc_bytes_$tag.txt
head -60 gpurun_out/pmc_bytes_$tag.txt
