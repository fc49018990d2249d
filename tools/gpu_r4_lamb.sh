#!/bin/bash
# LAMB phase kernel times inside the BERT-Large step (rocprofv3 kernel stats)
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/lamb_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model bert --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/lamb_prof.log 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/lamb_prof -name '*kernel_stats.csv' | head -1); grep -E 'lamb|sumsq' "$f" | cut -c1-160
tail -1 $GRAFT_REPO_ROOT/gpurun_out/lamb_prof.log | cut -c1-200
