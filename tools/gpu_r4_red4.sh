#!/bin/bash
# vectorised BN slice reduction + LAMB: tests, ResNet A/B (TTD_BN_REDUCE4), BERT LAMB kernel times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_misc.py tests/test_bert.py -m gpu > gpurun_out/red4_tests.log 2>&1 || { tail -30 gpurun_out/red4_tests.log; exit 1; }
tail -2 gpurun_out/red4_tests.log
for r in 1 2; do for f in 1 0; do
TTD_BN_REDUCE4=$f timeout -k 10 150 python bench.py > gpurun_out/red4_$f.log 2>&1 && bash tools/bench_val.sh "resnet reduce4=$f" gpurun_out/red4_$f.log || exit 1
done; done
timeout -k 10 200 python bench.py --model bert > gpurun_out/red4_bert.log 2>&1 && bash tools/bench_val.sh "bert" gpurun_out/red4_bert.log || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/red4_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model bert --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/red4_prof.log 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/red4_prof -name '*kernel_stats.csv' | head -1); grep -E 'lamb|reduce_slices|finalize_kernel' "$f" | cut -c1-160
