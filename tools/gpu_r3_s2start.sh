#!/bin/bash
# Re-entry check: GPU suite, smoke, ResNet bench, ResNet kernel stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_s2.log 2>&1 && tail -2 gpurun_out/t_s2.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s2.log 2>&1 && tail -2 gpurun_out/smoke_s2.log &&
timeout -k 10 200 python bench.py > gpurun_out/b_s2.log 2>&1 && tail -1 gpurun_out/b_s2.log &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/p_s2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/p_s2.log 2>&1 && python3 tools/kstats.py gpurun_out/p_s2/run_kernel_stats.csv "ResNet-50 b1024 r3 s2" 6 > gpurun_out/kstats_s2.md && head -40 gpurun_out/kstats_s2.md
