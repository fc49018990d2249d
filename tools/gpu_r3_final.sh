#!/bin/bash
# End-of-session check: full GPU suite, smoke, ResNet bench x2, BERT bench, fp8+LAMB bench, ResNet kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_final.log 2>&1; rc=$?; tail -3 gpurun_out/t_final.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 && tail -1 gpurun_out/smoke_final.log &&
timeout -k 10 200 python bench.py > gpurun_out/b_final1.log 2>&1 && tail -1 gpurun_out/b_final1.log | cut -c1-170 &&
timeout -k 10 200 python bench.py > gpurun_out/b_final2.log 2>&1 && tail -1 gpurun_out/b_final2.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bb_final.log 2>&1 && tail -1 gpurun_out/bb_final.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/b8_final.log 2>&1 && tail -1 gpurun_out/b8_final.log | cut -c1-170 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/p_final -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/p_final.log 2>&1 && python3 tools/kstats.py gpurun_out/p_final/run_kernel_stats.csv "ResNet-50 b1024 r3 session-2 final" 6 > gpurun_out/kstats_final.md && python3 tools/trace_step.py gpurun_out/p_final/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/streams_final.txt && head -12 gpurun_out/streams_final.txt
