#!/bin/bash
# End of session 3: full GPU suite, smoke, ResNet x2, BERT x2, fp8+LAMB, BERT + ResNet kernel-trace profiles
export TMPDIR=/tmp
mkdir -p gpurun_out/f3
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/f3/t.log 2>&1; rc=$?; tail -2 gpurun_out/f3/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f3/smoke.log 2>&1 && tail -1 gpurun_out/f3/smoke.log &&
timeout -k 10 200 python bench.py > gpurun_out/f3/b1.log 2>&1 && tail -1 gpurun_out/f3/b1.log | cut -c1-170 &&
timeout -k 10 200 python bench.py > gpurun_out/f3/b2.log 2>&1 && tail -1 gpurun_out/f3/b2.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/f3/bb1.log 2>&1 && tail -1 gpurun_out/f3/bb1.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/f3/bb2.log 2>&1 && tail -1 gpurun_out/f3/bb2.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/f3/b8.log 2>&1 && tail -1 gpurun_out/f3/b8.log | cut -c1-170 &&
timeout -k 10 120 python tools/attn_bench.py 128 > gpurun_out/f3/attn.txt 2>&1 && grep -v amdgpu gpurun_out/f3/attn.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f3/bert -o run --output-format csv -- python3 bench.py --model bert --steps 3 --warmup 2 > gpurun_out/f3/pbert.log 2>&1 &&
python3 tools/kstats.py gpurun_out/f3/bert/run_kernel_stats.csv "BERT-Large b128 r3 session 3" 6 > gpurun_out/f3/kstats_bert.md &&
python3 tools/trace_step.py gpurun_out/f3/bert/run_kernel_trace.csv --start embed_fwd_kernel --streams > gpurun_out/f3/streams_bert.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f3/rn -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/f3/prn.log 2>&1 &&
python3 tools/kstats.py gpurun_out/f3/rn/run_kernel_stats.csv "ResNet-50 b1024 r3 session 3" 6 > gpurun_out/f3/kstats_rn.md &&
python3 tools/trace_step.py gpurun_out/f3/rn/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/f3/streams_rn.txt &&
rm -f gpurun_out/f3/*/run_kernel_trace.csv && head -24 gpurun_out/f3/kstats_bert.md && grep "^stream" gpurun_out/f3/streams_bert.txt gpurun_out/f3/streams_rn.txt
