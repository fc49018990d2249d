#!/bin/bash
# full GPU suite + smoke + default bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/full_t.log 2>&1; rc=$?; tail -3 gpurun_out/full_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 && tail -2 gpurun_out/full_smoke.log &&
timeout -k 10 150 python bench.py > gpurun_out/full_b.log 2>&1 && tail -1 gpurun_out/full_b.log | cut -c1-240
timeout -k 10 240 python bench.py --model bert > gpurun_out/full_bb.log 2>&1 && tail -1 gpurun_out/full_bb.log | cut -c100-200 &&
timeout -k 10 200 python tools/attn_bench.py 128 > gpurun_out/full_attn.txt 2>&1 && tail -3 gpurun_out/full_attn.txt
