#!/bin/bash
# short end-of-session check: GPU suite, smoke, ResNet and BERT benches
export TMPDIR=/tmp
mkdir -p gpurun_out/c3
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c3/t.log 2>&1; rc=$?; tail -2 gpurun_out/c3/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c3/smoke.log 2>&1 && tail -1 gpurun_out/c3/smoke.log &&
timeout -k 10 200 python bench.py > gpurun_out/c3/b.log 2>&1 && tail -1 gpurun_out/c3/b.log | cut -c1-170 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/c3/bb.log 2>&1 && tail -1 gpurun_out/c3/bb.log | cut -c1-170
