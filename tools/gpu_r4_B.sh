#!/bin/bash
# full GPU suite + smoke + ResNet / BERT / fp8 profiles
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4_tall.log 2>&1; rc=$?; tail -3 gpurun_out/r4_tall.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1; tail -1 gpurun_out/r4_smoke.log
bash tools/gpu_r4_prof.sh
