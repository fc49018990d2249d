#!/bin/bash
# ResNet engine tests; A/B the late forward-projection join
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_lj.log 2>&1; rc=$?; tail -2 gpurun_out/t_lj.log; [ $rc -eq 0 ] || exit 1
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config']['final_loss'])" $1 $2; }
for i in 1 2 3; do
timeout -k 10 200 python bench.py > gpurun_out/lj1_$i.log 2>&1 && ms gpurun_out/lj1_$i.log late_join &&
TTD_LATE_PROJ_JOIN=0 timeout -k 10 200 python bench.py > gpurun_out/lj0_$i.log 2>&1 && ms gpurun_out/lj0_$i.log early_join || exit 1
done
