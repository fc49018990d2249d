#!/bin/bash
# fp8 e5m2 data gradients: kernel + engine tests, fp8 bench A/B; late forward-projection join A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gemm_conv.py tests/test_resnet_engine.py -x -q -m gpu --timeout 120 --timeout-method thread -k "fp8 or e5m2 or resnet or weight_prep" > gpurun_out/t_fp8dg.log 2>&1; rc=$?; tail -4 gpurun_out/t_fp8dg.log; [ $rc -eq 0 ] || exit 1
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config']['final_loss'])" $1 $2; }
for i in 1 2; do
timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/f8dg1_$i.log 2>&1 && ms gpurun_out/f8dg1_$i.log fp8_dgrad8 &&
TTD_FP8_DGRAD=0 timeout -k 10 200 python bench.py --precision fp8 --optimizer lamb > gpurun_out/f8dg0_$i.log 2>&1 && ms gpurun_out/f8dg0_$i.log fp8_dgrad16 &&
timeout -k 10 200 python bench.py --optimizer lamb > gpurun_out/bfl_$i.log 2>&1 && ms gpurun_out/bfl_$i.log bf16_lamb &&
timeout -k 10 200 python bench.py > gpurun_out/lj1_$i.log 2>&1 && ms gpurun_out/lj1_$i.log bf16_late_join &&
TTD_LATE_PROJ_JOIN=0 timeout -k 10 200 python bench.py > gpurun_out/lj0_$i.log 2>&1 && ms gpurun_out/lj0_$i.log bf16_early_join || exit 1
done
