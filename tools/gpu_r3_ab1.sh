#!/bin/bash
# round-3 A/B batch: BN-prologue dgrad, fp8 + LAMB, stream priority, side-stream wgrad grid size
bash tools/gpu_steps.sh \
 "200 t_new.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gemm_conv.py -k in_kernel_fold" \
 "120 a1.log python bench.py" "120 a0.log env TTD_DGRAD_BNPRO=0 python bench.py" \
 "120 a1b.log python bench.py" "120 a0b.log env TTD_DGRAD_BNPRO=0 python bench.py" \
 "120 np.log env TTD_MAIN_PRIO=0 python bench.py" \
 "120 w192.log env TTD_WGRAD_WGS=192 python bench.py" "120 w128.log env TTD_WGRAD_WGS=128 python bench.py" \
 "120 f8.log python bench.py --precision fp8 --optimizer lamb" "120 bfl.log python bench.py --optimizer lamb" \
 "200 bb.log python bench.py --model bert" "200 bbw192.log env TTD_WGRAD_WGS=192 python bench.py --model bert" \
 "200 bbw128.log env TTD_WGRAD_WGS=128 python bench.py --model bert"
for f in a1 a0 a1b a0b np w192 w128 f8 bfl bb bbw192 bbw128; do
  printf "%-8s " $f; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log || echo missing
done
