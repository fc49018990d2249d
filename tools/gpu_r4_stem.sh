#!/bin/bash
# stem weight gradient: row-invariant addressing hoisted out of the row loop; test, standalone, ResNet A/B vs the old kernel
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gemm_conv.py -k stem -m gpu > gpurun_out/stem_t.log 2>&1 || { tail -30 gpurun_out/stem_t.log; exit 1; }
tail -1 gpurun_out/stem_t.log
timeout -k 10 120 python tools/stem_bench.py 1024 && TTD_HIP_LIB_OVERRIDE=tensorflow_train_distributed_amd/lib/alt/libttd_hip_oldstem.so timeout -k 10 120 python tools/stem_bench.py 1024 || exit 1
for r in 1 2; do
timeout -k 10 150 python bench.py > gpurun_out/st_new.log 2>&1 && bash tools/bench_val.sh "new" gpurun_out/st_new.log || exit 1
TTD_HIP_LIB_OVERRIDE=tensorflow_train_distributed_amd/lib/alt/libttd_hip_oldstem.so timeout -k 10 150 python bench.py > gpurun_out/st_old.log 2>&1 && bash tools/bench_val.sh "old" gpurun_out/st_old.log || exit 1
done
