#!/bin/bash
# stem weight gradient variant: standalone vs the committed kernel (alt lib), plus its test
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gemm_conv.py -k stem -m gpu > gpurun_out/stem_t.log 2>&1 || { tail -30 gpurun_out/stem_t.log; exit 1; }
tail -1 gpurun_out/stem_t.log
for r in 1 2; do
timeout -k 10 120 python tools/stem_bench.py 1024 && TTD_HIP_LIB_OVERRIDE=tensorflow_train_distributed_amd/lib/alt/libttd_hip_oldstem.so timeout -k 10 120 python tools/stem_bench.py 1024 || exit 1
done
