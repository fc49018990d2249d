#!/bin/bash
# MN-major LDS-DMA as inline asm (no compiler vmcnt(0) drains in the wgrad main loops): numerics + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gemm_conv.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gl_t.log 2>&1; rc=$?; tail -3 gpurun_out/gl_t.log; [ $rc -eq 0 ] || exit 1
ALT=tensorflow_train_distributed_amd/lib/alt/libttd_hip_builtin.so
for i in 1 2; do
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 150 python bench.py > gpurun_out/gl_r0_$i.log 2>&1 && tail -1 gpurun_out/gl_r0_$i.log | cut -c100-175 || exit 1
timeout -k 10 150 python bench.py > gpurun_out/gl_r1_$i.log 2>&1 && tail -1 gpurun_out/gl_r1_$i.log | cut -c100-175 || exit 1
done
TTD_HIP_LIB_OVERRIDE=$ALT timeout -k 10 240 python bench.py --model bert > gpurun_out/gl_b0.log 2>&1 && tail -1 gpurun_out/gl_b0.log | cut -c100-190 || exit 1
timeout -k 10 240 python bench.py --model bert > gpurun_out/gl_b1.log 2>&1 && tail -1 gpurun_out/gl_b1.log | cut -c100-190 || exit 1
