#!/bin/bash
# weight-gradient workgroup target sweep after the asm-DMA change (ResNet-50 b1024 bf16)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for w in ${WGS_LIST:-128 160 208 256}; do
TTD_WGRAD_WGS=$w timeout -k 10 150 python bench.py > gpurun_out/wgs_${w}_$r.log 2>&1 && echo "wgs=$w $(tail -1 gpurun_out/wgs_${w}_$r.log | cut -c100-135)" || exit 1
done; done
