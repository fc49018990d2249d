#!/bin/bash
# BERT-Large: plain GEMMs on hipBLASLt (torch.addmm / mm: 1 = forward bias GEMMs, 2 = + plain data gradients) vs our persistent GEMM
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for f in ${BL_LIST:-2 1 0}; do
TTD_BERT_BLASLT=$f timeout -k 10 200 python bench.py --model bert > gpurun_out/bl_$f.log 2>&1 && bash tools/bench_val.sh "blaslt=$f" gpurun_out/bl_$f.log || { tail -20 gpurun_out/bl_$f.log; exit 1; }
done; done
