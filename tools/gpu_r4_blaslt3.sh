#!/bin/bash
# BERT-Large: weight gradients through hipBLASLt too (TTD_BERT_BLASLT=3) vs 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -c "
import torch
a=torch.randn(512,64,device='cuda').bfloat16(); b=torch.randn(512,32,device='cuda').bfloat16()
o=torch.empty(64,32,device='cuda')
torch.mm(a.t(), b, out_dtype=torch.float32, out=o)
print('mm out_dtype ok', (o - a.float().t() @ b.float()).abs().max().item())
" || exit 1
BL_LIST="3 2" bash tools/gpu_r4_blaslt.sh
