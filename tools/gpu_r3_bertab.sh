#!/bin/bash
# BERT-Large b128 A/B: side-stream wgrad workgroup target, main-stream priority
export TMPDIR=/tmp
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'])" $1 $2; }
for i in 1 2; do
timeout -k 10 200 python bench.py --model bert > gpurun_out/bab_d$i.log 2>&1 && ms gpurun_out/bab_d$i.log default &&
TTD_BERT_WGRAD_WGS=160 timeout -k 10 200 python bench.py --model bert > gpurun_out/bab_w160_$i.log 2>&1 && ms gpurun_out/bab_w160_$i.log wgs160 &&
TTD_BERT_WGRAD_WGS=224 timeout -k 10 200 python bench.py --model bert > gpurun_out/bab_w224_$i.log 2>&1 && ms gpurun_out/bab_w224_$i.log wgs224 &&
TTD_MAIN_PRIO=1 timeout -k 10 200 python bench.py --model bert > gpurun_out/bab_p1_$i.log 2>&1 && ms gpurun_out/bab_p1_$i.log main_prio || exit 1
done
