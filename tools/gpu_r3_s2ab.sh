#!/bin/bash
# weight-prep test + ResNet tests; A/B: wprep on/off, eager vs segmented graph; BERT bench + GEMM bench + trace.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_kernels_gemm_conv.py tests/test_resnet_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_ab.log 2>&1; rc=$?; tail -2 gpurun_out/t_ab.log; [ $rc -eq 0 ] || exit 1
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config']['final_loss'])" $1 $2; }
for i in 1 2; do
timeout -k 10 200 python bench.py > gpurun_out/ab_e$i.log 2>&1 && ms gpurun_out/ab_e$i.log eager_wprep &&
TTD_WPREP=0 timeout -k 10 200 python bench.py > gpurun_out/ab_n$i.log 2>&1 && ms gpurun_out/ab_n$i.log eager_nowprep &&
timeout -k 10 200 python bench.py --graph 1 > gpurun_out/ab_g$i.log 2>&1 && ms gpurun_out/ab_g$i.log graph || exit 1
done
timeout -k 10 200 python bench.py --model bert > gpurun_out/bert_s2.log 2>&1 && tail -1 gpurun_out/bert_s2.log &&
timeout -k 10 300 python tools/gemm_bench.py --tokens 65536 --only bert > gpurun_out/gemm_bert65k.txt 2>&1 && cat gpurun_out/gemm_bert65k.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/bert -o run -- python bench.py --model bert --steps 3 --warmup 2 > gpurun_out/prof_bert.log 2>&1 || { tail gpurun_out/prof_bert.log; exit 1; }
f=$(ls gpurun_out/prof/bert/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof/bert/run_kernel_trace.csv)
python tools/trace_step.py $f --start embed_fwd_kernel --streams > gpurun_out/prof/trace_bert.txt
head -40 gpurun_out/prof/trace_bert.txt; grep "^stream" gpurun_out/prof/trace_bert.txt
