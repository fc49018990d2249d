#!/bin/bash
# round-3 A/B batch 2: BERT side-stream wgrad grid size, ResNet default, kernel trace of the step
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "200 e1.log python bench.py --model bert" "200 e2.log env TTD_WGRAD_WGS=192 python bench.py --model bert" \
 "200 e3.log python bench.py --model bert" "200 e4.log env TTD_WGRAD_WGS=192 python bench.py --model bert" \
 "120 r1.log python bench.py" "120 r2.log python bench.py" \
 "240 prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/p1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2"
for f in e1 e2 e3 e4 r1 r2; do printf "%-4s " $f; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log || echo missing; done
python3 tools/trace_step.py gpurun_out/p1/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/streams_p1.txt && head -40 gpurun_out/streams_p1.txt
