#!/bin/bash
# BERT-Large b128 step: which main-stream kernels run with the chip to themselves (critical path)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/solob -o run -- python3 bench.py --model bert --steps 3 --warmup 2 > gpurun_out/solob.log 2>&1 || exit 1
cd tools && python3 solo_time.py ../gpurun_out/solob/run_kernel_trace.csv --start embed_fwd --top 25 > ../gpurun_out/solo_bert.txt && head -30 ../gpurun_out/solo_bert.txt
rm -f ../gpurun_out/solob/run_kernel_trace.csv
