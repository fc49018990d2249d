#!/bin/bash
# ResNet-50 b1024 step: which main-stream kernels run with the chip to themselves (critical path)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/solo -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/solo.log 2>&1 || exit 1
cd tools && python3 solo_time.py ../gpurun_out/solo/run_kernel_trace.csv --start stem_fwd --top 30 > ../gpurun_out/solo_resnet.txt && head -60 ../gpurun_out/solo_resnet.txt
rm -f ../gpurun_out/solo/run_kernel_trace.csv
