#!/bin/bash
# Round-4 start: ResNet bench, BERT bench, ResNet per-stream kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/r4_b0.log 2>&1 && tail -1 gpurun_out/r4_b0.log | cut -c1-200 &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/r4_bb0.log 2>&1 && tail -1 gpurun_out/r4_bb0.log | cut -c1-200 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_p0 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r4_p0.log 2>&1 && python3 tools/kstats.py gpurun_out/r4_p0/run_kernel_stats.csv "ResNet-50 b1024 r4 start" 6 > gpurun_out/r4_kstats0.md && python3 tools/trace_step.py gpurun_out/r4_p0/run_kernel_trace.csv --start stem_fwd --streams > gpurun_out/r4_streams0.txt && head -12 gpurun_out/r4_streams0.txt
timeout -k 10 120 python tools/pack_ab.py --tag new --steps 3 > gpurun_out/r4_pab_new.log 2>&1 && tail -1 gpurun_out/r4_pab_new.log &&
TTD_HIP_LIB_OVERRIDE=$PWD/tensorflow_train_distributed_amd/lib/libttd_hip_oldpack.so timeout -k 10 120 python tools/pack_ab.py --tag old --steps 3 > gpurun_out/r4_pab_old.log 2>&1 && tail -1 gpurun_out/r4_pab_old.log &&
python tools/pack_ab.py --compare new old > gpurun_out/r4_pab_cmp.txt 2>&1; head -30 gpurun_out/r4_pab_cmp.txt
