export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/b0.log 2>&1 && tail -1 gpurun_out/b0.log &&
timeout -k 10 200 python bench.py --model bert > gpurun_out/bb0.log 2>&1 && tail -1 gpurun_out/bb0.log &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/p0 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/p0.log 2>&1 && python3 tools/kstats.py gpurun_out/p0/run_kernel_stats.csv "ResNet-50 b1024 r3 start" 6 > gpurun_out/kstats_p0.md && head -30 gpurun_out/kstats_p0.md
