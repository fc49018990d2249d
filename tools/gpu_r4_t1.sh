export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_engine.py tests/test_kernels_misc.py -k "bf16_rounding or rccl or segmented or bucket or watchdog or probe or version or persistent" > gpurun_out/r4_t1.log 2>&1; rc=$?; tail -25 gpurun_out/r4_t1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --graph 1 > gpurun_out/r4_bg1.log 2>&1 && tail -1 gpurun_out/r4_bg1.log | cut -c1-300
timeout -k 10 120 python tools/graph_prio_probe2.py > gpurun_out/r4_gprio.log 2>&1; tail -6 gpurun_out/r4_gprio.log
