export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python tools/gemm_bench.py --tokens 65536 --only bert > gpurun_out/gemm_bert65k.txt 2>&1 || { tail gpurun_out/gemm_bert65k.txt; exit 1; }
cat gpurun_out/gemm_bert65k.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/bert -o run -- python bench.py --model bert --steps 3 --warmup 2 > gpurun_out/prof_bert.log 2>&1 || { tail gpurun_out/prof_bert.log; exit 1; }
f=$(ls gpurun_out/prof/bert/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof/bert/run_kernel_trace.csv)
python tools/trace_step.py $f --start embed_fwd_kernel --streams > gpurun_out/prof/trace_bert.txt
rm -f $f
head -40 gpurun_out/prof/trace_bert.txt; grep "^stream" gpurun_out/prof/trace_bert.txt
