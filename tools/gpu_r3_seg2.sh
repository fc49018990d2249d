export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for g in 0 1; do
  TTD_WGRAD_STREAM=0 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph $g > gpurun_out/b1s_g$g.json 2>/dev/null || exit 1
  tail -1 gpurun_out/b1s_g$g.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1stream graph=$g', d['ms_per_step'])"
done
for g in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/g$g -o run -- python bench.py --steps 3 --warmup 2 --graph $g > gpurun_out/prof_g$g.log 2>&1 || exit 1
  f=$(ls gpurun_out/prof/g$g/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof/g$g/run_kernel_trace.csv)
  python tools/trace_step.py $f --start stem_fwd_kernel --streams > gpurun_out/prof/trace_g$g.txt
  head -1 gpurun_out/prof/trace_g$g.txt; grep "^stream" gpurun_out/prof/trace_g$g.txt
  rm -f $f
done
