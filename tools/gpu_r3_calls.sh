export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/r -o run -- python bench.py --steps 2 --warmup 2 > gpurun_out/prof_r.log 2>&1 || { tail gpurun_out/prof_r.log; exit 1; }
f=$(ls gpurun_out/prof/r/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof/r/run_kernel_trace.csv)
python tools/trace_step.py $f --start stem_fwd_kernel --seq apply_kernel > gpurun_out/prof/calls_apply.txt
python tools/trace_step.py $f --start stem_fwd_kernel --seq pw_kernel > gpurun_out/prof/calls_pw.txt
python - $f > gpurun_out/prof/seq_main.txt <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "stem_fwd_kernel" in r["Kernel_Name"]]
last = rows[idx[-1]:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    n = r["Kernel_Name"].replace("ttdk::(anonymous namespace)::", "").replace("void ", "")
    n = (n.split("(")[0] if not n.startswith("big::") else n.split("(")[0])[:110]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%s %9.1f %8.1f grid=%s wg=%s %s" % (r["Stream_Id"], (s - t0) / 1e3, (e - s) / 1e3, r["Grid_Size_X"], r["Workgroup_Size_X"], n))
PY
gzip -f $f
grep -c . gpurun_out/prof/seq_main.txt
