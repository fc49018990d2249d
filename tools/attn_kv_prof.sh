#!/bin/bash
# Per-kernel mean times of the attention kernels (rocprofv3 --kernel-trace --stats over
# tools/attn_bench.py) for each TTD_ATTN_KV_DIAG mode given. usage: bash tools/attn_kv_prof.sh [modes...]
export TMPDIR=/tmp
mkdir -p gpurun_out/attn_prof
for m in "${@:-0}"; do
  TTD_ATTN_KV_DIAG=$m timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_prof/m$m -o run \
    --output-format csv -- python3 tools/attn_bench.py 128 > gpurun_out/attn_prof/m$m.log 2>&1 || exit 1
  f=$(find gpurun_out/attn_prof/m$m -name "*kernel_stats.csv" | head -1)
  echo "mode $m"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "attn" in r["Name"]:
        print("  %8.1f us x%-5s %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:90]))
PY
done
