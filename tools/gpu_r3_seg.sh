export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_resnet_engine.py -k "hipgraph or segmented" tests/test_bert.py > gpurun_out/t_seg.log 2>&1
rc=$?; echo "seg tests rc=$rc"; tail -12 gpurun_out/t_seg.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 0 > gpurun_out/b_eager$i.json 2> gpurun_out/b_eager$i.err || exit 1
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 1 > gpurun_out/b_seg$i.json 2> gpurun_out/b_seg$i.err || exit 1
  python - <<'PY' $i
import json,sys
i=sys.argv[1]
for k in ("eager","seg"):
    d=json.loads(open("gpurun_out/b_%s%s.json"%(k,i)).read().strip().splitlines()[-1])
    print(k, i, d["ms_per_step"], d["config"].get("hipgraph_capture"))
PY
done
