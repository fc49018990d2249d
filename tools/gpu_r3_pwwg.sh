export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_pw.py tests/test_resnet_engine.py > gpurun_out/t_pwwg.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/t_pwwg.log | tail -30; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    TTD_PW_WGRAD=$v timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_pwwg$v$i.json 2> gpurun_out/b_pwwg$v$i.err || exit 1
    tail -1 gpurun_out/b_pwwg$v$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pw_wgrad=$v', d['ms_per_step'], d['config']['final_loss'])"
  done
done
