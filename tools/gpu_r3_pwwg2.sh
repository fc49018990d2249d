export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_pw.py::test_pw_bn_backward_prologue_fused_weight_gradient tests/test_resnet_engine.py > gpurun_out/t_pwwg2.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/t_pwwg2.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/grad_path_check.py --attr pw_wgrad > gpurun_out/pwwg_check2.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/pwwg_check2.json')); print(d['rel_grad_on_vs_off'], d['cos_on_vs_off'], d['worst_vars'][:6])"
for i in 1 2; do
  for v in 0 1; do
    TTD_PW_WGRAD=$v timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_pwwg$v$i.json 2> gpurun_out/b_pwwg$v$i.err || exit 1
    tail -1 gpurun_out/b_pwwg$v$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pw_wgrad=$v', d['ms_per_step'], d['config']['final_loss'])"
  done
done
