export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_pw.py::test_pw_bn_backward_prologue_fused_weight_gradient > gpurun_out/t_sidepw.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_sidepw.log; [ $rc -eq 0 ] || exit $rc
run() {
  name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_spw_$name.json 2> gpurun_out/b_spw_$name.err || { tail -5 gpurun_out/b_spw_$name.err; exit 1; }
  tail -1 gpurun_out/b_spw_$name.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
}
for r in a b; do
run full$r TTD_SIDE_PW_WGS=0
run w128$r TTD_SIDE_PW_WGS=128
run w64$r TTD_SIDE_PW_WGS=64
run w192$r TTD_SIDE_PW_WGS=192
done
