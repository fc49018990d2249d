export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_engine.py > gpurun_out/t_rccl.log 2>&1; echo "rccl tests rc=$?"; tail -15 gpurun_out/t_rccl.log
timeout -k 10 400 python tools/comm_interference.py --out gpurun_out/interf.json > gpurun_out/interf.log 2>&1; echo "interf rc=$?"; tail -8 gpurun_out/interf.log
