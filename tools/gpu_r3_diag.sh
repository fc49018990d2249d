export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/seg_capture_diag.py > gpurun_out/diag1.json 2> gpurun_out/diag1.err || { tail -20 gpurun_out/diag1.err; exit 1; }
cat gpurun_out/diag1.json
TTD_CD_SIDE=0 timeout -k 10 120 python tools/seg_capture_diag.py > gpurun_out/diag2.json 2> gpurun_out/diag2.err || { tail -20 gpurun_out/diag2.err; exit 1; }
cat gpurun_out/diag2.json
TTD_WGRAD_STREAM=0 timeout -k 10 120 python tools/seg_capture_diag.py > gpurun_out/diag3.json 2> gpurun_out/diag3.err || { tail -20 gpurun_out/diag3.err; exit 1; }
cat gpurun_out/diag3.json
