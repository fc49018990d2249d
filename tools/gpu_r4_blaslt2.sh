#!/bin/bash
# BERT engine tests with the library path, then the step A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
TTD_BERT_BLASLT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bert.py -m gpu > gpurun_out/bl_t.log 2>&1 || { tail -30 gpurun_out/bl_t.log; exit 1; }
tail -1 gpurun_out/bl_t.log
BL_LIST="2 0" bash tools/gpu_r4_blaslt.sh
