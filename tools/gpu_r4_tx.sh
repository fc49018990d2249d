#!/bin/bash
# transformer kernel tests + BERT engine tests + BERT bench (native row offsets / RNG advance)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_transformer.py tests/test_bert.py tests/test_kernels_misc.py -m gpu > gpurun_out/tx_tests.log 2>&1 || { tail -30 gpurun_out/tx_tests.log; exit 1; }
tail -1 gpurun_out/tx_tests.log
timeout -k 10 200 python bench.py --model bert > gpurun_out/tx_bert.log 2>&1 && bash tools/bench_val.sh "bert" gpurun_out/tx_bert.log || exit 1
