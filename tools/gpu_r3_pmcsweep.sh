#!/bin/bash
# PMC sweep over whole training steps (2 steps after 1 warm-up): core SQ counters for BERT-Large b128
# and ResNet-50 b1024, FETCH_SIZE / WRITE_SIZE passes for BERT (one counter group per run:
# rocprofv3 does not split passes; TCC budget), kernel trace for durations.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcs
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
run() {  # model tag counters...
  m=$1; t=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmcs/${m}_$t -o run --output-format csv -- python3 bench.py --model $m --steps 2 --warmup 1 > gpurun_out/pmcs/${m}_$t.log 2>&1 || { echo "pmc $m $t failed"; tail -5 gpurun_out/pmcs/${m}_$t.log; return 1; }
}
run bert core $C1 && run bert fetch FETCH_SIZE && run bert write WRITE_SIZE && run resnet50 core $C1 || exit 1
python3 tools/pmc_kernels.py gpurun_out/pmcs/bert_core gpurun_out/pmcs/bert_fetch gpurun_out/pmcs/bert_write --min 3 --top 30 > gpurun_out/pmcs/bert_kernels.txt
python3 tools/pmc_kernels.py gpurun_out/pmcs/resnet50_core --min 2 --top 30 > gpurun_out/pmcs/resnet50_kernels.txt
find gpurun_out/pmcs -name "*kernel_trace.csv" -delete
cat gpurun_out/pmcs/bert_kernels.txt | cut -c1-230 | head -30; cat gpurun_out/pmcs/resnet50_kernels.txt | cut -c1-200 | head -30
