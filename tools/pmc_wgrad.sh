#!/bin/bash
# PMC passes over BERT's weight-gradient GEMM (fused bias row sums, split-K). usage: bash tools/pmc_wgrad.sh M N K
export TMPDIR=/tmp
M=$1; N=$2; K=$3
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
cmd="python3 tools/one_wgrad.py $M $N $K 10"
D=gpurun_out/pmcw_${M}_${N}
mkdir -p $D
timeout -k 10 120 python3 tools/one_wgrad.py $M $N $K 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C1 -d $D/p1 -o run --output-format csv -- $cmd > $D/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C2 -d $D/p2 -o run --output-format csv -- $cmd > $D/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py $D gemm256 > $D.txt && cat $D.txt
