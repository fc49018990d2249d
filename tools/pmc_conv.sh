#!/bin/bash
# PMC passes over one conv GEMM. usage: bash tools/pmc_conv.sh <layer> <op> <tag>
export TMPDIR=/tmp
L=$1; OP=$2; TAG=$3
mkdir -p gpurun_out/pmc_$TAG
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/pmc_$TAG/p1 -o run --output-format csv -- python3 tools/one_conv.py $L $OP 10 > gpurun_out/pmc_$TAG/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_$TAG/p2 -o run --output-format csv -- python3 tools/one_conv.py $L $OP 10 > gpurun_out/pmc_$TAG/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_$TAG/p3 -o run --output-format csv -- python3 tools/one_conv.py $L $OP 10 > gpurun_out/pmc_$TAG/p3.log 2>&1 || exit 1
echo ok
