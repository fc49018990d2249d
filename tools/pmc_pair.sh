#!/bin/bash
# Two rocprofv3 --pmc passes (issue/wait mix, then instruction / LDS counts) over one command,
# summarised per kernel by tools/pmc_summary.py.
# usage: bash tools/pmc_pair.sh LABEL KERNEL_SUBSTR -- CMD...
export TMPDIR=/tmp
L=$1; F=$2; shift 3
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
mkdir -p gpurun_out/pmc_$L
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc_$L/p1 -o run --output-format csv -- "$@" > gpurun_out/pmc_$L/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/pmc_$L/p2 -o run --output-format csv -- "$@" > gpurun_out/pmc_$L/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_$L "$F" > gpurun_out/pmc_$L.txt
cat gpurun_out/pmc_$L.txt
