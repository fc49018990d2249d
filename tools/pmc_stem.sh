#!/bin/bash
# PMC passes over the stem forward kernel (tools/stem_fwd_bench.py). usage: bash tools/pmc_stem.sh <tag>
export TMPDIR=/tmp
TAG=${1:-stem}
mkdir -p gpurun_out/pmc_$TAG
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/pmc_$TAG/p1 -o run --output-format csv -- python3 tools/stem_fwd_bench.py 256 > gpurun_out/pmc_$TAG/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_$TAG/p2 -o run --output-format csv -- python3 tools/stem_fwd_bench.py 256 > gpurun_out/pmc_$TAG/p2.log 2>&1 || exit 1
echo ok
