#!/bin/bash
# PMC passes over the LayerNorm backward kernel
export TMPDIR=/tmp
D=gpurun_out/pmc_ln
mkdir -p $D
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
C2="SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum"
timeout -s KILL 90 rocprofv3 --pmc $C1 -d $D/p1 -o run --output-format csv -- python3 tools/ln_bwd_only.py > $D/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C2 -d $D/p2 -o run --output-format csv -- python3 tools/ln_bwd_only.py > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
python3 tools/pmc_summary.py $D ln_bwd > $D.txt && cat $D.txt
