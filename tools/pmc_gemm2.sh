#!/bin/bash
# PMC passes: our persistent 256-row GEMM vs hipBLASLt at one shape. usage: bash tools/pmc_gemm2.sh M N K
export TMPDIR=/tmp
M=$1; N=$2; K=$3
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
for who in ours torch; do
  if [ $who = ours ]; then cmd="python3 tools/one_gemm.py $M $N $K 0 1 10"; else cmd="python3 tools/one_torch_gemm.py $M $N $K 10"; fi
  mkdir -p gpurun_out/pmc2_$who
  timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc2_$who/p1 -o run --output-format csv -- $cmd > gpurun_out/pmc2_$who/p1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/pmc2_$who/p2 -o run --output-format csv -- $cmd > gpurun_out/pmc2_$who/p2.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc2_ours gemm > gpurun_out/pmc2_ours.txt
python3 tools/pmc_summary.py gpurun_out/pmc2_torch Cijk > gpurun_out/pmc2_torch.txt || python3 tools/pmc_summary.py gpurun_out/pmc2_torch "" > gpurun_out/pmc2_torch.txt
cat gpurun_out/pmc2_ours.txt gpurun_out/pmc2_torch.txt
