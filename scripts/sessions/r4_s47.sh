#!/bin/bash
# Round 4 session 47: PMC of the SHIPPED GEMM default (opts 256|8192 = 8448,
# own-A two-phase kernel), two passes, each its own short run (no trace
# domains beyond the kernel trace).
set -o pipefail
cd "$(dirname "$0")/../.."
R=$(pwd)
mkdir -p gpurun_out/r4/pmc47
export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES"
P2="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace -d $R/gpurun_out/r4/pmc47/p1 -o p1 -- python3 $R/scripts/gemm_only.py 4096 8448 \
  > gpurun_out/r4/pmc47/p1.log 2>&1 || exit $?
echo "pass1 ok"
timeout -s KILL 90 rocprofv3 --pmc $P2 --kernel-trace -d $R/gpurun_out/r4/pmc47/p2 -o p2 -- python3 $R/scripts/gemm_only.py 4096 8448 \
  > gpurun_out/r4/pmc47/p2.log 2>&1 || exit $?
echo "pass2 ok"
python scripts/pmc_summary.py gemm256s2 gpurun_out/r4/pmc47/p1/p1_results.db > gpurun_out/r4/pmc47/summary.txt 2>&1
python scripts/pmc_summary.py gemm256s2 gpurun_out/r4/pmc47/p2/p2_results.db >> gpurun_out/r4/pmc47/summary.txt 2>&1
cat gpurun_out/r4/pmc47/summary.txt
