#!/bin/bash
# Round 4 session 57: PMC of the new GEMM default (LDS-staged C, non-temporal; opts 205056)
# next to the round-3 default (8448), same box, one pass each.
set -o pipefail
cd "$(dirname "$0")/../.."
R=$(pwd)
mkdir -p gpurun_out/r4/pmc57
export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES"
for o in 205056 8448; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace -d $R/gpurun_out/r4/pmc57/o$o -o o$o -- python3 $R/scripts/gemm_only.py 4096 $o \
    > gpurun_out/r4/pmc57/o$o.log 2>&1 || exit $?
  echo "pass $o ok"
  python scripts/pmc_summary.py gemm256s2 gpurun_out/r4/pmc57/o$o/o${o}_results.db > gpurun_out/r4/pmc57/summary_$o.txt 2>&1
  cat gpurun_out/r4/pmc57/summary_$o.txt
done
