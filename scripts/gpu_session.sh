#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r5
mkdir -p $O
S=${1:-s35}
export TMPDIR=/tmp
# solo PMC of the default GEMM (2-D per-XCD tile blocks, opts 205064) and of the previous default (205056)
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  -d $O/${S}_pmc_2d -o gemm --output-format csv -- python3 $R/scripts/gemm_only.py 4096 205064 > $O/${S}_pmc_2d.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  -d $O/${S}_pmc_2d_l2 -o gemm --output-format csv -- python3 $R/scripts/gemm_only.py 4096 205064 > $O/${S}_pmc_2d_l2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  -d $O/${S}_pmc_rr_l2 -o gemm --output-format csv -- python3 $R/scripts/gemm_only.py 4096 205056 > $O/${S}_pmc_rr_l2.log 2>&1 &&
KBENCH_GEMM_ONLY=1 timeout -k 10 150 python -u scripts/kbench.py > $O/${S}_kbench.jsonl 2> $O/${S}_kbench.log
