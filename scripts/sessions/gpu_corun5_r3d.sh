#!/bin/bash
# Config #5 round 3 d: the daemon's counter set with TCP->TCC requests per SE
# (lean: TCC misses split by L2 requests, not VMEM instructions).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
GPBS_HWC_SPEC=lean timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 5 --warmup 2 --reps ${REPS:-5} \
  --policies solo,gpbs-se,gpbs-budget --out gpurun_out/config5_r3d_lean.json > gpurun_out/config5_r3d_lean.log 2>&1
echo "config5d rc=$?"
