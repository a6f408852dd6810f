#!/bin/bash
# Config #5 round 3 b: the budget layout in the daemon path (gpbs-budget)
# next to gpbs-se and static-se, 5 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 5 --warmup 2 --reps ${REPS:-5} \
  --policies solo,static-se,gpbs-se,gpbs-budget --out gpurun_out/config5_r3c_5rep.json > gpurun_out/config5_r3c_5rep.log 2>&1
echo "config5b rc=$?"
