#!/bin/bash
# Config #5 round 3 h: shim tenants on one masked queue (their class home
# half) -- gpbs-budget / gpbs-se vs static-se, and the pre-fix multi-queue
# shim (+multiq) as the control; 5 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-5} \
  --policies solo,static-se,gpbs-budget,gpbs-se,gpbs-budget+multiq \
  --out gpurun_out/config5_r3h.json > gpurun_out/config5_r3h.log 2>&1
echo "config5h rc=$?"
