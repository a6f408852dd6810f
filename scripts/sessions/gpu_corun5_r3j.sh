#!/bin/bash
# Config #5 round 3 j: shim tenants choose among 3 same-mask queues by measured
# slice time (default now; early-abort exploration) vs the single-queue shim
# (+qp0), static-se and none; 5 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-5} \
  --policies solo,none,static-se,gpbs-budget,gpbs-budget+qp0 \
  --out gpurun_out/config5_r3j.json > gpurun_out/config5_r3j.log 2>&1
echo "config5j rc=$?"
