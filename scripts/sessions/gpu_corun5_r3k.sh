#!/bin/bash
# Config #5 round 3 k: the co-resident shim policy (gpbs, 2 contexts, no CU
# masks) with and without the measured queue choice (+qp3), next to none,
# static-se and the flagship gpbs-budget; 4 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-4} \
  --policies solo,none,gpbs,gpbs+qp3,static-se,gpbs-budget \
  --out gpurun_out/config5_r3k.json > gpurun_out/config5_r3k.log 2>&1
echo "config5k rc=$?"
