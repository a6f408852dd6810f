#!/bin/bash
# Config #5 round 3 e: why gpbs-se collapses in some runs -- per-step gate/run
# timelines, KFD queue counts, and two queue-set variants (tenant
# GPU_MAX_HW_QUEUES=2; both SE-half streams created at registration).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-3} \
  --policies solo,static-se,gpbs-se,gpbs-se+hwq2,gpbs-se+pre --out gpurun_out/config5_r3e.json > gpurun_out/config5_r3e.log 2>&1
echo "config5e rc=$?"
