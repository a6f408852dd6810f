#!/bin/bash
# Config #5 round 3 f: queue-set variants against the collapse (4 reps each):
# SE-half streams created at registration (+pre), with tenant
# GPU_MAX_HW_QUEUES=2 (+hwq2), tenant hwq 1, and the daemon process at 2 queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-4} \
  --daemon-hwq 2 --policies solo,static-se,gpbs-se,gpbs-se+pre,gpbs-se+pre+hwq2,gpbs-se+hwq1 \
  --out gpurun_out/config5_r3f.json > gpurun_out/config5_r3f.log 2>&1
echo "config5f rc=$?"
