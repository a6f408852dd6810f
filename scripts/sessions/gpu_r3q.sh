#!/bin/bash
# Round-3 GPU session q: same-mask queues differ (probe rotate arms), then
# config #5 with measured queue choice in the shim (+qp3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/queue_switch_probe.py --reps 3 --arms rotate,rotate-graph,fixed-graph \
  > gpurun_out/queue_rotate_probe.json 2> gpurun_out/queue_rotate_probe.log
echo "probe rc=$?"
timeout -k 10 800 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-5} \
  --policies solo,static-se,gpbs-budget+qp3,gpbs-se+qp3,gpbs-budget \
  --out gpurun_out/config5_r3i.json > gpurun_out/config5_r3i.log 2>&1
echo "config5i rc=$?"
