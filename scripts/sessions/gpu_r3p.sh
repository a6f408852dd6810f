#!/bin/bash
# Round-3 GPU session p: config #5 with one masked queue per shim tenant, then
# the two-process masked-queue switch probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_corun5_r3h.sh || exit 1
timeout -k 10 400 python -u scripts/queue_switch_probe.py --reps 2 > gpurun_out/queue_switch_probe.json 2> gpurun_out/queue_switch_probe.log
echo "probe rc=$?"
