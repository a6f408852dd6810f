#!/bin/bash
# Round 4 session 11: 8mix gpbs x 8 with the sibling-stack steal guard
# (credit.cpp runq_steal, boot sibling_steal=0) against session 10's
# bimodal [1.165 1.005 1.001 1.006 1.002 0.678 1.134 0.687]; none x 3 for
# the box's own reference.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/diag11
echo "== gpbs x8 $(date +%T)"
GPBS_DIAG_DIR=gpurun_out/r4/diag11 timeout -k 10 300 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,none --reps 8 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s11.json 2> gpurun_out/r4/s11.log
echo "rc=$? $(date +%T)"; python scripts/corun_log_policies.py gpurun_out/r4/s11.log | grep -v "^ "
ls -la gpurun_out/r4/diag11 | tail -4
