#!/bin/bash
# Round 4 session 10: engine trace rings of 8 gpbs 8mix runs (good and bad
# ones) for offline analysis of the steal / wake storms.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/diag
echo "== traces $(date +%T)"
GPBS_DIAG_DIR=gpurun_out/r4/diag timeout -k 10 240 python -u bench.py --gpus 1 --mix 8mix --policies gpbs --reps 8 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s10.json 2> gpurun_out/r4/s10.log
echo "rc=$? $(date +%T)"; python scripts/corun_log_policies.py gpurun_out/r4/s10.log | grep -v "^ "
ls -la gpurun_out/r4/diag | tail -9
