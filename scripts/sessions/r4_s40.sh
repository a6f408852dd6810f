#!/bin/bash
# Round 4 session 40: HIP's own hardware queues per process 8 (default) vs 4 vs 2
# (GPBS_HWQ) on the 8mix slow-run mode, one process each, same box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for hq in 8 4 2; do
  echo "== hwq=$hq $(date +%T)"
  GPBS_HWQ=$hq timeout -k 10 400 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,credit-fixed-ts,none --reps 6 \
    --steps 20 --warmup 3 --no-resolo --no-cu-check > gpurun_out/r4/s40_hwq$hq.json 2> gpurun_out/r4/s40_hwq$hq.log || exit $?
  python scripts/corun_log_policies.py gpurun_out/r4/s40_hwq$hq.log | grep -v "^   "
done
