#!/bin/bash
# Round 4 session 37: SE-mode runners without CU-masked queues (gate per
# workgroup only, GPBS_SE_MASKED=0) vs the default, one process each.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for mk in 1 0; do
  for mix in 4mix 8mix; do
    echo "== $mix masked=$mk $(date +%T)"
    GPBS_SE_MASKED=$mk timeout -k 10 400 python -u bench.py --gpus 1 --mix $mix --policies gpbs,credit-fixed,none --reps 5 \
      --steps 20 --warmup 3 --no-resolo --no-cu-check > gpurun_out/r4/s37_${mix}_m$mk.json 2> gpurun_out/r4/s37_${mix}_m$mk.log || exit $?
    python scripts/corun_log_policies.py gpurun_out/r4/s37_${mix}_m$mk.log | grep -v "^   "
  done
done
