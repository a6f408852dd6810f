#!/bin/bash
# Round 4 session 42: HIP's own hardware queues per process 12 vs 8, alternating processes
# (GPBS_HWQ) on the 8mix slow-run mode, one process each, same box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
n=0
for hq in 12 8 12 8; do
  n=$((n+1))
  echo "== hwq=$hq $(date +%T)"
  GPBS_HWQ=$hq timeout -k 10 400 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,credit-fixed-ts --reps 8 \
    --steps 20 --warmup 3 --no-resolo --no-cu-check > gpurun_out/r4/s42_${n}_hwq$hq.json 2> gpurun_out/r4/s42_${n}_hwq$hq.log || exit $?
  python scripts/corun_log_policies.py gpurun_out/r4/s42_${n}_hwq$hq.log | grep -v "^   "
done
