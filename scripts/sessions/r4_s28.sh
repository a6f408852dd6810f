#!/bin/bash
# Round 4 session 28: a 3x longer top of the PBS quantum range (memory
# tenants up to 33 ms, policy gpbs-q33) on the time-shared mixes.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for mix in phase-ts 8mix; do
  echo "== $mix $(date +%T)"
  timeout -k 10 400 python -u bench.py --gpus 1 --mix $mix --policies gpbs,gpbs-q33,credit-fixed-ts --reps 5 \
    --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s28_$mix.json 2> gpurun_out/r4/s28_$mix.log || exit $?
  python scripts/corun_log_policies.py gpurun_out/r4/s28_$mix.log | grep -v "norm\|hw samples"
done
