#!/bin/bash
# Round 4 session 23: hardware sampling backing off to 50 ms once no owner has
# changed for 20 ms (policy gpbs-slow50) vs the default, on every default mix.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for mix in 4mix phase phase-ts 8mix; do
  echo "== $mix $(date +%T)"
  timeout -k 10 400 python -u bench.py --gpus 1 --mix $mix --policies gpbs,gpbs-slow50 --reps 5 \
    --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s23_$mix.json 2> gpurun_out/r4/s23_$mix.log || exit $?
  python scripts/corun_log_policies.py gpurun_out/r4/s23_$mix.log | grep -v "norm\|tslice"
done
