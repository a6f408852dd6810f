#!/bin/bash
# Round 4 session 29: the class EWMA following a drop at alpha 1/2
# (gpbs-fall, boot class_fall=1) on the phase mixes and the 8mix.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for mix in phase-ts phase 8mix; do
  echo "== $mix $(date +%T)"
  timeout -k 10 400 python -u bench.py --gpus 1 --mix $mix --policies gpbs,gpbs-fall --reps 5 \
    --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s29_$mix.json 2> gpurun_out/r4/s29_$mix.log || exit $?
  python scripts/corun_log_policies.py gpurun_out/r4/s29_$mix.log | grep -v "norm\|hw samples"
done
