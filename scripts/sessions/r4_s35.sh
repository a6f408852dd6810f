#!/bin/bash
# Round 4 session 35: the CU-mask layout check on this box, next to a short
# 4mix (does a box where SE-partitioned policies lose break the assumed
# mask-bit -> shader-engine layout?).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 120 python -u scripts/cu_map_check.py > gpurun_out/r4/s35_cumap.json 2> gpurun_out/r4/s35_cumap.log || exit $?
cat gpurun_out/r4/s35_cumap.json
timeout -k 10 300 python -u bench.py --gpus 1 --mix 4mix --policies gpbs,static-se,none --reps 3 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s35_4mix.json 2> gpurun_out/r4/s35_4mix.log
echo "rc=$?"; python scripts/corun_log_policies.py gpurun_out/r4/s35_4mix.log | grep -v "^   "
