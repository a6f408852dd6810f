#!/bin/bash
# Round 4 session 13: k_hwc_attribute cost after device staging (rocprofv3
# kernel trace); the sampler cadence (duty cap 1 / 5 / 10 %, i.e. a hardware
# period of ~20 / ~4 / ~2 ms) on the 8mix and the 4mix; a final-tree co-run
# kernel trace (4mix, gpbs).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== rocprof attr $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_attr13 -o attr -- python3 scripts/attr_bench.py 500 \
  > gpurun_out/r4/s13_prof_attr.log 2>&1 || exit $?
python scripts/rocpd_summary.py gpurun_out/r4/prof_attr13/attr_results.db -o gpurun_out/r4/s13_attr_summary.txt | head -6
echo "== 8mix cadence $(date +%T)"
timeout -k 10 400 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,gpbs-d5,gpbs-d10 --reps 5 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s13_8mix.json 2> gpurun_out/r4/s13_8mix.log || exit $?
python scripts/corun_log_policies.py gpurun_out/r4/s13_8mix.log
echo "== 4mix cadence $(date +%T)"
timeout -k 10 400 python -u bench.py --gpus 1 --mix 4mix --policies gpbs,gpbs-d5,gpbs-d10,static-se --reps 5 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s13_4mix.json 2> gpurun_out/r4/s13_4mix.log || exit $?
python scripts/corun_log_policies.py gpurun_out/r4/s13_4mix.log
echo "== rocprof co-run $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_corun13 -o corun -- python3 bench.py --gpus 1 \
  --mix 4mix --policies gpbs --reps 1 --steps 10 --warmup 2 --no-resolo > gpurun_out/r4/s13_prof_corun.log 2>&1
echo "rocprof corun rc=$?"; python scripts/rocpd_summary.py gpurun_out/r4/prof_corun13/corun_results.db -o gpurun_out/r4/s13_corun_summary.txt | head -30
