#!/bin/bash
# Round 4 session 18: the fused PBS metric (GPBS_HWC_FUSE / policy gpbs-fuse:
# every metric tick from hardware-calibrated modeled deltas) -- the phase GPU
# test both ways, then gpbs vs gpbs-fuse on every default mix.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
echo "== phase test $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_phase.py -s \
  > gpurun_out/r4/s18_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error|to_memory_ms|to_compute_ms|fuse_ticks" gpurun_out/r4/s18_tests.log | head -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mix in phase-ts 8mix phase 4mix; do
  echo "== $mix $(date +%T)"
  extra=""; [ $mix = 4mix ] && extra=",static-se"; [ $mix = phase ] && extra=",credit-fixed"; [ $mix = phase-ts ] && extra=",credit-fixed-ts"
  timeout -k 10 400 python -u bench.py --gpus 1 --mix $mix --policies gpbs,gpbs-fuse$extra --reps 5 \
    --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s18_$mix.json 2> gpurun_out/r4/s18_$mix.log || exit $?
  python scripts/corun_log_policies.py gpurun_out/r4/s18_$mix.log | grep -v "norm\|hw samples"
done
