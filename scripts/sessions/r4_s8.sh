#!/bin/bash
# Round 4 session 8: the 8mix after the queue fixes (shared keyed masked
# queues, cap 2 per mask, sampler budget 5 %): none / static-se / gpbs x 5,
# with the bench's 8 normal HW queues and with 4 (GPBS_HWQ=4); then the GPU
# tests.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
run() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 240 env "$@" > gpurun_out/r4/s8_$name.json 2> gpurun_out/r4/s8_$name.log
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  python scripts/corun_log_policies.py gpurun_out/r4/s8_$name.log | grep -v "^ " 
  grep -o '"_end_over_start_rate[^}]*}' gpurun_out/r4/s8_$name.json | head -2
  grep -o '"masked_queues_created": [0-9]*' gpurun_out/r4/s8_$name.log | sort | uniq -c | head -3
  return $rc
}
B="python -u bench.py --gpus 1 --mix 8mix --policies none,static-se,gpbs --reps 5 --steps 20 --warmup 3"
run hwq8 GPBS_X=0 $B && \
run hwq4 GPBS_HWQ=4 $B
echo "== gpu tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4/s8_gpu_tests.log 2>&1
echo "tests rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4/s8_gpu_tests.log | grep -v PASSED | head; tail -2 gpurun_out/r4/s8_gpu_tests.log
