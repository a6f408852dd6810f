#!/bin/bash
# Round-3 GPU session f: 8mix HW-queue budget A/B (default / one masked stream
# per runner / 2 HW queues per process), 3 reps each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step NAME SECONDS cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) exit $rc ;; esac
  return 0
}
P=static-se,credit-fixed-ts,gpbs-ts,gpbs
step q8_default 300 python -u bench.py --mix 8mix --policies $P --reps 3 --out gpurun_out/q8_default.json
GPBS_ONE_MASKED=1 step q8_one 300 python -u bench.py --mix 8mix --policies $P --reps 3 --out gpurun_out/q8_one.json
GPU_MAX_HW_QUEUES=2 step q8_hwq2 300 python -u bench.py --mix 8mix --policies $P --reps 3 --out gpurun_out/q8_hwq2.json
