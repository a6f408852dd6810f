#!/bin/bash
# Round-3 GPU session h: GEMM fence-free finish A/B; 8mix with the region
# quantum (time-shared class regions rotate in one quantum).
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
KBENCH_GEMM_ONLY=1 step kbench_gemm_h 200 python -u scripts/kbench.py
step b8_region 400 python -u bench.py --mix 8mix --out gpurun_out/b8_region.json
