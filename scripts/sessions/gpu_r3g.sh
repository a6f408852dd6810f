#!/bin/bash
# Round-3 GPU session g: GEMM variant A/B (2-phase, streaming C stores, 2-D
# XCD blocks), stamps, then the full default bench on the final policy set.
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
KBENCH_GEMM_ONLY=1 step kbench_gemm_g 200 python -u scripts/kbench.py
step stamps_ntc2d 120 python -u scripts/gemm_stamps.py 4096 1288
step bench_full_c 700 python -u bench.py --out gpurun_out/bench_full_c.json
