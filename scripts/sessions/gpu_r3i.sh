#!/bin/bash
# Round-3 GPU session i: the GPU test suite on the final kernels, GEMM stamps
# and kernel trace of the default kernel, then the full default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
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
step gpu_tests 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step stamps_default 120 python -u scripts/gemm_stamps.py 4096 256
step bench_full_d 600 python -u bench.py --out gpurun_out/bench_full_d.json
