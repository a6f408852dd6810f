#!/bin/bash
# Round-3 GPU session m: one-phase GEMM variant -- tests, A/B, stamps.
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
step gemm_variant_tests_m 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm"
KBENCH_GEMM_ONLY=1 step kbench_gemm_m 200 python -u scripts/kbench.py
step stamps_1phase 120 python -u scripts/gemm_stamps.py 4096 16640
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
