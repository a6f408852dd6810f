#!/bin/bash
# Round-3 GPU session j: GEMM A/B incl. balanced staging, kernel trace of the
# default GEMM vs hipBLASLt, PMC passes of the default kernel.
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
KBENCH_GEMM_ONLY=1 step kbench_gemm_j 200 python -u scripts/kbench.py
step stamps_bal 120 python -u scripts/gemm_stamps.py 4096 4352
mkdir -p gpurun_out/ktrace_gemm_j
(cd /tmp && export TMPDIR=/tmp KBENCH_GEMM_ONLY=1 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ktrace_gemm_j" -o run -- python3 "$R/scripts/kbench.py" > "$R/gpurun_out/ktrace_gemm_j/log.txt" 2>&1; echo "ktrace rc=$?")
OPTS="256" bash scripts/pmc_gemm.sh
