#!/bin/bash
# Round-3 GPU session e: full default bench (masked-stream pool), sampler duty
# 1 % A/B on 4mix + phase, GEMM PMC passes, kernel trace of the GEMM bench.
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
step bench_full_b 600 python -u bench.py --out gpurun_out/bench_full_b.json
GPBS_HWC_DUTY=1 step duty1_4mix 200 python -u bench.py --mix 4mix --policies none,static-se,gpbs --out gpurun_out/duty1_4mix.json
GPBS_HWC_DUTY=1 step duty1_phase 200 python -u bench.py --mix phase --policies static-se,gpbs --out gpurun_out/duty1_phase.json
bash scripts/pmc_gemm.sh || exit 1
mkdir -p gpurun_out/ktrace_gemm
(cd /tmp && export TMPDIR=/tmp KBENCH_GEMM_ONLY=1 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ktrace_gemm" -o run -- python3 "$R/scripts/kbench.py" > "$R/gpurun_out/ktrace_gemm/log.txt" 2>&1; echo "ktrace rc=$?")
