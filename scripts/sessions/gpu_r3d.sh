#!/bin/bash
# Round-3 GPU session d: GEMM phase stamps, --mix all with the masked-stream
# pool (8mix after 4mix/phase in one process), rocprofv3 scheduler-kernel summary.
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
step stamps_s2b 120 python -u scripts/gemm_stamps.py 4096 256
step ball_pool 500 python -u bench.py --reps 2 --reps-extra 2 --policies none,static-se,gpbs --out gpurun_out/ball_pool.json
bash scripts/prof_r3.sh
