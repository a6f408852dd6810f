#!/bin/bash
# Round-3 GPU session r: the new queue-probe GPU test, then the GPU suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step NAME SECONDS cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc secs=$(( $(date +%s) - t0 ))"
  case $rc in 124|134|137|139) exit $rc ;; esac
  return 0
}
step queue_probe_test 200 python -u -m pytest tests/test_gpu_queue_probe.py -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider
step gpu_tests_r 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke_r 200 python -u -c "import __graft_entry__ as g; g.smoke()"
