#!/bin/bash
# Round-3 GPU session l: xGMI gang exchange test, then the final full bench.
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
step gang_xgmi_test 200 python -u -m pytest tests/test_gpu_gang_xgmi.py -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider
step bench_full_e 600 python -u bench.py --out gpurun_out/bench_full_e.json
step rehearse_ipc2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --rehearse-ipc --counters model --mix 4mix --policies none,gpbs --reps 1 \
  --steps 5 --warmup 2 --out gpurun_out/rehearse_ipc2.json
