#!/bin/bash
# Round-3 GPU session o: the driver's N>1 path with every mix (4mix, phase,
# 8mix), rehearsed with 2 ranks on one GPU (gated IPC all-reduce tenant, native
# gang coordinator); not a measurement.
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
step rehearse_all2 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --rehearse-ipc --counters model --reps 1 --reps-extra 1 \
  --steps 5 --warmup 2 --out gpurun_out/rehearse_all2.json
