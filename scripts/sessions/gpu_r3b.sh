#!/bin/bash
# Round-3 GPU session: IPC all-reduce revocation debug (2 ranks), GEMM
# per-barrier stamps, then the full default bench (all mixes, 5 reps).
# Each GPU step under its own time limit; the session stops at the first
# step that fails in a way that may leave the GPU unhealthy.
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
if [ -z "${SKIP_IPC:-}" ]; then
  step ipc_debug 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 scripts/ipc_debug.py
fi
if [ -z "${SKIP_STAMPS:-}" ]; then
  step gemm_stamps 120 python -u scripts/gemm_stamps.py 4096
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  step bench_full 1000 python -u bench.py --out gpurun_out/bench_full.json
fi
