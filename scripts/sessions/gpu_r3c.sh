#!/bin/bash
# Round-3 GPU session c: 2-phase GEMM A/B + stamps, IPC all-reduce (yielding
# barrier) test + revocation debug, 8mix alone (HW-queue leak check).
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
step stamps_s2 120 python -u scripts/gemm_stamps.py 4096 256
step stamps_4 120 python -u scripts/gemm_stamps.py 4096 4
KBENCH_GEMM_ONLY=1 step kbench_gemm 200 python -u scripts/kbench.py
step ipc_test 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ipc_coll.py
step ipc_debug 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 scripts/ipc_debug.py
step b8_alone 400 python -u bench.py --mix 8mix --policies none,static-se,gpbs --reps 3 --out gpurun_out/b8_alone.json
