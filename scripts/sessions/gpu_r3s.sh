#!/bin/bash
# Round-3 GPU session s: the driver's bench command on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/bench_driver_s.json > gpurun_out/bench_driver_s.log 2>&1
echo "bench rc=$?"
