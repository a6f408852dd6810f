#!/bin/bash
# Round-3 GPU session x: the driver's bench command on the final tree (context
# restarts off again), then smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --resolo --out gpurun_out/bench_driver_x.json > gpurun_out/bench_driver_x.log 2>&1
rc=$?; echo "bench rc=$rc"; case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_x.log 2>&1
echo "smoke rc=$?"
