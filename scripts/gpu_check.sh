#!/bin/bash
# One GPU-box pass: gpu tests, smoke, default bench. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed: $?"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -3 gpurun_out/bench_default.log
