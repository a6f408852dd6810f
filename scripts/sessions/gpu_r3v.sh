#!/bin/bash
# Round-3 GPU session v: counting-context restart every 1000 samples -- hwc
# GPU tests, then the 8mix alone with hw counters and the solo re-measure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hwc.py tests/test_gpu_se_hwc.py tests/test_gpu_phase.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hwc_tests_v.log 2>&1
rc=$?; echo "hwc tests rc=$rc"; case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 600 python -u bench.py --mix 8mix --reps 5 --resolo --out gpurun_out/bench_8mix_v.json > gpurun_out/bench_8mix_v.log 2>&1
echo "bench8 rc=$?"
