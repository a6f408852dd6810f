#!/bin/bash
# fp8 path on the GPU box: numerics tests, microbench, rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fp8.py tests/test_llama.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8_tests.log 2>&1 || { echo "fp8 tests failed"; tail -60 gpurun_out/fp8_tests.log; exit 1; }
tail -4 gpurun_out/fp8_tests.log
rm -f gpurun_out/fp8_bench.jsonl
timeout -k 10 400 python -u scripts/fp8_bench.py --out gpurun_out/fp8_bench.jsonl > gpurun_out/fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/fp8_bench.log; exit 1; }
cat gpurun_out/fp8_bench.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp8 -o fp8 -- python3 -u scripts/fp8_bench.py --skip-model --iters 20 > gpurun_out/fp8_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/fp8_prof.log; exit 1; }
find gpurun_out/prof_fp8 -name '*stats*' | head
