#!/bin/bash
# Full GPU pass: every gpu test, smoke, profile of the fp8 graph decode, fp8 LLM co-run, headline bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec3 -o dec -- python3 -u scripts/fp8_bench.py --skip-linear --variants fp8+graph --steps 200 > gpurun_out/fp8_prof_dec.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/fp8_prof_dec.log; exit 1; }
timeout -k 10 600 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --policies solo,none,gpbs --out gpurun_out/llm_corun_fp8.json > gpurun_out/llm_corun_fp8.log 2>&1 || { echo "corun failed"; tail -30 gpurun_out/llm_corun_fp8.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
