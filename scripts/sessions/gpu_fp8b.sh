#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8_tests.log 2>&1 || { echo "fp8 tests failed"; tail -60 gpurun_out/fp8_tests.log; exit 1; }
tail -2 gpurun_out/fp8_tests.log
rm -f gpurun_out/fp8_bench_var.jsonl
timeout -k 10 300 python -u scripts/fp8_bench.py --skip-linear --variants fp8+graph --steps 20 --out gpurun_out/fp8_bench_var.jsonl > gpurun_out/fp8_bench_var.log 2>&1 && timeout -k 10 300 python -u scripts/fp8_bench.py --skip-linear --variants fp8+graph --steps 200 --out gpurun_out/fp8_bench_var.jsonl >> gpurun_out/fp8_bench_var.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/fp8_bench_var.log; exit 1; }
cat gpurun_out/fp8_bench_var.jsonl
