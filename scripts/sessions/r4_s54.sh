#!/bin/bash
# Round 4 session 54: LDS-staged C with non-temporal full-line stores
# (opts bit 17): numerics against fp32 first, then the kbench GEMM rows.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm256_variants" -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4/s54_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4/s54_tests.log; [ $rc -eq 0 ] || exit $rc
KBENCH_GEMM_ONLY=1 timeout -k 10 400 python -u scripts/kbench.py --iters 30 > gpurun_out/r4/s54_kbench.jsonl 2> gpurun_out/r4/s54_kbench.log
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/r4/s54_kbench.jsonl
exit $rc
