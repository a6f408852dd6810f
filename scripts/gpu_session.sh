#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s16}
timeout -k 10 180 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm256_variants and 262144" > $O/${S}_gemmp_test.log 2>&1 &&
KBENCH_GEMM_ONLY=1 timeout -k 10 120 python -u scripts/kbench.py > $O/${S}_kbench.jsonl 2> $O/${S}_kbench.log
