#!/bin/bash
# Round 4 session 39: the GPU suite on the last tree (incl. the CU-map test).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/s39_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4/s39_tests.log; grep -E "FAILED|cu_mask" gpurun_out/r4/s39_tests.log | head -5
