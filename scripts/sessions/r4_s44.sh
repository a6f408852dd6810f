#!/bin/bash
# Round 4 session 44: smoke() and the GPU suite with 12 HIP queues by default.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4/s44_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r4/s44_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/s44_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4/s44_tests.log; grep -E "FAILED" gpurun_out/r4/s44_tests.log | head -5
