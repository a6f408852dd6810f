#!/bin/bash
# Round 4 session 12: GPU tests + the driver's default bench on the guarded tree.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/s12_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date +%T)"; tail -3 gpurun_out/r4/s12_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 600 python -u bench.py > gpurun_out/r4/s12_bench.json 2> gpurun_out/r4/s12_bench.log
echo "bench rc=$? $(date +%T)"; cat gpurun_out/r4/s12_bench.json | cut -c1-600
python scripts/corun_log_policies.py gpurun_out/r4/s12_bench.log | grep -v "^ "
