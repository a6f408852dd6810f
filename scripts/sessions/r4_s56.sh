#!/bin/bash
# Round 4 session 56: the GEMM default with non-temporal LDS-staged C stores: smoke(),
# the GPU suite, then the driver's default bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4/s56_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r4/s56_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/s56_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4/s56_tests.log; grep -E "FAILED" gpurun_out/r4/s56_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r4/s56_bench.json 2> gpurun_out/r4/s56_bench.log
rc=$?; echo "bench rc=$rc $(date +%T)"
python scripts/corun_log_policies.py gpurun_out/r4/s56_bench.log | grep -v "^  "
python -c "
import json; d=json.loads(open('gpurun_out/r4/s56_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['gpbs_vs_static_se'])"
exit $rc
