#!/bin/bash
# Round 4 session 36: final-tree validation (with the CU-map preflight) -- smoke(), the GPU suite, the
# driver's default bench (now 4mix + phase + phase-ts + 8mix).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4/s36_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r4/s36_smoke.log
[ $rc -eq 0 ] || exit $rc
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/s36_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date +%T)"; tail -3 gpurun_out/r4/s36_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 900 python -u bench.py > gpurun_out/r4/s36_bench.json 2> gpurun_out/r4/s36_bench.log
echo "bench rc=$? $(date +%T)"
python scripts/corun_log_policies.py gpurun_out/r4/s36_bench.log | grep -v "^  "
python -c "
import json; d=json.loads(open('gpurun_out/r4/s36_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['gpbs_vs_static_se'], [r.get('cu_map_ok') for r in d['ranks']])"
