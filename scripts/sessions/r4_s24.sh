#!/bin/bash
# Round 4 session 24: the GPU suite on the back-off default, then config #5
# over 5 reps through the bench contract.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4/s24_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date +%T)"; tail -3 gpurun_out/r4/s24_tests.log; grep -E "FAILED|Error" gpurun_out/r4/s24_tests.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== llm5 x5 $(date +%T)"
timeout -k 10 900 python -u bench.py --mix llm5 --reps 5 --steps 50 --warmup 25 \
  --policies solo,none,static-se,gpbs-budget --out gpurun_out/r4/s24_llm5_full.json \
  > gpurun_out/r4/s24_llm5.json 2> gpurun_out/r4/s24_llm5.log
echo "llm5 rc=$? $(date +%T)"; python -c "
import json; d=json.loads(open('gpurun_out/r4/s24_llm5.json').read().strip().splitlines()[-1])
for p, v in d['policies'].items(): print(p, v)
print(d.get('gpbs_vs_static_se'))"
