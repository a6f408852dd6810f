#!/bin/bash
# Round 4 session 17: config #5 again with the counter service up for every
# gpbs-budget variant (session 16 ran the '+' variants without counters);
# then 8mix gpbs x 6 with per-run trace rings (a slow-mode episode in s16).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4/diag17
export PYTHONUNBUFFERED=1
echo "== llm5 $(date +%T)"
timeout -k 10 900 python -u bench.py --mix llm5 --reps 3 --steps 50 --warmup 25 \
  --policies solo,static-se,gpbs-budget,gpbs-budget+hwq2+qp0,gpbs-budget+hwq2+qp0+nox --out gpurun_out/r4/s17_llm5_full.json \
  > gpurun_out/r4/s17_llm5.json 2> gpurun_out/r4/s17_llm5.log || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/r4/s17_llm5.json').read().strip().splitlines()[-1])
for p, v in d['policies'].items(): print(p, v)"
echo "== 8mix traces $(date +%T)"
GPBS_DIAG_DIR=gpurun_out/r4/diag17 timeout -k 10 300 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,none --reps 6 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s17_8mix.json 2> gpurun_out/r4/s17_8mix.log
echo "rc=$? $(date +%T)"; python scripts/corun_log_policies.py gpurun_out/r4/s17_8mix.log | grep -v "^   "
