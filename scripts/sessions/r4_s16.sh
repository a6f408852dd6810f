#!/bin/bash
# Round 4 session 16: cross-class steals off (boot class_steal=0, policy
# gpbs-nox / llm5 +nox) on the 8mix, the time-shared phase mix and config #5
# (with the reduced queue footprint: tenants GPU_MAX_HW_QUEUES=2, one masked
# queue per half).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
echo "== 8mix $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,gpbs-nox --reps 5 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s16_8mix.json 2> gpurun_out/r4/s16_8mix.log || exit $?
python scripts/corun_log_policies.py gpurun_out/r4/s16_8mix.log | grep -v "^   "
echo "== phase-ts $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --mix phase-ts --policies gpbs,gpbs-nox --reps 5 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s16_phasets.json 2> gpurun_out/r4/s16_phasets.log || exit $?
python scripts/corun_log_policies.py gpurun_out/r4/s16_phasets.log | grep -v "^   "
echo "== llm5 $(date +%T)"
timeout -k 10 900 python -u bench.py --mix llm5 --reps 3 --steps 50 --warmup 25 \
  --policies solo,static-se,gpbs-budget+hwq2+qp0,gpbs-budget+hwq2+qp0+nox --out gpurun_out/r4/s16_llm5_full.json \
  > gpurun_out/r4/s16_llm5.json 2> gpurun_out/r4/s16_llm5.log
echo "llm5 rc=$? $(date +%T)"; python -c "
import json; d=json.loads(open('gpurun_out/r4/s16_llm5.json').read().strip().splitlines()[-1])
for p, v in d['policies'].items(): print(p, v)"
