#!/bin/bash
# Round 4 session 22: config #5, the daemon's counter sampler backing off to
# 50 ms once the layout has not changed for 20 ms (GPBS_HWC_SLOW_US=50000)
# vs the default cadence, same box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
for slow in 0 50000; do
  echo "== llm5 slow_us=$slow $(date +%T)"
  GPBS_HWC_SLOW_US=$slow timeout -k 10 700 python -u bench.py --mix llm5 --reps 3 --steps 50 --warmup 25 \
    --policies solo,static-se,gpbs-budget --out gpurun_out/r4/s22_llm5_slow${slow}_full.json \
    > gpurun_out/r4/s22_llm5_slow$slow.json 2> gpurun_out/r4/s22_llm5_slow$slow.log || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/r4/s22_llm5_slow$slow.json').read().strip().splitlines()[-1])
for p, v in d['policies'].items(): print(p, v)"
done
