#!/bin/bash
# Round 4 session 45: config #5 over 5 reps on the final tree (12 HIP queues
# per process, class-half probe, 5 s warm-up).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
echo "== llm5 x5 $(date +%T)"
timeout -k 10 900 python -u bench.py --mix llm5 --reps 5 --steps 50 --warmup 25 \
  --policies solo,none,static-se,gpbs-budget --out gpurun_out/r4/s45_llm5_full.json \
  > gpurun_out/r4/s45_llm5.json 2> gpurun_out/r4/s45_llm5.log
echo "llm5 rc=$? $(date +%T)"; python -c "
import json; d=json.loads(open('gpurun_out/r4/s45_llm5.json').read().strip().splitlines()[-1])
for p, v in d['policies'].items(): print(p, v)
print(d.get('gpbs_vs_static_se'))"
