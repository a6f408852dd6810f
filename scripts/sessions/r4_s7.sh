#!/bin/bash
# Round 4 session 7: config #5 through the bench contract (bench.py --mix
# llm5): solo, none, static-se, gpbs (daemon budget layout, live counters,
# shim queue choice remembered across runs) and gpbs with a reduced queue
# footprint (tenants GPU_MAX_HW_QUEUES=2, no queue prober), 3 reps.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
echo "== llm5 $(date +%T)"
timeout -k 10 1000 python -u bench.py --mix llm5 --reps 2 --steps 50 --warmup 25 \
  --policies solo,none,none+hwq2,static-se,gpbs-budget,gpbs-budget+hwq2+qp0 --out gpurun_out/r4/s7_llm5_full.json \
  > gpurun_out/r4/s7_llm5.json 2> gpurun_out/r4/s7_llm5.log
echo "llm5 rc=$? $(date +%T)"; tail -c 1500 gpurun_out/r4/s7_llm5.json
