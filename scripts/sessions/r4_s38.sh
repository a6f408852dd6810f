#!/bin/bash
# Round 4 session 38: a process-wide budget of masked queues
# (GPBS_MASKED_MAX 0 = none / 6 / 5) on the 8mix, one process each, same box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for mx in 0 6 5; do
  echo "== masked_max=$mx $(date +%T)"
  GPBS_MASKED_MAX=$mx timeout -k 10 400 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,credit-fixed-ts --reps 6 \
    --steps 20 --warmup 3 --no-resolo --no-cu-check > gpurun_out/r4/s38_mx$mx.json 2> gpurun_out/r4/s38_mx$mx.log || exit $?
  MX=$mx python - <<'PY'
import json, os
mx = os.environ["MX"]
for ln in open(f"gpurun_out/r4/s38_mx{mx}.log"):
    i = ln.find(': {"policy"')
    if i < 0:
        continue
    r = json.loads(ln[i + 2:])
    e = r["engine"]
    q = {n: d.get("queue") for n, d in e["runner"].items()}
    print(r["policy"], round(r["aggregate"], 3), q, e["gpu"].get("masked_queues_created"))
PY
done
