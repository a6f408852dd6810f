#!/bin/bash
# Round 4 session 33: 8mix gpbs x 10 with and without the interleaved
# class-half queue preallocation (GPBS_QUEUE_PREALLOC), one process each.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for pre in 0 1; do
  echo "== prealloc=$pre $(date +%T)"
  GPBS_QUEUE_PREALLOC=$pre timeout -k 10 400 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,atc --reps 8 \
    --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s33_8mix_pre$pre.json 2> gpurun_out/r4/s33_8mix_pre$pre.log || exit $?
  PRE=$pre python - <<'PY'
import json, os
pre = os.environ["PRE"]
for ln in open(f"gpurun_out/r4/s33_8mix_pre{pre}.log"):
    i = ln.find(': {"policy"')
    if i < 0:
        continue
    r = json.loads(ln[i + 2:])
    if r["policy"] != "gpbs":
        continue
    q = {n: d.get("queue") for n, d in r["engine"]["runner"].items()}
    print(r["policy"], round(r["aggregate"], 3), q)
PY
done
