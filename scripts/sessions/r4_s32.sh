#!/bin/bash
# Round 4 session 32: 8mix gpbs x 12 with each runner's masked-queue index
# per run (does a slow run use a different queue set?).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u bench.py --gpus 1 --mix 8mix --policies gpbs,atc --reps 8 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s32_8mix.json 2> gpurun_out/r4/s32_8mix.log
echo "rc=$?"
python - <<'PY'
import json
for ln in open("gpurun_out/r4/s32_8mix.log"):
    i = ln.find(': {"policy"')
    if i < 0:
        continue
    r = json.loads(ln[i + 2:])
    q = {n: d.get("queue") for n, d in r["engine"]["runner"].items()}
    print(r["policy"], round(r["aggregate"], 3), q)
PY
