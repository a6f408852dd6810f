#!/bin/bash
# Config #5 round 3 g: is the collapse the daemon's hardware-counter sampling
# (+nohwc: daemon on modeled counters) or the layout history (static split
# that starts on swapped halves for 1.5 s, no daemon)?  4 reps each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 4 --warmup 2 --reps ${REPS:-4} \
  --policies solo,static-se,static-se+swap1.5,gpbs-se,gpbs-se+nohwc \
  --out gpurun_out/config5_r3g.json > gpurun_out/config5_r3g.log 2>&1
echo "config5g rc=$?"
