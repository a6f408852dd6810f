#!/bin/bash
# Round-3 GPU session y: the 8mix drift with the hardware sampler's bursts of 5 ms
# (1 % duty cap only): does it follow the number of samples?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GPBS_HWC_BURST_MS=5 timeout -k 10 600 python -u bench.py --mix 8mix --reps 5 --resolo --out gpurun_out/bench_8mix_z.json > gpurun_out/bench_8mix_z.log 2>&1
echo "bench8 rc=$?"
