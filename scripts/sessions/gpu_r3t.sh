#!/bin/bash
# Round-3 GPU session t: is the 8mix drift within the mix (fresh process, 8mix
# only) and do the solo rates drift with it (re-measured after the runs)?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --mix 8mix --reps 5 --resolo --out gpurun_out/bench_8mix_t.json > gpurun_out/bench_8mix_t.log 2>&1
echo "bench8 rc=$?"
