#!/bin/bash
# Round-3 GPU session u: the 8mix drift with modeled counters (is it the
# hardware-counter sampler?), solo rates re-measured after the runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --mix 8mix --reps 5 --resolo --counters model --out gpurun_out/bench_8mix_u.json > gpurun_out/bench_8mix_u.log 2>&1
echo "bench8 rc=$?"
