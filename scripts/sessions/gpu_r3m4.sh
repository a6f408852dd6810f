#!/bin/bash
# Round-3: the 4mix with modeled counters and the solo re-measure (does the
# late step of the partitioned policies follow the device-counting service?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --mix 4mix --counters model --resolo --reps 6 --out gpurun_out/bench_4mix_model.json > gpurun_out/bench_4mix_model.log 2>&1
echo "bench4 rc=$?"
