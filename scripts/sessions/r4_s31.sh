#!/bin/bash
# Round 4 session 31: rocprofv3 kernel traces of the final tree's 8mix and
# 4mix gpbs co-runs (modeled counters: the process cannot open its own
# counting context under rocprofv3).  Last steps of the call: rocprofv3 has
# crashed in its own teardown after writing the database before.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== rocprof 8mix $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_8mix31 -o corun -- python3 bench.py --gpus 1 \
  --mix 8mix --policies gpbs --reps 1 --steps 10 --warmup 2 --no-resolo --counters model > gpurun_out/r4/s31_prof_8mix.log 2>&1
echo "rocprof rc=$?"
python scripts/rocpd_summary.py gpurun_out/r4/prof_8mix31/corun_results.db -o gpurun_out/r4/s31_8mix_summary.txt | head -16
