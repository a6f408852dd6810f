#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec -o dec -- python3 -u scripts/fp8_bench.py --skip-linear --variants fp8+graph --steps 20 > gpurun_out/fp8_prof_dec.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/fp8_prof_dec.log; exit 1; }
tail -3 gpurun_out/fp8_prof_dec.log
find gpurun_out/prof_dec | head
