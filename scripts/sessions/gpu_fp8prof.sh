#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec2 -o dec -- python3 -u scripts/fp8_bench.py --skip-linear --variants fp8+graph --steps 200 > gpurun_out/fp8_prof_dec.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/fp8_prof_dec.log; exit 1; }
grep tok_per_s gpurun_out/fp8_prof_dec.log
timeout -k 10 600 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --policies solo,none,gpbs --out gpurun_out/llm_corun_fp8.json > gpurun_out/llm_corun_fp8.log 2>&1 || { echo "corun failed"; tail -30 gpurun_out/llm_corun_fp8.log; exit 1; }
tail -c 1500 gpurun_out/llm_corun_fp8.log
