#!/bin/bash
# Round 4 session 48: GEMM priority variants (no per-segment s_setprio flips
# / MFMA segments at priority 3) next to the shipped own-A kernel, one process.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
KBENCH_GEMM_ONLY=1 timeout -k 10 300 python -u scripts/kbench.py --iters 30 > gpurun_out/r4/s48_kbench.jsonl 2>&1 || exit $?
grep -v "amdgpu.ids" gpurun_out/r4/s48_kbench.jsonl
