#!/bin/bash
# Round 4 session 55: LDS-staged C with vs without non-temporal stores, two
# more kbench processes (GEMM rows only).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for i in 1 2; do
  KBENCH_GEMM_ONLY=1 timeout -k 10 300 python -u scripts/kbench.py --iters 30 > gpurun_out/r4/s55_kbench_$i.jsonl 2> gpurun_out/r4/s55_kbench_$i.log || exit $?
  grep -E '"ms"' gpurun_out/r4/s55_kbench_$i.jsonl | grep -E "own-a|torch"
done
