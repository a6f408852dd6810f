#!/bin/bash
# Round 4 session 52: LDS-staged C (opts bit 16) vs the shipped own-A kernel,
# two kbench processes, then a rocprofv3 kernel trace of each alone.
set -o pipefail
cd "$(dirname "$0")/../.."
R=$(pwd)
mkdir -p gpurun_out/r4/kt52
export TMPDIR=/tmp
for i in 1 2; do
  KBENCH_GEMM_ONLY=1 timeout -k 10 300 python -u scripts/kbench.py --iters 30 > gpurun_out/r4/s52_kbench_$i.jsonl 2> gpurun_out/r4/s52_kbench_$i.log || exit $?
  grep -E '"ms"' gpurun_out/r4/s52_kbench_$i.jsonl | grep -v amdgpu.ids
done
for o in 8448 73984; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4/kt52/o$o -o o$o -- python3 $R/scripts/gemm_only.py 4096 $o \
    > gpurun_out/r4/kt52/o$o.log 2>&1 || exit $?
  echo "trace $o ok"
done
