#!/bin/bash
# Config #5 (Llama-3-8B fp8 decode + Llama-1B bf16 trainer, 1x MI355X), 5 reps
# of none / static-se / gpbs-se (live hardware counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 5 --warmup 2 --reps ${REPS:-5} \
  --policies solo,none,static-se,gpbs-se --out gpurun_out/config5_r3_5rep.json > gpurun_out/config5_r3_5rep.log 2>&1
echo "config5 rc=$?"
