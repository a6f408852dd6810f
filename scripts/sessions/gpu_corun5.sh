#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --policies solo,none,gpbs,gpbs+prio,gpbs-spatial --out gpurun_out/llm_corun_fp8_v3.json > gpurun_out/llm_corun_fp8_v3.log 2>&1 || { echo "corun failed"; tail -30 gpurun_out/llm_corun_fp8_v3.log; exit 1; }
echo done
