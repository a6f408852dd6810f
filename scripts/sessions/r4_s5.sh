#!/bin/bash
# Round 4 session 5: attribution kernel (exactness, cost, rocprofv3 trace),
# then the queue-budget probe (solo GEMM rate vs CU-masked queues held by the
# process), without and with the device-counting context.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "hwc_attribute or two_pools" -s > gpurun_out/r4/s5_tests.log 2>&1
echo "tests rc=$?"; grep -E "k_hwc_attribute|passed|failed" gpurun_out/r4/s5_tests.log
echo "== rocprof attr $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_attr5 -o attr -- python3 scripts/attr_bench.py 500 \
  > gpurun_out/r4/s5_prof_attr.log 2>&1
echo "rocprof rc=$?"; grep rc= gpurun_out/r4/s5_prof_attr.log
echo "== queue budget, no counters $(date +%T)"
timeout -k 10 240 python -u scripts/queue_budget.py --step 4 --max 48 > gpurun_out/r4/s5_qbudget.log 2>&1
echo "qb rc=$?"; grep -v RESULT gpurun_out/r4/s5_qbudget.log | tail -14
echo "== queue budget, counters $(date +%T)"
timeout -k 10 240 python -u scripts/queue_budget.py --counters --step 4 --max 48 > gpurun_out/r4/s5_qbudget_hwc.log 2>&1
echo "qb hwc rc=$?"; grep -v RESULT gpurun_out/r4/s5_qbudget_hwc.log | tail -14
bash scripts/sessions/r4_s6.sh
