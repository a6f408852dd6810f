#!/bin/bash
# Round 4 session 14: k_hwc_attribute with the lane-independent work hoisted
# (exactness vs the host twin, own-stamp cost, rocprofv3 trace), then config
# #5 through the bench contract (session 7's policy set).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== attr tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "hwc_attribute or two_pools or hwc_attr" -s > gpurun_out/r4/s14_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "k_hwc_attribute|passed|failed|Error" gpurun_out/r4/s14_tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== rocprof attr $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_attr14 -o attr -- python3 scripts/attr_bench.py 500 \
  > gpurun_out/r4/s14_prof_attr.log 2>&1 || exit $?
grep rc= gpurun_out/r4/s14_prof_attr.log
python scripts/rocpd_summary.py gpurun_out/r4/prof_attr14/attr_results.db -o gpurun_out/r4/s14_attr_summary.txt | head -5
bash scripts/sessions/r4_s7.sh
