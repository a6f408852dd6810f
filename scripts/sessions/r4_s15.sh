#!/bin/bash
# Round 4 session 15: k_hwc_attribute with 8-lane partition totals
# (exactness incl. the new slot layouts / idle XCDs, cost, rocprofv3); the
# time-shared phase mix; the 8-rank --rehearse-ipc pre-flight record on one GPU.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== attr tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "hwc_attribute or two_pools or hwc_attr" -s > gpurun_out/r4/s15_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "k_hwc_attribute|passed|failed|Error|assert" gpurun_out/r4/s15_tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== rocprof attr $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_attr15 -o attr -- python3 scripts/attr_bench.py 500 \
  > gpurun_out/r4/s15_prof_attr.log 2>&1 || exit $?
grep rc= gpurun_out/r4/s15_prof_attr.log
python scripts/rocpd_summary.py gpurun_out/r4/prof_attr15/attr_results.db -o gpurun_out/r4/s15_attr_summary.txt | head -5
echo "== phase-ts $(date +%T)"
timeout -k 10 400 python -u bench.py --gpus 1 --mix phase-ts --policies gpbs,credit-fixed-ts,none,static-se --reps 5 \
  --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s15_phasets.json 2> gpurun_out/r4/s15_phasets.log || exit $?
python scripts/corun_log_policies.py gpurun_out/r4/s15_phasets.log
echo "== rehearse8 $(date +%T)"
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 8 --rehearse-ipc --mix 4mix --policies gpbs,none --reps 1 --steps 5 --warmup 1 --counters model \
  --no-resolo > gpurun_out/r4/s15_rehearse8.json 2> gpurun_out/r4/s15_rehearse8.log
echo "rehearse rc=$? $(date +%T)"; tail -c 1200 gpurun_out/r4/s15_rehearse8.json
