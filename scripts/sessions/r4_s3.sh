#!/bin/bash
# Round 4 session 3: the attribution kernel (exactness, cost, rocprofv3
# kernel trace), the async-sampling probe, then the 8mix under sampler and
# quantum policies interleaved in one process (6 reps each, randomized order).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "hwc_attribute or two_pools" -s > gpurun_out/r4/s3_tests.log 2>&1
echo "tests rc=$?"; grep -E "k_hwc_attribute|passed|failed" gpurun_out/r4/s3_tests.log
echo "== rocprof attr $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_attr -o attr -- python3 scripts/attr_bench.py 500 \
  > gpurun_out/r4/s3_prof_attr.log 2>&1
echo "rocprof rc=$?"; tail -2 gpurun_out/r4/s3_prof_attr.log
echo "== async probe $(date +%T)"
timeout -k 10 200 python -u scripts/hwc_drift.py --variants async --segs 2 --load-s 5 --timeout 150 \
  --out gpurun_out/r4/s3_async.json > gpurun_out/r4/s3_async.log 2>&1
echo "async rc=$?"; tail -5 gpurun_out/r4/s3_async.log
echo "== 8mix sampler policies $(date +%T)"
timeout -k 10 800 python -u bench.py --gpus 1 --mix 8mix --reps 6 --steps 20 --warmup 3 \
  --policies none,credit-fixed-ts,credit-fixed-ts4,gpbs-model,gpbs-r3s,gpbs-b5,gpbs-f4,atc,gpbs \
  > gpurun_out/r4/s3_8mix_sampler.json 2> gpurun_out/r4/s3_8mix_sampler.log
echo "8mix rc=$? $(date +%T)"
