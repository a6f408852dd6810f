#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s11}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_se_hwc.py tests/test_gpu_phase.py \
  > $O/${S}_gputest.log 2>&1 &&
timeout -k 10 420 python -u bench.py --mix 8mix --reps 5 --policies static-se,credit-fixed-ts,credit-classq,gpbs \
  --out $O/${S}_8mix.json > $O/${S}_8mix.out 2> $O/${S}_8mix.log &&
timeout -k 10 300 python -u bench.py --mix 4mix --reps 5 --policies static-se,credit-fixed,gpbs \
  --out $O/${S}_4mix.json > $O/${S}_4mix.out 2> $O/${S}_4mix.log
