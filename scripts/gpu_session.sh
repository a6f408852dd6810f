#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s5}
timeout -k 10 120 python -u scripts/pipe_probe.py --queues 8 --ms 150 > $O/${S}_pipe_probe.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_se_hwc.py tests/test_gpu_phase.py tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread > $O/${S}_gputest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --mix 8mix --reps 3 --policies none,static-se,credit-classq,gpbs --out $O/${S}_8mix.json > $O/${S}_8mix.log 2>&1 &&
timeout -k 10 400 python -u bench.py --mix phase-ts --reps 3 --out $O/${S}_phasets.json > $O/${S}_phasets.log 2>&1
