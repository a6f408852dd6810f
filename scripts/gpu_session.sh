#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s25}
timeout -k 10 360 python -u bench.py --mix phase-ts --reps 5 --policies credit-fixed-ts,gpbs,gpbs-dwell50,gpbs-dwell150 \
  --out $O/${S}_phasets.json > $O/${S}_phasets.out 2> $O/${S}_phasets.log &&
timeout -k 10 360 python -u bench.py --mix phase --reps 5 --policies credit-fixed,gpbs,gpbs-dwell50,gpbs-dwell150,static-se \
  --out $O/${S}_phase.json > $O/${S}_phase.out 2> $O/${S}_phase.log
