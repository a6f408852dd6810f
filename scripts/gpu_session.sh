#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s31}
for M in 8mix phase-ts phase 4mix; do
  timeout -k 10 300 python -u bench.py --mix $M --reps 3 --policies gpbs,atc,credit-fixed-ts30,gpbs-w \
    --out $O/${S}_$M.json > $O/${S}_$M.out 2> $O/${S}_$M.log || exit $?
done
