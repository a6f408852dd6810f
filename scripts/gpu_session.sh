#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s10}
timeout -k 10 420 python -u bench.py --mix 8mix --reps 5 --policies none,static-se,gpbs-split,credit-fixed-ts,credit-classq,gpbs \
  --out $O/${S}_8mix.json > $O/${S}_8mix.out 2> $O/${S}_8mix.log &&
timeout -k 10 300 python -u bench.py --mix phase-ts --reps 5 \
  --out $O/${S}_phasets.json > $O/${S}_phasets.out 2> $O/${S}_phasets.log
