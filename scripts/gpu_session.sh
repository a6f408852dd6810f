#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s29}
timeout -k 10 300 python -u bench.py --mix 8mix --reps 3 --policies atc,atc-nox,gpbs,gpbs-nox \
  --out $O/${S}_8mix.json > $O/${S}_8mix.out 2> $O/${S}_8mix.log &&
timeout -k 10 300 python -u bench.py --mix 4mix --reps 3 --policies atc,atc-nox,gpbs \
  --out $O/${S}_4mix.json > $O/${S}_4mix.out 2> $O/${S}_4mix.log
