#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s8}
timeout -k 10 300 python -u bench.py --mix 4mix --reps 5 --policies static-se,gpbs,gpbs-model,gpbs-noalign \
  --out $O/${S}_4mix_ab.json > $O/${S}_4mix_ab.out 2> $O/${S}_4mix_ab.log &&
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/${S}_bench.json > $O/${S}_bench.out 2> $O/${S}_bench.log
