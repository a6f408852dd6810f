#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s12}
timeout -k 10 300 python -u bench.py --mix phase-ts --reps 5 \
  --out $O/${S}_phasets.json > $O/${S}_phasets.out 2> $O/${S}_phasets.log &&
timeout -k 10 420 python -u bench.py --mix llm5 --reps 2 --policies static-se,static-se+ishift1,static-se+ishift2,static-se+ishift3,static-se+tshift1 \
  --out $O/${S}_llm5.json > $O/${S}_llm5.out 2> $O/${S}_llm5.log &&
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/${S}_bench.json > $O/${S}_bench.out 2> $O/${S}_bench.log
