#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s37}
timeout -k 10 900 python -u bench.py --mix llm5 --reps 5 --out $O/${S}_llm5.json > $O/${S}_llm5.out 2> $O/${S}_llm5.log
