#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s34}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${S}_smoke.log 2>&1 &&
timeout -k 10 700 python -u bench.py --out $O/${S}_bench.json > $O/${S}_bench.out 2> $O/${S}_bench.log
