#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s21}
# GEMM tile-to-XCD mapping A/B under co-run: default (205056) vs + 2-D XCD blocks (bit 3), separate processes
timeout -k 10 240 python -u bench.py --mix 4mix --reps 5 --policies static-se,gpbs --out $O/${S}_4mix_def.json > $O/${S}_4mix_def.out 2> $O/${S}_4mix_def.log &&
timeout -k 10 240 python -u bench.py --mix 4mix --reps 5 --policies static-se,gpbs --gemm-opts 205064 --out $O/${S}_4mix_2d.json > $O/${S}_4mix_2d.out 2> $O/${S}_4mix_2d.log &&
timeout -k 10 300 python -u bench.py --mix 8mix --reps 5 --policies credit-classq,gpbs --out $O/${S}_8mix_def.json > $O/${S}_8mix_def.out 2> $O/${S}_8mix_def.log &&
timeout -k 10 300 python -u bench.py --mix 8mix --reps 5 --policies credit-classq,gpbs --gemm-opts 205064 --out $O/${S}_8mix_2d.json > $O/${S}_8mix_2d.out 2> $O/${S}_8mix_2d.log
