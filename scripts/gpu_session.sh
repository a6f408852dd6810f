#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s13}
timeout -k 10 120 python -u bench.py --mix 8mix --reps 1 --policies gpbs --kernel-trace \
  --out $O/${S}_8mix_ktrace.json > $O/${S}_8mix_ktrace.out 2> $O/${S}_8mix_ktrace.log &&
timeout -k 10 300 python -u bench.py --mix phase-ts --reps 5 \
  --out $O/${S}_phasets.json > $O/${S}_phasets.out 2> $O/${S}_phasets.log &&
KBENCH_GEMM_ONLY=1 timeout -k 10 120 python -u scripts/kbench.py > $O/${S}_kbench.jsonl 2> $O/${S}_kbench.log &&
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/${S}_bench.json > $O/${S}_bench.out 2> $O/${S}_bench.log
