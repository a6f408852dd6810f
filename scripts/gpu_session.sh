#!/bin/bash
# One GPU session (gpurun): each GPU step under its own time limit, chained
# with && so the first failure ends the session.  Overwritten per session;
# the commit history holds the earlier ones.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
S=${1:-s36}
# 8-rank --rehearse-ipc of the headline mix on one GPU (every rank on cuda:0), final tree
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 \
  bench.py --gpus 8 --mix 4mix --steps 3 --warmup 1 --reps 1 --rehearse-ipc --policies none,gpbs --hang-dump-s 120 \
  --out $O/${S}_rehearse8.json > $O/${S}_rehearse8.out 2> $O/${S}_rehearse8.log
