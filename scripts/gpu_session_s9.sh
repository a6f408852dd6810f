#!/bin/bash
# GPU session: 8-rank --rehearse-ipc of the headline mix on one GPU (every
# rank on cuda:0; the whole N > 1 control path, the compact line at N = 8).
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 \
  bench.py --gpus 8 --mix 4mix --steps 3 --warmup 1 --reps 1 --rehearse-ipc --policies none,gpbs --hang-dump-s 120 \
  --out $O/s9_rehearse8.json > $O/s9_rehearse8.out 2> $O/s9_rehearse8.log
