#!/bin/bash
# Round 4 session 19: the default bench's every mix (4mix, phase, phase-ts,
# 8mix) through the multi-rank path: 4 ranks on one GPU (--rehearse-ipc,
# modeled counters), 1 rep each.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
echo "== rehearse4 all mixes $(date +%T)"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 4 --rehearse-ipc --steps 5 --warmup 1 --reps 1 --reps-extra 1 --counters model \
  > gpurun_out/r4/s19_rehearse4.json 2> gpurun_out/r4/s19_rehearse4.log
echo "rc=$? $(date +%T)"; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r4/s19_rehearse4.json') if l.startswith('{')][-1]
print('value', d['value'], 'n_gpus', d['n_gpus'], 'mixes', {m: v.get('value') for m, v in d.get('mixes', {}).items()})
for r in d['ranks']: print(r['rank'], {m: (x['coll'], x['ipc_selftest'], (x.get('gang') or {}).get('timeouts')) for m, x in r['mixes'].items()})"
