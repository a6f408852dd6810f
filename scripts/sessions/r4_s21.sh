#!/bin/bash
# Round 4 session 21: queues per layout key (GPBS_KEY_QUEUES 1 vs 2) on the
# time-shared mixes, same box, one process per setting.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
for q in 1 2; do
  for mix in phase-ts 8mix; do
    echo "== $mix Q=$q $(date +%T)"
    GPBS_KEY_QUEUES=$q timeout -k 10 300 python -u bench.py --gpus 1 --mix $mix --policies gpbs,credit-fixed-ts --reps 5 \
      --steps 20 --warmup 3 --no-resolo > gpurun_out/r4/s21_${mix}_q$q.json 2> gpurun_out/r4/s21_${mix}_q$q.log || exit $?
    python scripts/corun_log_policies.py gpurun_out/r4/s21_${mix}_q$q.log | grep -v "^   "
    grep -o '"masked_queues_created": [0-9]*' gpurun_out/r4/s21_${mix}_q$q.log | sort | uniq -c | tail -2
  done
done
