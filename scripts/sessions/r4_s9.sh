#!/bin/bash
# Round 4 session 9: are the slow 8mix runs host-starved?  gpbs + none x 8
# with per-run host CPU / context-switch / cgroup-throttle records, runners
# spinning (default) vs sleeping 20 us between completion polls.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
run() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 240 env "$@" > gpurun_out/r4/s9_$name.json 2> gpurun_out/r4/s9_$name.log
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  python scripts/corun_log_policies.py gpurun_out/r4/s9_$name.log | grep -v "^ "
  python - gpurun_out/r4/s9_$name.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('[corun] ') and ': {"policy"' in l:
        r = json.loads(l[l.index('{'):])
        print(r['policy'], round(r['aggregate'], 3), r.get('host'))
PY
  return $rc
}
B="python -u bench.py --gpus 1 --mix 8mix --policies none,gpbs --reps 8 --steps 20 --warmup 3"
run spin GPBS_X=0 $B && \
run poll20 GPBS_RUNNER_POLL_US=20 $B
