#!/bin/bash
# Round 4 session 6: what makes the default-sampler gpbs runs bimodal?  8mix,
# gpbs only, 8 reps per variant, one process each:
#   V1 defaults; V2 no 1 ms modeled-block copy (GPBS_HWC_WATCH=0);
#   V3 host-written VRAM partition table (no k_partition_switch dispatch);
#   V4 modeled counters.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
run() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 200 env "$@" > gpurun_out/r4/s6_$name.json 2> gpurun_out/r4/s6_$name.log
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  python scripts/corun_log_policies.py gpurun_out/r4/s6_$name.log | head -2
  return $rc
}
B="python -u bench.py --gpus 1 --mix 8mix --policies gpbs --reps 8 --steps 20 --warmup 3"
run V1_default GPBS_X=0 $B && \
run V2_nowatch GPBS_HWC_WATCH=0 $B && \
run V3_bar GPBS_TABLE_MODE=bar $B && \
run V4_model GPBS_X=0 $B --counters model
