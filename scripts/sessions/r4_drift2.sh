#!/bin/bash
# Round 4: where does the live-counter drift come from?  8mix, gpbs only,
# 12 reps, solo rates re-measured after the runs (--resolo), per variant:
#   A round-3 sampler (owner-change bursts, no budget, no model fallback)
#   D round-4 defaults (2 % sample budget, no owner bursts, model fallback)
#   B round-3 sampler with host attribution (no k_hwc_attribute launches)
#   C modeled counters.  GPU state per run rides the JSON.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
run() {  # name, env..., -- args
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 240 env "$@" > gpurun_out/r4/drift2_$name.json 2> gpurun_out/r4/drift2_$name.log
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  tail -c 300 gpurun_out/r4/drift2_$name.json; echo
  return $rc
}
B="python -u bench.py --gpus 1 --mix 8mix --policies gpbs --reps 12 --resolo --steps 20 --warmup 3"
R3="GPBS_HWC_OWNER_BURST=1 GPBS_HWC_BUDGET=0 GPBS_HWC_MODEL_FALLBACK=0"
run A_r3 $R3 $B && \
run D_new GPBS_X=0 $B && \
run B_hostattr $R3 GPBS_HWC_DEVICE=0 $B && \
run C_model GPBS_X=0 $B --counters model
