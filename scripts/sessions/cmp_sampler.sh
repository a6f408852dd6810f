#!/bin/bash
# Sampler-cost A/B on the 4-tenant mix, one box: the same bench under
# several counter sets / periods, and with no sampler (modeled counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
POLS=${POLS:-none,static-se,gpbs}
run() {  # run NAME [ENV=VAL ...] -- [bench args]
  local name=$1; shift
  local envs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  echo "== $name"
  timeout -k 10 300 env "${envs[@]}" python -u bench.py --mix ${MIX:-4mix} --steps 20 --warmup 5 --reps ${REPS:-3} \
    --policies $POLS --out gpurun_out/cmp_${MIX:-4mix}_$name.json "$@" > gpurun_out/cmp_${MIX:-4mix}_$name.log 2>&1 || exit 1
}
for v in ${VARIANTS:-lean1ms lean4ms lean2 model}; do
  case $v in
    lean1ms) run lean1ms GPBS_HWC_SPEC=lean GPBS_HWC_DUTY=0 ;;
    lean2_1ms) run lean2_1ms GPBS_HWC_SPEC=lean2 GPBS_HWC_DUTY=0 ;;
    default) run default ;;
    lean4ms) run lean4ms GPBS_HWC_SPEC=lean GPBS_HWC_PERIOD_US=4000 GPBS_HWC_DUTY=0 ;;
    lean2)   run lean2 GPBS_HWC_SPEC=lean2 GPBS_HWC_DUTY=0 ;;
    full1ms) run full1ms GPBS_HWC_SPEC=full ;;
    nowatch) run nowatch GPBS_HWC_WATCH=0 ;;
    duty2)   run duty2 GPBS_HWC_DUTY=2 ;;
    noburst) run noburst GPBS_HWC_BURST_MS=0 ;;
    model)   run model GPBS_HWC_SPEC=lean -- --counters model ;;
  esac
done
