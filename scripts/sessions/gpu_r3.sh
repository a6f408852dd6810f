#!/bin/bash
# Round-3 GPU session: each step under its own time limit; stop at the first
# fault / abort / timeout.  usage: scripts/gpu_r3.sh STEP...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LOG=gpurun_out/session.log
echo "session $(date) steps: $*" >> "$LOG"
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$LOG"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))" | tee -a "$LOG"
  tail -n 25 "gpurun_out/$name.log" | tee -a "$LOG"
  if [ $rc -ne 0 ] && { [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }; then
    echo "fatal rc=$rc in $name: stopping" | tee -a "$LOG"; exit $rc
  fi
  return $rc
}
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
for step in "$@"; do
  case $step in
    phase)   run phase 300 $PYT tests/test_gpu_phase.py -s || exit 1 ;;
    runtime) run runtime 400 $PYT tests/test_gpu_runtime.py -s || exit 1 ;;
    tests)   run tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests || exit 1 ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bquick)  run bquick 900 python -u bench.py --steps 10 --warmup 3 --reps 2 --reps-extra 2 \
                --out gpurun_out/bquick.json || exit 1 ;;
    bphase)  run bphase 900 python -u bench.py --mix phase --steps 20 --warmup 5 --reps 3 \
                --policies ${POLS:-none,static-se,credit-fixed,gpbs} --out gpurun_out/bphase.json || exit 1 ;;
    b8)      run b8 900 python -u bench.py --mix 8mix --steps 20 --warmup 5 --reps 3 \
                --policies ${POLS:-none,static-se,credit-fixed,gpbs} --out gpurun_out/b8.json || exit 1 ;;
    b4)      run b4 900 python -u bench.py --mix 4mix --steps 20 --warmup 5 --reps 3 \
                --policies ${POLS:-none,static-se,credit-fixed,gpbs,gpbs-se8} --out gpurun_out/b4.json || exit 1 ;;
    bench)   run bench 1100 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/bench.json || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
