#!/bin/bash
# One GPU-box session: each step has its own time limit; a fault, abort,
# segfault or timeout stops the session (no further GPU work).
# usage: scripts/gpu_session.sh STEP... where STEP is one of
#   warm | tests | smoke | bench | bench8 | prof | census
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LOG=gpurun_out/session.log
echo "session start $(date) steps: $*" > "$LOG"

run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))" | tee -a "$LOG"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))" | tee -a "$LOG"
  tail -n 30 "gpurun_out/$name.log" >> "$LOG"
  case $rc in
    124|134|137|139) echo "fatal rc=$rc in $name: stopping session" | tee -a "$LOG"; exit $rc ;;
  esac
  if [ $rc -ge 128 ]; then echo "signal rc=$rc in $name: stopping" | tee -a "$LOG"; exit $rc; fi
  return 0
}

for step in "$@"; do
  case $step in
    warm)   run warm 400 python -c "import torch; print(torch.__version__, torch.cuda.get_device_name(0))" ;;
    tests)  run tests 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider ;;
    kbench) run kbench 300 python scripts/kbench.py ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps 10 --warmup 2 --out gpurun_out/bench_detail.json ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --policies gpbs ;;
    *)      echo "unknown step $step" | tee -a "$LOG" ;;
  esac
done
echo "session done $(date)" | tee -a "$LOG"
