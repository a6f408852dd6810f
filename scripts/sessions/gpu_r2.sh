#!/bin/bash
# Round-2 GPU session: each step under its own time limit; stop at the first
# fault / abort / timeout.  usage: scripts/gpu_r2.sh STEP...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LOG=gpurun_out/session.log
echo "session $(date) steps: $*" > "$LOG"
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
  return 0
}
for step in "$@"; do
  case $step in
    se)      run se 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_se_hwc.py -s ;;
    tests)   run tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bquick)  run bquick 600 python bench.py --steps 10 --warmup 2 --reps 2 --out gpurun_out/bquick.json ;;
    bench)   run bench 900 python bench.py --steps 20 --warmup 5 --out gpurun_out/bench.json ;;
    bclean0) GPBS_HWC_CLEAN=0 run bclean0 600 python bench.py --steps 20 --warmup 5 --reps 3 \
                --policies none,gpbs-ts,credit-fixed-ts,gpbs --out gpurun_out/bclean0.json ;;
    bts)     run bts 600 python bench.py --steps 20 --warmup 5 --reps 3 \
                --policies none,gpbs-ts,credit-fixed-ts,gpbs --out gpurun_out/bts.json ;;
    gemm2)   run gemm2 600 python bench.py --mix gemm2 --steps 20 --warmup 5 --reps 3 \
                --policies none,static,gpbs-share,gpbs --out gpurun_out/gemm2.json ;;
    gemm2m)  run gemm2m 600 python bench.py --mix gemm2 --steps 20 --warmup 5 --reps 2 --counters model \
                --policies none,gpbs-share,gpbs --out gpurun_out/gemm2m.json ;;
    gemm2np) GPBS_SHARE_PROBE=0 run gemm2np 600 python bench.py --mix gemm2 --steps 20 --warmup 5 --reps 2 \
                --policies none,gpbs --out gpurun_out/gemm2np.json ;;
    hwcper) for per in ${HWC_PERIODS:-1000 4000 10000}; do
               GPBS_HWC_PERIOD_US=$per run hwcper_$per 600 python bench.py --mix ${HWC_MIX:-gemm2} --steps 20 --warmup 5 \
                 --reps 2 --policies ${HWC_POLICIES:-none,gpbs} --out gpurun_out/hwcper_${HWC_MIX:-gemm2}_$per.json
             done ;;
    bbar)    run bdev 600 python bench.py --steps 20 --warmup 5 --reps 3 --policies none,gpbs,credit-fixed \
                --out gpurun_out/bdev.json && \
             GPBS_TABLE_MODE=bar run bbar 600 python bench.py --steps 20 --warmup 5 --reps 3 --policies none,gpbs,credit-fixed \
                --out gpurun_out/bbar.json ;;
    blat)    run blat 900 python bench.py --steps 20 --warmup 5 --reps 3 --policies none,gpbs,gpbs-lat,credit-fixed \
                --out gpurun_out/blat.json ;;
    blatv)   run blat_base 600 python bench.py --steps 20 --warmup 5 --reps 3 --policies none,gpbs,gpbs-lat \
                --out gpurun_out/blat_base.json && \
             GPBS_MEM_CHUNK=131072 run blat_c128 600 python bench.py --steps 20 --warmup 5 --reps 3 --policies none,gpbs,gpbs-lat \
                --out gpurun_out/blat_c128.json && \
             GPBS_HOLD_ALL=1 run blat_all 600 python bench.py --steps 20 --warmup 5 --reps 3 --policies none,gpbs,gpbs-lat \
                --out gpurun_out/blat_all.json ;;
    bkeep)   run bkeep 600 python bench.py --steps 20 --warmup 5 --reps 3 --keep-engines \
                --policies none,gpbs-ts,gpbs --out gpurun_out/bkeep.json ;;
    rehearse) GPBS_HANG_DUMP_S=${GPBS_HANG_DUMP_S:-45} run rehearse 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --reps 1 --rehearse --policies none,gpbs \
                --out gpurun_out/rehearse.json ;;
    rehearse4) GPBS_HANG_DUMP_S=${GPBS_HANG_DUMP_S:-60} run rehearse4 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
                --master-port 29534 bench.py --gpus 4 --steps 5 --warmup 1 --reps 2 --rehearse --policies none,gpbs-lat,gpbs \
                --out gpurun_out/rehearse4.json ;;
    rehearse8) GPBS_HANG_DUMP_S=${GPBS_HANG_DUMP_S:-90} run rehearse8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
                --master-port 29535 bench.py --gpus 8 --steps 3 --warmup 1 --reps 1 --rehearse --policies none,gpbs \
                --out gpurun_out/rehearse8.json ;;
    roctx)   export GPBS_ROCTX=1
             run roctx 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/roctx \
                -o run -- python bench.py --steps 5 --warmup 1 --reps 1 --policies gpbs --counters model \
                --out gpurun_out/roctx_bench.json
             unset GPBS_ROCTX ;;
    prof)    cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
             run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o run -- python3 bench.py \
                --steps 10 --warmup 2 --reps 1 --policies none,gpbs --out gpurun_out/prof_bench.json
             if ls gpurun_out/prof_r2/*/run_results.db >/dev/null 2>&1 || ls gpurun_out/prof_r2/run_results.db >/dev/null 2>&1; then
               db=$(ls gpurun_out/prof_r2/*/run_results.db gpurun_out/prof_r2/run_results.db 2>/dev/null | head -1)
               python3 scripts/rocpd_summary.py "$db" -o gpurun_out/prof_r2_summary.txt
             fi ;;
    micro)   run micro 600 python -u scripts/microbench.py --out gpurun_out/microbench.json ;;
    tmicro)  run tmicro 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_microbench.py ;;
    llmsplit) run llmsplit 1100 python -u -m pbs_amd.bench.llm_corun --fp8 --graph --seconds 5 --warmup 2 \
                --policies "${LLM_POLICIES:-solo,none,se:1/3,se:2/2,se:1/3@solo,se:2/2@solo}" --reps "${LLM_REPS:-1}" \
                --out gpurun_out/llm_split.json ;;
    kbench)  run kbench 600 python -u scripts/kbench.py ;;
    mmref)   cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
             run mmref 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mmref -o run -- \
                python3 scripts/mm_ref.py 4096 ;;
    *) echo "unknown step $step" | tee -a "$LOG" ;;
  esac
done
echo "session done $(date)" | tee -a "$LOG"
