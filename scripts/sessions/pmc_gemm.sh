#!/bin/bash
# rocprofv3 PMC passes over the tenant GEMM (4096^3, 10 launches) for the
# default 4-phase kernel (opts 4) and the 2-phase kernel (opts 256); one
# counter pass per run, within the per-block limits.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for opts in ${OPTS:-4 256}; do
  for pass in 1 2; do
    case $pass in
      1) P="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" ;;
      2) P="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" ;;
    esac
    d="$R/gpurun_out/pmc_gemm_${opts}_p$pass"
    mkdir -p "$d"
    timeout -s KILL 90 rocprofv3 --pmc $P -d "$d" -o run -- python3 "$R/scripts/gemm_only.py" 4096 $opts \
      > "$d/log.txt" 2>&1
    rc=$?
    echo "pmc opts=$opts pass=$pass rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    python3 "$R/scripts/pmc_summary.py" gemm256 $(find "$d" -name "*counter_collection.csv") > "$d/summary.txt" 2>&1
  done
done
