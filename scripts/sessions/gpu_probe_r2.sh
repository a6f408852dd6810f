#!/bin/bash
# Round-2 probe session: counter dimensions, SE separation, sample latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -s KILL 60 scripts/hwc_probe2.bin list > gpurun_out/probe/list.txt 2>&1 || { echo "list rc=$?"; exit 1; }
echo "list ok: $(wc -l < gpurun_out/probe/list.txt) lines"
timeout -s KILL 60 scripts/hwc_probe2.bin sep "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,TCC_REQ,TCC_MISS,TCP_TCC_READ_REQ,TCP_TCC_WRITE_REQ,GRBM_GUI_ACTIVE" > gpurun_out/probe/sep.txt 2>&1 || { echo "sep rc=$?"; cat gpurun_out/probe/sep.txt; exit 1; }
cat gpurun_out/probe/sep.txt
timeout -s KILL 90 scripts/hwc_probe2.bin lat "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,TCC_REQ,TCC_MISS,TCP_TCC_READ_REQ,TCP_TCC_WRITE_REQ,GRBM_GUI_ACTIVE" > gpurun_out/probe/lat.txt 2>&1 || { echo "lat rc=$?"; cat gpurun_out/probe/lat.txt; exit 1; }
cat gpurun_out/probe/lat.txt
