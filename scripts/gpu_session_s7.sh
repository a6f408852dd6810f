#!/bin/bash
# GPU session: GEMM epilogue PMC + kbench, 8-rank IPC rehearsal on one GPU.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  -d $O/pmc_gemm_new -o gemm --output-format csv -- python3 $R/scripts/gemm_only.py 4096 205056 > $O/s7_pmc.log 2>&1 &&
KBENCH_GEMM_ONLY=1 timeout -k 10 300 python -u scripts/kbench.py --iters 20 > $O/s7_kbench.jsonl 2> $O/s7_kbench.log &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 \
  bench.py --gpus 8 --steps 3 --warmup 1 --reps 1 --reps-extra 1 --rehearse-ipc --policies none,gpbs --hang-dump-s 90 \
  --out $O/s7_rehearse8.json > $O/s7_rehearse8.out 2> $O/s7_rehearse8.log
