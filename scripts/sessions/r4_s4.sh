#!/bin/bash
# Round 4 session 4: the GPU test suite, the driver's bench command with the
# solo rates re-measured after every mix (drift check over the full
# sequence), and the 8-rank N > 1 rehearsal on one GPU (per-rank pre-flight
# fields: counted agent / BDF, IPC self-test, gang transport, node totals).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
echo "== 8mix gpbs, shared queues $(date +%T)"
timeout -k 10 200 python -u bench.py --gpus 1 --mix 8mix --policies gpbs --reps 8 --steps 20 --warmup 3 \
  > gpurun_out/r4/s4_8mix_shared.json 2> gpurun_out/r4/s4_8mix_shared.log
echo "8mix rc=$?"; python scripts/corun_log_policies.py gpurun_out/r4/s4_8mix_shared.log | head -2
grep -o '"masked_queues_created": [0-9]*' gpurun_out/r4/s4_8mix_shared.log | sort | uniq -c | head -3
echo "== gpu tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4/s4_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4/s4_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4/s4_gpu_tests.log
echo "== driver bench + resolo $(date +%T)"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --resolo --out gpurun_out/r4/s4_bench_full.json \
  > gpurun_out/r4/s4_bench_line.json 2> gpurun_out/r4/s4_bench.log || { echo "bench failed"; tail -30 gpurun_out/r4/s4_bench.log; exit 1; }
echo "bench ok $(date +%T)"
echo "== 8-rank rehearsal $(date +%T)"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --rehearse-ipc --mix 4mix --steps 4 --warmup 1 --reps 1 \
  > gpurun_out/r4/s4_rehearse8.json 2> gpurun_out/r4/s4_rehearse8.log
echo "rehearse rc=$? $(date +%T)"
