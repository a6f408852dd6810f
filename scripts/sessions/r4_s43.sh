#!/bin/bash
# Round 4 session 43: the driver's default bench with GPBS_HWQ=12 (HIP's own
# hardware queues per process) before making it the default.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
GPBS_HWQ=12 timeout -k 10 900 python -u bench.py > gpurun_out/r4/s43_bench.json 2> gpurun_out/r4/s43_bench.log
echo "bench rc=$? $(date +%T)"
python scripts/corun_log_policies.py gpurun_out/r4/s43_bench.log | grep -v "^  "
