#!/bin/bash
# Round 4 session 46: the driver's default bench on the final tree (12 HIP queues by default)
# (another box: how robust is the 4mix margin over static-se?).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u bench.py > gpurun_out/r4/s46_bench.json 2> gpurun_out/r4/s46_bench.log
echo "bench rc=$? $(date +%T)"
python scripts/corun_log_policies.py gpurun_out/r4/s46_bench.log | grep -v "^  "
python -c "
import json; d=json.loads(open('gpurun_out/r4/s46_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['gpbs_vs_static_se'])"
