#!/bin/bash
# rocprofv3 kernel-trace summary of the scheduler kernels (k_adapt,
# k_hwc_attribute, k_partition_switch, k_counter_reduce) next to the tenant
# kernels; summaries land in gpurun_out/prof_r3/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/prof_r3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r3" -o run -- \
  python3 "$R/scripts/prof_target.py" > "$R/gpurun_out/prof_r3/target.log" 2>&1
echo "rocprof rc=$?"
