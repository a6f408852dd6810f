#!/bin/bash
# Round-3 final GPU pass on the final tree: the GPU suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
echo "smoke rc=$?"
