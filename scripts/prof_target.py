"""rocprofv3 target for the round-3 scheduler-kernel summary.

Under rocprofv3 the profiler owns the rocprofiler-sdk counter service, so the
bench runs on modeled counters (the device PBS update k_adapt still runs
every metric tick); k_hwc_attribute -- which only runs on live hardware
samples -- is exercised by its self-test on inputs of the live layout
(32 partitions x 32 tenants), so the trace carries its real cost too.

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 scripts/prof_target.py
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pbs_amd.ops import kernels as K  # noqa: E402

L = K.lib()
worst = C.c_double(0)
rc = L.gpbs_hip_hwc_attr_selftest(11, 200, C.byref(worst))
print(f"hwc_attr_selftest rc={rc} max_rel={worst.value:.3g}", flush=True)
import bench  # noqa: E402

sys.argv = ["bench.py", "--mix", "4mix", "--policies", "none,gpbs", "--reps", "1", "--steps", "20", "--warmup", "3",
            "--counters", "model", "--out", os.path.join(ROOT, "gpurun_out", "prof_r3_bench.json")]
bench.main()
