"""k_hwc_attribute cost: back-to-back launches on a live-layout snapshot
(for rocprofv3 --kernel-trace; prints the runtime's own measurements)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pbs_amd.ops import kernels as K  # noqa: E402

out = (C.c_double * 3)()
rc = K.lib().gpbs_hip_hwc_attr_bench(int(sys.argv[1]) if len(sys.argv) > 1 else 500, out)
print(f"rc={rc} kernel_us={out[2]:.2f} per_launch_us={out[0]:.2f} launch_wait_us={out[1]:.2f}")
