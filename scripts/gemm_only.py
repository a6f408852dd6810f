"""Run the tenant GEMM alone (for rocprofv3 PMC collection)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pbs_amd.ops import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
opts = int(sys.argv[2]) if len(sys.argv) > 2 else 0
K.lib().gpbs_hip_set_gemm_opts(opts)
A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    K.gemm_bf16(A, B)
torch.cuda.synchronize()
print("done")
