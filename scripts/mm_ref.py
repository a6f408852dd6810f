"""hipBLASLt reference GEMM for the tenant GEMM's shape (C = A Bt^T, bf16,
4096^3): run under `rocprofv3 --kernel-trace --stats` to record which
library kernel (macro tile, waves, depth) torch.mm picks on gfx950."""
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
bt = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    c = a @ bt.t()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    c = a @ bt.t()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print(f"torch.mm {n}^3 bf16 (A Bt^T): {dt * 1e6:.1f} us  {2 * n ** 3 / dt / 1e12:.0f} TF/s")
