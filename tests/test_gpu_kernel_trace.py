"""The in-process kernel trace (csrc/hip/hwc.cpp Trace, bench.py
--kernel-trace) on a real MI355X: rocprofiler-sdk kernel-dispatch records in
the counter tool's own context, next to the live device-counting service --
the combination rocprofv3 cannot give (its tool takes the SDK and the
scheduler falls back to modeled counters).

Runs in a subprocess: the tool registers before the HIP runtime initialises.
"""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import json, sys
sys.path.insert(0, %r)
from pbs_amd.counters import hwc
assert hwc.trace_enable(True)
assert hwc.init(gpu=0)
import torch
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
assert hwc.start()
from pbs_amd.ops import kernels as K
n = 4096
A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
C = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
hwc.trace_stats(reset=True)
for _ in range(20):
    K.gemm_bf16(A, B, C)
s0 = hwc.sample()  # the counters keep working with the trace on
torch.cuda.synchronize()
st = hwc.trace_stats(reset=True)
print("RESULT " + json.dumps({"trace": st, "counted": sum(x[0] for x in s0)}))
"""


def test_kernel_trace_runs_beside_live_counters():
    r = subprocess.run([sys.executable, "-c", CODE % ROOT], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1][7:])
    st = out["trace"]
    assert st is not None and st["dropped"] == 0
    gemm = [k for k in st["kernels"] if "gemm" in k[0]]
    assert gemm, st["kernels"][:5]
    name, calls, total_ns, max_ns = gemm[0]
    assert calls >= 20
    # 4096^3 bf16 on MFMA: 80-200 us a call (1.3 PFLOP/s is ~105 us)
    assert 60e3 < total_ns / calls < 300e3, gemm[0]
    assert out["counted"] > 0
