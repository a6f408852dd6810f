"""Live CDNA4 hardware counters (rocprofiler-sdk device counting service):
per-XCD instruction / busy-cycle / L2 request / L2 miss counts move when a
tenant kernel runs on that XCD, and an HBM stream's misses per instruction are
an order of magnitude above an MFMA GEMM's.  Runs in a subprocess: the sampler must register before the HIP
runtime initialises, which the pytest process has already done."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CODE = r"""
import json, sys
sys.path.insert(0, %r)
from pbs_amd.counters import hwc
assert hwc.init()
import torch
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
assert hwc.start()
from pbs_amd.ops import kernels as K
A = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
B = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
s0 = hwc.sample()
for _ in range(5):
    K.gemm_bf16(A, B)
torch.cuda.synchronize()
s1 = hwc.sample()
src = torch.empty(256 << 20, device="cuda", dtype=torch.float32)
dst = torch.empty_like(src)
torch.cuda.synchronize()
s2 = hwc.sample()
for _ in range(5):
    dst.copy_(src)
torch.cuda.synchronize()
s3 = hwc.sample()
dd = lambda a, b: [[y - x for x, y in zip(x0, x1)] for x0, x1 in zip(a, b)]
print(json.dumps({"d": dd(s0, s1), "s": dd(s2, s3)}))
"""


def test_hardware_counters_move_on_every_xcd():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", CODE % root], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    d, s = res["d"], res["s"]
    assert len(d) == 8 and len(s) == 8
    for x, (inst, busy, req, miss) in enumerate(d):
        assert inst > 0 and busy > 0 and req > 0 and miss > 0, (x, d[x])
    # the property the PBS classifier needs from the counters: an HBM stream
    # misses L2 per instruction far more often than an LDS-tiled MFMA GEMM
    g_rate = sum(x[3] for x in d) * 1e5 / sum(x[0] for x in d)
    s_rate = sum(x[3] for x in s) * 1e5 / max(1, sum(x[0] for x in s))
    assert all(x[3] > 0 for x in s), s
    assert s_rate > 10 * g_rate, (s_rate, g_rate)
