"""Live CDNA4 hardware counters (rocprofiler-sdk device counting service):
per-XCD instruction / busy-cycle / L2 counts move when a tenant kernel runs
on that XCD.  Runs in a subprocess: the sampler must register before the HIP
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
print(json.dumps({"d": [[b - a for a, b in zip(x0, x1)] for x0, x1 in zip(s0, s1)]}))
"""


def test_hardware_counters_move_on_every_xcd():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", CODE % root], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])["d"]
    assert len(d) == 8
    for x, (inst, busy, req, miss) in enumerate(d):
        assert inst > 0 and busy > 0 and req > 0, (x, d[x])
