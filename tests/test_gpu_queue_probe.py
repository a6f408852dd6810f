"""Measured queue choice of the tenant shim (QueueProber) on an MI355X.

Config #5's collapse was head-of-line blocking: a latency tenant's CU-masked
queue mapped onto the same hardware pipe as a co-runner whose grids overfill
its own mask stalls behind it (profiles/llm5/queue_rotate_probe.txt: of four
queues with one mask, one ran a decode-like step at 15.5-17 ms and three at
2.5 ms).  Here a child process runs a GEMM on SEs {0,1} while this process
runs a decode-like step of small GEMVs through QueueProber over three queues
masked to SEs {2,3}; the queue it settles on must be within 1.5x of the
fastest of the three, timed afterwards on each.
"""
import os
import subprocess
import sys
import time

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

BULK = r"""
import sys, time
sys.path.insert(0, %(root)r)
import torch
from pbs_amd.ops import kernels as K
from pbs_amd.runtime.tenant import se_cu_words
torch.cuda.set_device(0)
s = torch.cuda.ExternalStream(K.cumask_stream(se_cu_words((0, 1))))
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
with torch.cuda.stream(s):
    a @ b
s.synchronize()
print("ready", flush=True)
t_end = time.monotonic() + %(seconds)f
while time.monotonic() < t_end:
    with torch.cuda.stream(s):
        for _ in range(4):
            a @ b
    s.synchronize()
print("done", flush=True)
"""


def test_queue_prober_settles_on_a_fast_queue_next_to_an_overfilling_gemm():
    from pbs_amd.ops import kernels as K
    from pbs_amd.runtime.tenant import QueueProber, se_cu_words
    torch.cuda.set_device(0)
    qs = [torch.cuda.ExternalStream(K.cumask_stream(se_cu_words((2, 3)))) for _ in range(3)]
    x = torch.randn(8, 4096, device="cuda", dtype=torch.bfloat16)
    ws = [torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16) for _ in range(12)]

    def step(s):
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            y = x
            for i in range(48):
                y = (y @ ws[i % 12]) * 0.01
        s.synchronize()
        return 1e3 * (time.perf_counter() - t0)
    for s in qs:
        step(s)
    bulk = subprocess.Popen([sys.executable, "-c", BULK % {"root": ROOT, "seconds": 12.0}],
                            stdout=subprocess.PIPE, text=True)
    try:
        assert bulk.stdout.readline().strip() == "ready"
        time.sleep(0.3)
        pr = QueueProber(3)
        t_end = time.monotonic() + 2.0
        while time.monotonic() < t_end:
            pr.record(step(qs[pr.current()]))
        chosen = pr.current()
        assert not pr.exploring and pr.explorations >= 1
        per = []
        for s in qs:
            ts = sorted(step(s) for _ in range(8))
            per.append(ts[4])
    finally:
        bulk.wait(timeout=60)
    assert bulk.returncode == 0
    assert per[chosen] <= 1.5 * min(per), (chosen, per)
