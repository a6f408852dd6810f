"""The scheduler puts no work on the GPU's queues.

A time-shared memory region (three HBM streams on the memory SEs next to a
GEMM on the compute SEs) under the flagship runtime path: partition table
in BAR-written VRAM, PBS update and counter attribution on the host, the
modeled counter block read through the BAR, live hardware counters on.  An
in-process kernel trace (rocprofiler-sdk kernel-dispatch records in the
counter tool's own context) must show only the tenants' kernels: no
k_partition_switch, k_adapt, k_hwc_attribute, k_counter_reduce, and no
copy / fill blit -- while the engine switched owners, took hardware samples
and attributed them on the host.

Runs in a subprocess: the counter tool registers with rocprofiler-sdk
before the HIP runtime initialises.
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
import json, sys, time
sys.path.insert(0, %r)
from pbs_amd.counters import hwc
hwc.trace_enable(True)
assert hwc.init()
import torch
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
assert hwc.start()
from pbs_amd.runtime.gpu import GpuContext, Runner
from pbs_amd.core.config import MI355X_PROFILE
from pbs_amd.core.engine import Engine
from pbs_amd.bench.corun import BUDGET_OVERRIDES
prof = dict(MI355X_PROFILE); prof.update(BUDGET_OVERRIDES); prof["class_budget"] = 1
prof["mem_split"] = 0  # the memory region time-shared: switches all the time
e = Engine(**prof)
for x in range(8):
    for c in range(4):
        e.pool_assign(0, e.partition_add(0, x, c))
e.tenant_create("Domain-0", nslots=1)
names = ("gemm", "hbm", "hbm_b", "hbm_c")
tids = {n: e.tenant_create(n, nslots=32) for n in names}
ctx = GpuContext(0, nctx=4, table_mode="bar")
ctx.set_se_mode(True)
ctx.attach(e, nctx=4, device_adapt=False)
ctx.param("device_attr", 0)
ctx.set_hwc(True)
e.start()
rs = {"gemm": Runner(ctx, "gemm", tids["gemm"], M=4096, N=4096, K=4096)}
for n in names[1:]:
    rs[n] = Runner(ctx, "stream", tids[n], bytes=1 << 28)
def topup():
    for n, r in rs.items():
        st = r.stats()
        if st.submitted - st.units_done < 200:
            r.submit(200)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:  # settle: classes, layout
    topup(); time.sleep(0.002)
hwc.trace_stats(reset=True)
g0 = ctx.stats()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.5:
    topup(); time.sleep(0.002)
tr = hwc.trace_stats()
g1 = ctx.stats()
out = {"trace": tr, "switches": g1["switches"] - g0["switches"], "hwc": ctx.hwc_stats(),
       "units": {n: r.stats().units_done for n, r in rs.items()},
       "layout": {n: e.tenant_info(t).budget_ctx for n, t in tids.items()}}
for r in rs.values():
    r.cancel()
for r in rs.values():
    r.wait(120)
e.stop()
out["check"] = e.check()
for r in rs.values():
    r.close()
ctx.close(); e.close()
print("RESULT " + json.dumps(out))
"""

SCHED = ("k_partition_switch", "k_adapt", "k_hwc_attribute", "k_counter_reduce", "copyBuffer", "fillBuffer",
         "copyImage", "fillImage")


def test_scheduler_puts_no_kernel_on_the_gpu_queues():
    r = subprocess.run([sys.executable, "-c", CODE % ROOT], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1][7:])
    tr = out["trace"]
    print(json.dumps({k: v for k, v in out.items() if k != "trace"}, indent=1))
    print(json.dumps(tr["kernels"], indent=1))
    assert tr is not None and tr["dispatches"] > 0 and tr["dropped"] == 0, tr
    names = [k[0] for k in tr["kernels"]]
    bad = [n for n in names if any(s in n for s in SCHED)]
    assert not bad, bad
    # ... while the scheduler was busy: owner switches in the time-shared
    # memory region, hardware samples attributed on the host
    assert out["switches"] > 10, out
    assert out["hwc"]["samples"] > 0 and out["hwc"]["attr_host"] > 0, out["hwc"]
    assert out["hwc"]["attr_kernel_launches"] == 0, out["hwc"]
    assert all(v > 0 for v in out["units"].values()), out["units"]
    assert out["check"] == ""
