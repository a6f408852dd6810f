"""Process-exit probe under a profiler: which step's teardown crashes.

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 scripts/exit_probe.py MODE

MODE: torch (a CUDA tensor only), lib (+ load libgpbs_hip), ctx (+ a
GpuContext in SE mode with the masked-queue burst), runner (+ one GEMM runner
that completes a few units), hwc (the in-process counter tool first; not under
rocprofv3, which holds the SDK).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
if mode == "hwc":
    from pbs_amd.counters import hwc
    assert hwc.init()
import torch  # noqa: E402

torch.cuda.set_device(0)
x = torch.ones(1024, device="cuda")
torch.cuda.synchronize()
if mode in ("lib", "pool", "ctx0", "ctxdev", "ctx", "runner", "hwc"):
    from pbs_amd.ops import kernels as K
    K.lib()
if mode == "pool":  # only the CU-masked queue burst
    import ctypes as C
    buf = (C.c_int * 64)()
    K.lib().gpbs_hip_masked_pool_prealloc(0, buf, 64)
if mode in ("ctx0", "ctxdev"):  # a context without SE mode (no masked queues); ctxdev: device table
    from pbs_amd.runtime.gpu import GpuContext
    ctx = GpuContext(0, nctx=4, table_mode="bar" if mode == "ctx0" else "device")
    ctx.close()
if mode in ("ctx", "runner", "hwc"):
    from pbs_amd.runtime.gpu import GpuContext
    ctx = GpuContext(0, nctx=4, table_mode="bar")
    ctx.set_se_mode(True)
if mode in ("runner", "hwc"):
    from pbs_amd.core.engine import Engine
    from pbs_amd.runtime.gpu import Runner
    e = Engine(partitions=[(0, xx, c) for xx in range(8) for c in range(4)])
    e.tenant_create("Domain-0", nslots=1)
    t = e.tenant_create("g", nslots=32)
    ctx.attach(e, nctx=4)
    e.start()
    r = Runner(ctx, "gemm", t, M=1024, N=1024, K=1024)
    r.submit(8)
    r.wait(60)
    r.close()
    e.stop()
    ctx.close()
    e.close()
print(f"exit_probe {mode}: done", flush=True)
