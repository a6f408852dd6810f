#!/usr/bin/env python3
"""Freshness of the modeled counter block as the host sees it (round 6):
a backlogged GEMM tenant, ungated on the whole GPU and then gated to one
shader engine per XCD (units 4x longer), and 200 reads of its counter 1 ms
apart through the BAR mapping and through a device-to-host copy; a fresh
read sees a new value nearly every time."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.set_device(0)
from pbs_amd.runtime.gpu import CTX, XCDS, GpuContext, Runner  # noqa: E402

ctx = GpuContext(0, nctx=4)
T = 3
r = Runner(ctx, "gemm", T, gate=False, engine_wake=False, M=4096, N=4096, K=4096)
out = {}


def probe(name, n=200):
    for mode, m in ((0, "bar"), (1, "copy")):
        last = C.c_int64(0)
        rc = ctx.L.gpbs_gpu_block_probe(ctx.h, T, n, 1000, mode, C.byref(last))
        out[f"{name}_{m}"] = {"changed_of": n - 1, "changed": rc}


r.submit(20000)
time.sleep(0.05)
probe("ungated")
r.cancel()
r.wait(60)
ctx.set_se_mode(True)
ctx.set_owners([T if c == 0 else -1 for x in range(XCDS) for c in range(CTX)])
r.set_gate(True)
r.submit(20000)
time.sleep(0.05)
probe("one_se_per_xcd")
st = r.stats()
out["units_done"] = st.units_done
r.cancel()
r.wait(120)
r.close()
ctx.close()
print("RESULT " + json.dumps(out), flush=True)
