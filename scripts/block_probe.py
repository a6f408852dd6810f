#!/usr/bin/env python3
"""Freshness of the modeled counter block as the host sees it (round 6):
a backlogged GEMM tenant on the whole GPU, and 200 reads of its counter
1 ms apart through the BAR mapping and through a device-to-host copy; a
fresh read sees a new value nearly every time."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.set_device(0)
from pbs_amd.runtime.gpu import GpuContext, Runner  # noqa: E402

ctx = GpuContext(0, nctx=4)
r = Runner(ctx, "gemm", 3, gate=False, engine_wake=False, M=4096, N=4096, K=4096)
r.submit(4000)
time.sleep(0.1)
out = {"cnt_bar": None}
for mode, name in ((0, "bar"), (1, "copy"), (0, "bar2")):
    last = C.c_int64(0)
    rc = ctx.L.gpbs_gpu_block_probe(ctx.h, 3, 200, 1000, mode, C.byref(last))
    out[name] = {"changed_of_199": rc, "last": last.value}
r.cancel()
r.wait(60)
r.close()
ctx.close()
print("RESULT " + json.dumps(out), flush=True)
