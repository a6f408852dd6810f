"""Does this GPU's CU-mask bit layout match the one gpbs assumes?

Every SE-exclusive layout builds its CU masks from one assumption
(csrc/hip/runtime.cpp se_cu_mask, runtime/tenant.py se_cu_words): mask bit b
is logical CU b/8 of XCD b%8, and logical CU i sits on shader engine i%4.
The tenant kernels' gate reads the REAL shader engine from HW_ID.  If a chip
enumerated its CUs differently, a queue masked to "SE s" would put
workgroups on other SEs, the gate would turn them away, and every
SE-partitioned policy would lose throughput on that box alone.

For each SE s this creates ONE queue masked to "SE s of every XCD", launches
the census kernel (a workgroup per slot, each reporting its XCD and HW_ID)
and reports which (XCD, SE) the workgroups really ran on.  Four queues, no
churn.  Prints one JSON line; "ok": every workgroup on its intended SE and
every XCD covered.

    python scripts/cu_map_check.py [--blocks 2048] [--device 0]

bench.py runs it in a child process before it touches the GPU and records
the verdict per rank (`ranks[i].cu_map_ok`).
"""
from __future__ import annotations

import argparse
import collections
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(args.device)

    from pbs_amd.ops import kernels as K
    from pbs_amd.runtime.tenant import se_cu_words
    L = K.lib()
    out = torch.zeros(args.blocks * 4, dtype=torch.int32, device=f"cuda:{args.device}")
    res = {"ok": True, "se": {}}
    for s in range(4):
        h = K.cumask_stream(se_cu_words((s,)), device=args.device)
        out.zero_()
        rc = L.gpbs_hip_census(K._ptr(out), args.blocks, None, 0, 0, C.c_void_p(h))
        torch.cuda.synchronize()
        rows = [r for r in out.view(args.blocks, 4).cpu().tolist() if r[3] == 0xC0FFEE]
        ses = collections.Counter(((r[1] & 0xFFFFFFFF) >> 13) & 3 for r in rows)
        xcds = sorted({r[0] & 7 for r in rows})
        good = rc == 0 and set(ses) == {s} and len(xcds) == 8
        res["se"][s] = {"rc": rc, "workgroups": len(rows), "real_se": dict(ses), "xcds": xcds, "ok": good}
        res["ok"] &= good
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
