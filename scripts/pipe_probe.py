"""Which CU-masked queues interfere (pipe probe).

Creates CU-masked queues in a fixed order -- four on the compute half (SEs
{0,1} of every XCD), then K on the memory half (SEs {2,3}) -- and, with
back-to-back 4096^3 GEMMs (torch.mm) on one compute queue at a time, measures
a stream copy's rate on each memory queue in turn (and alone, with no GEMM).  A memory queue whose copies slow down far more than
the others shares a hardware pipe with the compute queue: a GEMM dispatch
waiting for CUs blocks the next dispatch of every queue on its pipe.  Prints
one JSON line per (compute queue, memory queue) and a summary keyed by the creation
index difference.

    python scripts/pipe_probe.py [--queues 8] [--ms 150]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pbs_amd.ops import kernels as K  # noqa: E402
from pbs_amd.runtime.tenant import se_cu_words  # noqa: E402


def rate(stream, src, dst, ms):
    """Copies per ms on `stream` over a window of `ms`."""
    n = 0
    with torch.cuda.stream(stream):
        dst.copy_(src)
        stream.synchronize()
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            for _ in range(4):
                dst.copy_(src)
            n += 4
            stream.synchronize()
    return n / ((time.perf_counter() - t0) * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queues", type=int, default=8)
    ap.add_argument("--ms", type=float, default=150.0)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    n = 4096
    A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    Cm = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    src = torch.randn(64 << 20, device="cuda", dtype=torch.float32)  # 256 MiB
    dst = torch.empty_like(src)
    summary = {}
    # creation order: 4 compute-half queues, then the memory-half ones (12
    # queues in all, inside the ~20-queue budget before oversubscription)
    nc = 4
    cqs = [torch.cuda.ExternalStream(K.cumask_stream(se_cu_words((0, 1)))) for _ in range(nc)]
    mqs = [torch.cuda.ExternalStream(K.cumask_stream(se_cu_words((2, 3)))) for _ in range(args.queues)]
    base = {j: rate(s, src, dst, args.ms / 2) for j, s in enumerate(mqs)}
    import threading
    for ci, cq in enumerate(cqs):
        stop = threading.Event()

        def gemms():
            with torch.cuda.stream(cq):
                while not stop.is_set():
                    for _ in range(8):
                        torch.mm(A, B.t(), out=Cm)
                    cq.synchronize()
        th = threading.Thread(target=gemms)
        th.start()
        time.sleep(0.05)
        for j, s in enumerate(mqs):
            r = rate(s, src, dst, args.ms)
            mi = nc + j  # creation index of the memory queue
            rec = {"cq": ci, "mq": mi, "diff": mi - ci, "alone": round(base[j], 3), "with_gemm": round(r, 3),
                   "ratio": round(r / base[j], 3)}
            print(json.dumps(rec), flush=True)
            summary.setdefault((mi - ci) % 4, []).append(rec["ratio"])
        stop.set()
        th.join()
        torch.cuda.synchronize()
    print(json.dumps({"ratio_by_diff_mod4": {str(k): sorted(v) for k, v in sorted(summary.items())}}), flush=True)


if __name__ == "__main__":
    main()
