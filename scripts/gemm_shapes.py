"""Tenant GEMM vs torch.mm across shapes (C = A Bt^T, bf16), to split the
4096^3 gap into per-unit fixed cost (prologue, epilogue: one 256x256 unit per
CU at 4096^2) and K-loop rate.  Variants and torch interleaved per round in
one process; median of rounds.

    python scripts/gemm_shapes.py [--iters 20] [--opts 205064,2097192]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pbs_amd.ops import kernels as K  # noqa: E402
from scripts.kbench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--opts", default="205064,2097192")
    ap.add_argument("--shapes", default="4096x4096x4096,4096x4096x8192,4096x4096x16384,8192x8192x8192")
    args = ap.parse_args()
    L = K.lib()
    s = K._stream()
    q = K.work_queue()
    opts = [int(v) for v in args.opts.split(",")]
    for sh in args.shapes.split(","):
        m, n, k = (int(v) for v in sh.split("x"))
        A = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        Cm = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        res = {o: [] for o in opts}
        res["torch"] = []
        for _ in range(5):
            for o in opts:
                L.gpbs_hip_set_gemm_opts(o)
                res[o].append(timed(lambda: L.gpbs_hip_gemm_bf16(K._ptr(A), K._ptr(B), K._ptr(Cm), m, n, k, K._ptr(q),
                                                                 None, 0, 0, None, None, 0, s), args.iters, q.zero_))
            res["torch"].append(timed(lambda: torch.mm(A, B.t(), out=Cm), args.iters))
        L.gpbs_hip_set_gemm_opts(205064)
        tmm = sorted(res["torch"])[2]
        for key, v in res.items():
            ms = sorted(v)[2]
            print(json.dumps({"shape": [m, n, k], "variant": str(key), "ms": round(ms, 4),
                              "tflops": round(2 * m * n * k / ms / 1e9, 1), "vs_torch": round(tmm / ms, 3)}), flush=True)
        del A, B, Cm


if __name__ == "__main__":
    main()
