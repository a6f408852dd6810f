"""Shader-engine-granular interference map on one MI355X.

An MI355X XCD has four shader engines (SE) of 8 CUs; a CU mask can confine a
kernel to any set of SEs (hipExtStreamCreateWithCUMask: bit b = logical CU
b/8 of XCD b%8, which sits on SE (b/8)%4).  SE-disjoint confinement is also
what makes the SQ/TCP hardware counters exactly attributable per tenant
(profiles/hwc/se_separation_probe.txt).  This script measures, for the 4-mix
tenant kernels, what each tenant achieves on k SEs per XCD with w workgroups
per CU, and what SE-disjoint arrangements of GEMM + stream (+ reduce) give
against full co-residence (the `none` policy).

    python scripts/se_interfere.py [--ms 80] [--out FILE]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPU_MAX_HW_QUEUES"] = str(max(8, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))

import torch  # noqa: E402

from pbs_amd.ops import kernels as K  # noqa: E402


def se_bits(ses):
    return [b for b in range(256) if ((b // 8) % 4) in ses]


_streams = {}


def stream_for(L, ses, name):
    key = (name, tuple(sorted(ses)) if ses is not None else None)
    if key in _streams:
        return _streams[key]
    if ses is None or len(ses) == 4:
        h = torch.cuda.Stream().cuda_stream
    else:
        words = [0] * 8
        for b in se_bits(ses):
            words[b // 32] |= 1 << (b % 32)
        arr = (C.c_uint32 * 8)(*words)
        h = L.gpbs_gpu_cumask_stream(0, arr, 8, 0)
        if not h:
            raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    _streams[key] = h
    return h


class Loop:
    """n back-to-back units of one tenant kernel on one (masked) stream."""

    def __init__(self, L, kind, ses, grid, n, bufs, slot):
        self.L, self.kind, self.grid, self.n, self.bufs = L, kind, grid, n, bufs
        self.h = stream_for(L, ses, slot)
        self.ext = torch.cuda.ExternalStream(self.h)
        self.q = torch.zeros(n * 16 + 16, dtype=torch.int32, device="cuda")
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(n)]

    def launch(self, start_ev):
        s = C.c_void_p(self.ext.cuda_stream)
        self.ext.wait_event(start_ev)
        for i in range(self.n):
            qp = C.c_void_p(self.q.data_ptr() + i * 64)
            if self.kind == "gemm":
                A, B, Cm = self.bufs
                n = A.shape[0]
                rc = self.L.gpbs_hip_gemm_bf16(K._ptr(A), K._ptr(B), K._ptr(Cm), n, n, n, qp, None, 0, 0, None, None,
                                               self.grid, s)
            elif self.kind == "stream":
                src, dst = self.bufs
                rc = self.L.gpbs_hip_stream_copy(K._ptr(src), K._ptr(dst), src.numel() * 4, 1 << 19, qp, None, 0, 0,
                                                 None, None, self.grid, s)
            else:
                a, b, o = self.bufs
                rc = self.L.gpbs_hip_reduce_bf16(K._ptr(a), K._ptr(b), K._ptr(o), a.numel() * 2, 1 << 19, qp, None, 0,
                                                 0, None, None, self.grid, s)
            assert rc == 0, rc
            self.ev[i].record(self.ext)


def run(loops):
    start = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    start.record()
    for lp in loops.values():
        lp.launch(start)
    torch.cuda.synchronize()
    ts = {k: [start.elapsed_time(e) for e in lp.ev] for k, lp in loops.items()}
    window = min(t[-1] for t in ts.values())
    return {k: sum(1 for x in t if x <= window) / window for k, t in ts.items()}, window


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=float, default=80.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--set", default="4mix", choices=["4mix", "phase"],
                    help="4mix: the round-2 scans + GEMM/stream/reduce arrangements; phase: arrangements of the "
                         "phase mix's tenant sets (two GEMMs + a stream, a GEMM + two streams, two tenants)")
    args = ap.parse_args()
    L = K.lib()
    n = 4096
    bufs = {
        "gemm": (torch.randn(n, n, device="cuda", dtype=torch.bfloat16),
                 torch.randn(n, n, device="cuda", dtype=torch.bfloat16),
                 torch.empty(n, n, device="cuda", dtype=torch.bfloat16)),
        "stream": (torch.randn(1 << 28, device="cuda"), torch.empty(1 << 28, device="cuda")),
        "reduce": (torch.randn(1 << 27, device="cuda", dtype=torch.bfloat16),
                   torch.randn(1 << 27, device="cuda", dtype=torch.bfloat16),
                   torch.empty(1 << 27, device="cuda", dtype=torch.bfloat16)),
    }
    unit_ms = {"gemm": 0.125, "stream": 0.40, "reduce": 0.16}
    out = []

    def emit(rec):
        out.append(rec)
        print(json.dumps(rec), flush=True)

    def loops_for(spec, scale=1.0):
        # spec: {name: (kind, ses, wg_per_cu)}; grid = wg/CU x CUs in the mask
        res = {}
        for name, (kind, ses, w) in spec.items():
            ncu = 8 * 8 * (len(ses) if ses is not None else 4)
            grid = max(1, int(w * ncu))
            cnt = int(args.ms * scale / unit_ms[kind] * (4 / (len(ses) if ses else 4))) + 4
            res[name] = Loop(L, kind, ses, grid, cnt, bufs[kind], name)
        return res

    solo = {}
    for kind in ("gemm", "stream", "reduce"):
        run(loops_for({kind: (kind, None, 1)}, 0.2))  # warm
        r, _ = run(loops_for({kind: (kind, None, 1)}))
        solo[kind] = r[kind]
    emit({"solo_units_per_ms": solo, "note": "default grids (1 WG/CU), whole GPU"})

    def norm(r, kinds):
        return {k: round(v / solo[kinds[k]], 3) for k, v in r.items()}

    if args.set == "phase":
        G, S = "gemm", "stream"
        arrs = [
            # two GEMMs + a stream (phase tenant in its GEMM phase, hbm on)
            ("2g+s shared", {"g": (G, None, 1), "p": (G, None, 1), "s": (S, None, 1)}),
            ("g1|p1|s2", {"g": (G, (0,), 1), "p": (G, (1,), 1), "s": (S, (2, 3), 2)}),
            ("g2|p1|s1", {"g": (G, (0, 1), 1), "p": (G, (2,), 1), "s": (S, (3,), 4)}),
            ("gp2|s2", {"g": (G, (0, 1), 1), "p": (G, (0, 1), 1), "s": (S, (2, 3), 2)}),
            ("gp3|s1", {"g": (G, (0, 1, 2), 1), "p": (G, (0, 1, 2), 1), "s": (S, (3,), 4)}),
            ("gp-all|s2", {"g": (G, None, 1), "p": (G, None, 1), "s": (S, (2, 3), 2)}),
            ("gp-all|s1", {"g": (G, None, 1), "p": (G, None, 1), "s": (S, (3,), 4)}),
            ("g2|p2|s-all", {"g": (G, (0, 1), 1), "p": (G, (2, 3), 1), "s": (S, None, 1)}),
            # a GEMM + two streams (phase tenant streaming, hbm on)
            ("g+2s shared", {"g": (G, None, 1), "p": (S, None, 1), "s": (S, None, 1)}),
            ("g2|p1|s1 s", {"g": (G, (0, 1), 1), "p": (S, (2,), 4), "s": (S, (3,), 4)}),
            ("g2|ps2", {"g": (G, (0, 1), 1), "p": (S, (2, 3), 2), "s": (S, (2, 3), 2)}),
            ("g-all|ps2", {"g": (G, None, 1), "p": (S, (2, 3), 2), "s": (S, (2, 3), 2)}),
            # two GEMMs (hbm off)
            ("2g shared", {"g": (G, None, 1), "p": (G, None, 1)}),
            ("g2|p2", {"g": (G, (0, 1), 1), "p": (G, (2, 3), 1)}),
            ("g3|p1", {"g": (G, (0, 1, 2), 1), "p": (G, (3,), 1)}),
            # a GEMM + a stream (hbm off, phase streaming)
            ("g+s shared", {"g": (G, None, 1), "p": (S, None, 1)}),
            ("g2|p2 s", {"g": (G, (0, 1), 1), "p": (S, (2, 3), 2)}),
            ("g3|p1 s", {"g": (G, (0, 1, 2), 1), "p": (S, (3,), 4)}),
            ("g-all|p2 s", {"g": (G, None, 1), "p": (S, (2, 3), 2)}),
        ]
        for name, spec in arrs:
            r, win = run(loops_for(spec))
            kinds = {k: v[0] for k, v in spec.items()}
            nr = norm(r, kinds)
            emit({"arrangement": name, "window_ms": round(win, 1), **nr, "sum": round(sum(nr.values()), 3)})
        if args.out:
            with open(args.out, "w") as f:
                for rec in out:
                    f.write(json.dumps(rec) + "\n")
        return

    # --- single tenants on k SEs per XCD, w workgroups per CU
    for kind, wlist in (("stream", (1, 2, 4, 8)), ("reduce", (1, 2, 4)), ("gemm", (1,))):
        for k in (1, 2, 3, 4):
            for w in wlist:
                ses = tuple(range(4 - k, 4))
                r, win = run(loops_for({kind: (kind, ses, w)}))
                emit({"solo_scan": kind, "ses": k, "wg_per_cu": w, "norm": round(r[kind] / solo[kind], 3)})

    # --- arrangements of GEMM + stream (+ reduce)
    arrs = [
        ("shared-2", {"gemm": ("gemm", None, 1), "hbm": ("stream", None, 1)}),
        ("g3|s1 w4", {"gemm": ("gemm", (0, 1, 2), 1), "hbm": ("stream", (3,), 4)}),
        ("g3|s1 w8", {"gemm": ("gemm", (0, 1, 2), 1), "hbm": ("stream", (3,), 8)}),
        ("g2|s2 w2", {"gemm": ("gemm", (0, 1), 1), "hbm": ("stream", (2, 3), 2)}),
        ("g2|s2 w4", {"gemm": ("gemm", (0, 1), 1), "hbm": ("stream", (2, 3), 4)}),
        ("shared-3", {"gemm": ("gemm", None, 1), "hbm": ("stream", None, 1), "coll": ("reduce", None, 1)}),
        ("g2|s1|r1 w4", {"gemm": ("gemm", (0, 1), 1), "hbm": ("stream", (2,), 4), "coll": ("reduce", (3,), 4)}),
        ("g2|s1|r1 w8", {"gemm": ("gemm", (0, 1), 1), "hbm": ("stream", (2,), 8), "coll": ("reduce", (3,), 8)}),
        ("g2|sr2 w2", {"gemm": ("gemm", (0, 1), 1), "hbm": ("stream", (2, 3), 2), "coll": ("reduce", (2, 3), 2)}),
        ("g3|sr1 w4", {"gemm": ("gemm", (0, 1, 2), 1), "hbm": ("stream", (3,), 4), "coll": ("reduce", (3,), 4)}),
        ("g3|sr1 w2", {"gemm": ("gemm", (0, 1, 2), 1), "hbm": ("stream", (3,), 2), "coll": ("reduce", (3,), 2)}),
        ("gall+sr1 w4", {"gemm": ("gemm", None, 1), "hbm": ("stream", (3,), 4), "coll": ("reduce", (3,), 4)}),
    ]
    for name, spec in arrs:
        r, win = run(loops_for(spec))
        kinds = {k: v[0] for k, v in spec.items()}
        nr = norm(r, kinds)
        emit({"arrangement": name, "window_ms": round(win, 1), **nr, "sum": round(sum(nr.values()), 3)})
    if args.out:
        with open(args.out, "w") as f:
            for rec in out:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
