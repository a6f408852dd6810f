"""GEMM x stream interference on one MI355X: where should a compute-bound and
a bandwidth-bound tenant live relative to each other?

Arrangements (each tenant loops its kernel on its own stream; throughput is
taken over the window where both run, normalised to solo):

  shared      both kernels on every CU (co-resident waves, default sharing)
  cu:<f>      inside every XCD the stream gets a fraction f of the CUs and the
              GEMM the rest (hipExtStreamCreateWithCUMask; the CU-mask bit ->
              (XCD, CU) map is discovered with the census kernel)
  xcd:<k>     the stream gets k whole XCDs, the GEMM the other 8-k

    python scripts/interfere.py [--ms 60]
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

NBITS = 256


def mask_stream(L, bits):
    words = [0] * ((NBITS + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    arr = (C.c_uint32 * len(words))(*words)
    h = L.gpbs_gpu_cumask_stream(0, arr, len(words), 0)
    if not h:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    return h


def discover(L):
    """bit -> (xcc, cu-key) using one-bit CU masks and the census kernel."""
    out = {}
    buf = torch.zeros(8 * 4, dtype=torch.int32, device="cuda")
    for b in range(NBITS):
        h = mask_stream(L, [b])
        buf.zero_()
        rc = L.gpbs_hip_census(K._ptr(buf), 8, None, 0, 0, C.c_void_p(h))
        assert rc == 0
        torch.cuda.synchronize()
        v = buf.view(8, 4).cpu().tolist()
        L.gpbs_gpu_stream_destroy(C.c_void_p(h))
        keys = {(r[0], (r[1] >> 8) & 0xFF) for r in v if r[3] == 0xC0FFEE}
        out[b] = sorted(keys)
    return out


class Loop:
    def __init__(self, L, kind, stream_h, n, args):
        self.L, self.kind, self.h, self.n, self.args = L, kind, stream_h, n, args
        self.q = torch.zeros(n * 16, dtype=torch.int32, device="cuda")
        self.ext = torch.cuda.ExternalStream(stream_h) if stream_h else torch.cuda.current_stream()
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(n)]

    def launch(self, start_ev):
        s = C.c_void_p(self.ext.cuda_stream)
        self.ext.wait_event(start_ev)
        for i in range(self.n):
            qp = C.c_void_p(self.q.data_ptr() + i * 64)
            if self.kind == "gemm":
                A, B, Cm = self.args
                n = A.shape[0]
                rc = self.L.gpbs_hip_gemm_bf16(K._ptr(A), K._ptr(B), K._ptr(Cm), n, n, n, qp, None, 0, 0, None, None,
                                               0, s)
            else:
                src, dst = self.args
                nb = src.numel() * 4
                rc = self.L.gpbs_hip_stream_copy(K._ptr(src), K._ptr(dst), nb, 1 << 19, qp, None, 0, 0, None, None, 0,
                                                 s)
            assert rc == 0
            self.ev[i].record(self.ext)

    def times(self, start_ev):
        return [start_ev.elapsed_time(e) for e in self.ev]


def run(L, arr, loops, solo):
    start = torch.cuda.Event(enable_timing=True)
    for lp in loops.values():
        lp.q.zero_()
    torch.cuda.synchronize()
    start.record()
    for lp in loops.values():
        lp.launch(start)
    torch.cuda.synchronize()
    ts = {k: lp.times(start) for k, lp in loops.items()}
    window = min(t[-1] for t in ts.values())
    res = {"arrangement": arr, "window_ms": round(window, 2)}
    for k, t in ts.items():
        done = sum(1 for x in t if x <= window)
        rate = done / window if window > 0 else 0
        res[k] = round(rate / solo[k], 3) if solo.get(k) else round(rate, 3)
    if solo:
        res["sum"] = round(res["gemm"] + res["stream"], 3)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=float, default=60.0)
    args = ap.parse_args()
    L = K.lib()
    n = 4096
    A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    Cm = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    src = torch.randn(1 << 28, device="cuda")
    dst = torch.empty_like(src)
    ng = int(args.ms / 0.17)
    ns = int(args.ms / 0.40)

    def loops_for(gbits, sbits):
        gs = mask_stream(L, gbits) if gbits is not None else torch.cuda.Stream().cuda_stream
        ss = mask_stream(L, sbits) if sbits is not None else torch.cuda.Stream().cuda_stream
        return {"gemm": Loop(L, "gemm", gs, ng, (A, B, Cm)), "stream": Loop(L, "stream", ss, ns, (src, dst))}

    solo = {}
    lg = loops_for(None, None)
    for k in ("gemm", "stream"):
        r = run(L, "solo-" + k, {k: lg[k]}, {})
        solo[k] = r[k]
    print(json.dumps({"solo_per_ms": solo}))
    out = [run(L, "shared", loops_for(None, None), solo)]
    print(json.dumps(out[0]))
    bitmap = discover(L)
    print(json.dumps({"cu_mask_map": {str(b): [list(k) for k in v] for b, v in bitmap.items() if b < 80}}))
    # one CU-mask bit may select one CU in every XCD (mask replicated per XCD)
    # or one CU of one XCD; group the bits by the XCDs they reach.
    per_xcd = {}
    for b, keys in bitmap.items():
        if not keys:
            continue
        xs = tuple(sorted({k[0] for k in keys}))
        per_xcd.setdefault(xs if len(xs) > 1 else xs[0], []).append(b)
    print(json.dumps({"groups": {str(k): len(v) for k, v in per_xcd.items()}}))

    allbits = sorted(b for v in per_xcd.values() for b in v)
    for frac in (0.125, 0.25, 0.375, 0.5):
        sb, gb = [], []
        for x, bits in per_xcd.items():
            k = max(1, int(round(len(bits) * frac)))
            sb += bits[:k]
            gb += bits[k:]
        out.append(run(L, f"cu:{frac}", loops_for(gb, sb), solo))
    for k in ((1, 2, 3, 4) if len(per_xcd) == 8 else ()):
        xs = sorted(per_xcd)
        sb = [b for x in xs[:k] for b in per_xcd[x]]
        gb = [b for x in xs[k:] for b in per_xcd[x]]
        out.append(run(L, f"xcd:{k}", loops_for(gb, sb), solo))
    # stream restricted, GEMM everywhere (co-resident on the stream's CUs)
    for frac in (0.25, 0.5):
        sb = []
        for x, bits in per_xcd.items():
            sb += bits[:max(1, int(round(len(bits) * frac)))]
        out.append(run(L, f"overlap:{frac}", loops_for(allbits, sb), solo))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
