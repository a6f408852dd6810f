"""Solo kernel microbench for the tenant kernels (gfx950).

Reports GEMM TF/s (bf16 MFMA, fp32 acc), stream-copy and reduce-copy TB/s
(bytes read + written) across launch grids, each against the PyTorch/hipBLASLt
equivalent, as one JSON line per measurement.  Used to size the default grids
(see SUNROLL in csrc/hip/tenant_kernels.hip).

    python scripts/kbench.py [--iters 20]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pbs_amd.ops import kernels as K  # noqa: E402


def timed(fn, iters, pre=None):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for _ in range(3):
        if pre:
            pre()
        fn()
    torch.cuda.synchronize()
    ts = []
    for a, b in ev:
        if pre:
            pre()
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    L = K.lib()
    s = K._stream()
    q = K.work_queue()
    zero = q.zero_
    dev = "cuda"
    out = []
    n = 4096 if not os.environ.get("KBENCH_NO_GEMM") else 256  # KBENCH_NO_GEMM: streams / reduce only
    A = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    B = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    Cm = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    # A/B of the tile queue (plain vs XCD-range), interleaved rounds in one
    # process (cross-box timings are not comparable: DVFS).
    names = {0: "plain-queue", 1: "xcd-range", 2: "deep-prefetch", 4: "staggered-groups",
             12: "staggered-2d-blocks", 13: "staggered-xcd-range-2d-blocks"}
    if os.environ.get("KBENCH_GEMM_ONLY"):
        names = {4: "staggered-groups", 256 | 4096: "2phase-balanced", 256 | 8192: "2phase-own-a", 256 | 16384: "1phase",
                 256 | 8192 | 32768: "2phase-own-a-mfma32",
                 256 | 8192 | 65536: "2phase-own-a-lds-c",
                 256 | 8192 | 65536 | 131072: "2phase-own-a-lds-c-nt",
                 256 | 8192 | 65536 | 131072 | 8: "2phase-own-a-lds-c-nt-2d-blocks",
                 256 | 8192 | 65536 | 131072 | 8 | 1: "2phase-own-a-lds-c-nt-2d-blocks-xcd-range",
                 262144: "pipelined-1-barrier",
                 524288: "pipelined-1-barrier-asm-reads",
                 32: "4wave", 32 | (1 << 20): "4wave-agpr-acc"}
        if os.environ.get("KBENCH_GEMM_VARIANTS"):  # comma-separated opts values
            names = {int(v): names.get(int(v), str(v)) for v in os.environ["KBENCH_GEMM_VARIANTS"].split(",")}
    ab = {k: [] for k in names}
    for _ in range(5):
        for opt in names:
            L.gpbs_hip_set_gemm_opts(opt)
            ab[opt].append(timed(lambda: L.gpbs_hip_gemm_bf16(K._ptr(A), K._ptr(B), K._ptr(Cm), n, n, n, K._ptr(q),
                                                              None, 0, 0, None, None, 0, s), args.iters, zero))
    L.gpbs_hip_set_gemm_opts(256 | 8192 | 65536 | 131072 | 8)
    for opt, v in ab.items():
        ms = sorted(v)[len(v) // 2]
        out.append({"kernel": "gemm_bf16", "variant": names[opt], "shape": [n, n, n],
                    "ms": ms, "tflops": 2 * n ** 3 / ms / 1e9, "min_ms": min(v)})
    ms = timed(lambda: torch.mm(A, B.t(), out=Cm), args.iters)
    out.append({"kernel": "torch.mm", "shape": [n, n, n], "ms": ms, "tflops": 2 * n ** 3 / ms / 1e9})
    # correctness of every variant against torch (fp32 reference of a slice)
    ref = (A[:512].float() @ B.float().t())
    for opt in names:
        L.gpbs_hip_set_gemm_opts(opt)
        zero()
        Cm.zero_()
        L.gpbs_hip_gemm_bf16(K._ptr(A), K._ptr(B), K._ptr(Cm), n, n, n, K._ptr(q), None, 0, 0, None, None, 0, s)
        torch.cuda.synchronize()
        err = (Cm[:512].float() - ref).abs().max().item()
        out.append({"kernel": "gemm_bf16", "variant": names[opt], "check_max_abs_err": err,
                    "ok": err < 0.02 * ref.abs().max().item()})
    L.gpbs_hip_set_gemm_opts(256 | 8192 | 65536 | 131072 | 8)
    if os.environ.get("KBENCH_GEMM_ONLY"):
        for r in out:
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))
        return

    nbytes = 1 << 30
    src = torch.empty(nbytes // 4, device=dev, dtype=torch.float32).normal_()
    dst = torch.empty_like(src)
    for grid in (256, 512, 1024, 2048):
        ms = timed(lambda: L.gpbs_hip_stream_copy(K._ptr(src), K._ptr(dst), nbytes, 1 << 19, K._ptr(q), None, 0, 0,
                                                  None, None, grid, s), args.iters, zero)
        out.append({"kernel": "stream_copy", "bytes": nbytes, "grid": grid, "ms": ms, "tbps": 2 * nbytes / ms / 1e9})
    ms = timed(lambda: dst.copy_(src), args.iters)
    out.append({"kernel": "torch.copy_", "bytes": nbytes, "ms": ms, "tbps": 2 * nbytes / ms / 1e9})
    sopts = {0: "u16-nt", 1: "u16-ts", 2: "u8-nt", 3: "u8-ts"}
    sab = {k: [] for k in sopts}
    for _ in range(3):
        for opt in sopts:
            L.gpbs_hip_set_stream_opts(opt)
            sab[opt].append(timed(lambda: L.gpbs_hip_stream_copy(K._ptr(src), K._ptr(dst), nbytes, 1 << 19, K._ptr(q),
                                                                 None, 0, 0, None, None, 256, s), args.iters, zero))
    L.gpbs_hip_set_stream_opts(0)
    for opt, v in sab.items():
        ms = sorted(v)[len(v) // 2]
        out.append({"kernel": "stream_copy", "variant": sopts[opt], "opts": opt, "bytes": nbytes, "grid": 256,
                    "ms": ms, "tbps": 2 * nbytes / ms / 1e9})

    rb = 256 << 20
    a = torch.randn(rb // 2, device=dev, dtype=torch.bfloat16)
    b = torch.randn_like(a)
    o = torch.empty_like(a)
    for grid in (256, 512, 1024):
        ms = timed(lambda: L.gpbs_hip_reduce_bf16(K._ptr(a), K._ptr(b), K._ptr(o), rb, 1 << 19, K._ptr(q), None, 0, 0,
                                                  None, None, grid, s), args.iters, zero)
        out.append({"kernel": "reduce_bf16", "bytes": rb, "grid": grid, "ms": ms, "tbps": 3 * rb / ms / 1e9})
    # reduce variants (gpbs_hip_set_reduce_opts): unroll / temporal loads,
    # stores / 512-thread workgroups, interleaved rounds against torch.add
    ropts = {0: "u6-nt", 8: "u6-ts", 9: "u8-ts", 10: "u4-ts", 11: "u12-ts", 24: "w512-u6-ts", 25: "w512-u8-ts",
             26: "w512-u4-ts"}
    rab = {k: [] for k in ropts}
    tadd = []
    for _ in range(3):
        for opt in ropts:
            L.gpbs_hip_set_reduce_opts(opt)
            rab[opt].append(timed(lambda: L.gpbs_hip_reduce_bf16(K._ptr(a), K._ptr(b), K._ptr(o), rb, 1 << 19,
                                                                 K._ptr(q), None, 0, 0, None, None, 256, s),
                                  args.iters, zero))
        tadd.append(timed(lambda: torch.add(a, b, out=o), args.iters))
    L.gpbs_hip_set_reduce_opts(8)
    for opt, v in rab.items():
        ms = sorted(v)[len(v) // 2]
        out.append({"kernel": "reduce_bf16", "variant": ropts[opt], "opts": opt, "bytes": rb, "grid": 256, "ms": ms,
                    "tbps": 3 * rb / ms / 1e9})
    ms = sorted(tadd)[len(tadd) // 2]
    out.append({"kernel": "torch.add", "bytes": rb, "ms": ms, "tbps": 3 * rb / ms / 1e9})

    W = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
    x = torch.randn(4096, device=dev, dtype=torch.bfloat16)
    y = torch.empty(8192, device=dev, dtype=torch.float32)
    for grid in (256, 512):
        ms = timed(lambda: L.gpbs_hip_gemv_bf16(K._ptr(W), K._ptr(x), K._ptr(y), 8192, 4096, K._ptr(q), None, 0, 0,
                                                None, None, grid, s), args.iters, zero)
        out.append({"kernel": "gemv_bf16", "shape": [8192, 4096], "grid": grid, "ms": ms,
                    "tbps": W.numel() * 2 / ms / 1e9})
    for r in out:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
