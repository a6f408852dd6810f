"""Per-barrier timing of the tenant GEMM's K loop (diagnostic build, opts bit 6).

Lane 0 of every wave of the first 64 workgroups records s_memtime after each
of the 8 barriers of K-tiles 8..23 (csrc/hip/tenant_kernels.hip, STAMP);
this prints, per wave group (wr = 0 / 1, the staggered halves), the median
cycles of every barrier interval, the cycles per K-tile, the in-kernel clock
(s_memtime over s_memrealtime) and the MFMA busy fraction they imply
(2 waves x 64 MFMA x 16 cycles per SIMD per K-tile), next to the TF/s of the
plain and the stamped build timed in the same process.

    python scripts/gemm_stamps.py [n] [opts]   (opts 256: the 2-phase kernel, 4 intervals per K-tile)
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pbs_amd.ops import kernels as K  # noqa: E402

TILES, SLOTS, WGS = 16, 10, 64


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    base = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    nint = 2 if base & 16384 else (4 if base & 256 else 8)  # barrier intervals per K-tile
    L = K.lib()
    L.gpbs_hip_set_gemm_dbg.restype = C.c_int
    L.gpbs_hip_set_gemm_dbg.argtypes = [C.c_void_p]
    s = K._stream()
    q = K.work_queue()
    A = torch.rand(n, n, device="cuda", dtype=torch.bfloat16) * 2 - 1
    B = torch.rand(n, n, device="cuda", dtype=torch.bfloat16) * 2 - 1
    Cm = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    words = L.gpbs_hip_set_gemm_dbg(None)
    dbg = torch.zeros(words, device="cuda", dtype=torch.int32)
    assert L.gpbs_hip_set_gemm_dbg(C.c_void_p(dbg.data_ptr())) == words

    def run(opts, iters=20):
        L.gpbs_hip_set_gemm_opts(opts)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in ev:
            q.zero_()
            a.record()
            rc = L.gpbs_hip_gemm_bf16(K._ptr(A), K._ptr(B), K._ptr(Cm), n, n, n, K._ptr(q), None, 0, 0, None, None,
                                      0, s)
            assert rc == 0
            b.record()
        torch.cuda.synchronize()
        return sorted(a.elapsed_time(b) for a, b in ev)[iters // 2]

    # warm the clocks, then interleave plain / stamped rounds
    for _ in range(3):
        run(base)
    res = {"plain": [], "stamp": []}
    for _ in range(5):
        res["plain"].append(run(base))
        res["stamp"].append(run(base | 64))
    L.gpbs_hip_set_gemm_opts(256 | 8192 | 65536 | 131072)
    tf = {k: 2 * n ** 3 / (sorted(v)[2]) / 1e9 for k, v in res.items()}
    ref = A[:256].float() @ B.float().t()
    err = (Cm[:256].float() - ref).abs().max().item()
    raw = dbg.cpu().numpy().astype(np.uint32).astype(np.int64)
    st = raw[:WGS * 8 * TILES * SLOTS].reshape(WGS, 8, TILES, SLOTS)
    ph = raw[WGS * 8 * TILES * SLOTS:].reshape(-1, 4)  # per WG: entry, loop start, loop end, stores done (10 ns)
    ph = ph[(ph != 0).all(axis=1)]
    cyc = st[..., :nint + 1]
    d = np.diff(cyc, axis=-1) % (1 << 32)            # nint intervals per tile
    per_tile = (cyc[..., nint] - cyc[..., 0]) % (1 << 32)
    real = (st[..., 9] % (1 << 32)).astype(np.int64)
    # clock: memtime cycles over realtime (100 MHz) across the stamped tiles
    dc = (cyc[:, :, -1, 0] - cyc[:, :, 0, 0]) % (1 << 32)
    dr = (real[:, :, -1] - real[:, :, 0]) % (1 << 32)
    ok = dr > 0
    ghz = float(np.median(dc[ok] / dr[ok] * 0.1)) if ok.any() else None
    out = {"n": n, "opts": base, "tflops_plain": round(tf["plain"], 1), "tflops_stamp": round(tf["stamp"], 1),
           "max_abs_err": round(err, 4), "clock_ghz": round(ghz, 3) if ghz else None}
    for g in (0, 1):
        dd = d[:, 4 * g:4 * g + 4]
        out[f"group{g}_interval_cycles_median"] = [int(np.median(dd[..., k])) for k in range(nint)]
        out[f"group{g}_interval_cycles_p90"] = [int(np.percentile(dd[..., k], 90)) for k in range(nint)]
    if len(ph):
        t0 = ph[:, 0].min()
        rel = (ph - t0) % (1 << 32) / 100.0  # us from the first workgroup's entry
        out["wg_phase_us"] = {"n_wg": int(len(ph)),
                              "entry_p50_max": [round(float(np.median(rel[:, 0])), 2), round(float(rel[:, 0].max()), 2)],
                              "prologue_p50": round(float(np.median(rel[:, 1] - rel[:, 0])), 2),
                              "loop_p50_max": [round(float(np.median(rel[:, 2] - rel[:, 1])), 2),
                                               round(float((rel[:, 2] - rel[:, 1]).max()), 2)],
                              "epilogue_p50_max": [round(float(np.median(rel[:, 3] - rel[:, 2])), 2),
                                                   round(float((rel[:, 3] - rel[:, 2]).max()), 2)],
                              "last_done": round(float(rel[:, 3].max()), 2)}
    pt = float(np.median(per_tile))
    out["cycles_per_ktile_median"] = int(pt)
    out["mfma_busy_implied"] = round(2 * 64 * 16 / pt, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
