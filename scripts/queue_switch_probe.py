#!/usr/bin/env python3
"""Two processes on CU-masked HIP queues: does moving a process's kernels
from one masked queue to another hurt the pair?  (Config #5's collapse:
profiles/llm5/config5_r3g_swap_nohwc.json -- a static SE split that starts
on the swapped halves and then moves collapsed the decode tenant to 3x its
step time and the trainer to 1.27x, and stayed collapsed.)

    python scripts/queue_switch_probe.py [--seconds 5] [--swap-at 1.5] [--reps 3]

Process "lat": a decode-like step of 96 small GEMVs (bf16 [8, 4096] x
[4096, 4096]), synchronised per step.  Process "bulk": one 8192^3 bf16 GEMM
per step.  Arms (every arm a fresh pair of processes):
  fixed     lat on SEs {2,3}, bulk on {0,1} for the whole run
  swap      the first --swap-at seconds on the swapped halves, then as fixed
  lat-only  lat starts on {0,1} and moves to {2,3}; bulk stays on {0,1}
  pre       like swap, but each process creates both masked streams up front
            and the swap is a choice between two existing queues
  fixed-graph / swap-graph   as fixed / swap, the lat step replayed from a HIP graph
  rotate / rotate-graph      lat creates 4 queues with the SAME mask {2,3} and
            times 12 steps on each while bulk runs (per-queue medians)
Output: per arm and rep, per-process step-time medians before / after the
swap and a 250 ms timeline; JSON on stdout.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _proc(kind, arm, seconds, swap_at, start, q):
    import torch

    from pbs_amd.ops import kernels as K
    from pbs_amd.runtime.tenant import se_cu_words
    torch.cuda.set_device(0)
    home = (2, 3) if kind == "lat" else (0, 1)
    other = (0, 1) if kind == "lat" else (2, 3)
    moves = arm in ("swap", "pre", "swap-graph") or (arm == "lat-only" and kind == "lat")
    if arm.startswith("rotate") and kind == "bulk":
        seconds = max(seconds, 3.0)
    first = other if moves else home
    streams = {}

    def stream(ses):
        if ses not in streams:
            streams[ses] = torch.cuda.ExternalStream(K.cumask_stream(se_cu_words(ses)))
        return streams[ses]
    if arm == "pre":
        stream((0, 1))
        stream((2, 3))
    rot = []
    if arm.startswith("rotate") and kind == "lat":  # K queues with the same mask, created together
        rot = [torch.cuda.ExternalStream(K.cumask_stream(se_cu_words(home))) for _ in range(4)]
    if kind == "lat":
        x = torch.randn(8, 4096, device="cuda", dtype=torch.bfloat16)
        ws = [torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16) for _ in range(12)]

        def step():
            y = x
            for i in range(96):
                y = (y @ ws[i % 12]) * 0.01
            return y
    else:
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)

        def step():
            return a @ b
    step()
    torch.cuda.synchronize()
    if kind == "lat" and arm.endswith("-graph"):  # the decode tenant replays a captured HIP graph
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        step = g.replay
        step()
        torch.cuda.synchronize()
    start.wait(timeout=600)
    if rot:  # 12 steps on each queue after 0.5 s of the bulk running; medians of the last 8
        time.sleep(0.5)
        per = []
        for s in rot:
            ts = []
            for _ in range(12):
                t1 = time.perf_counter()
                with torch.cuda.stream(s):
                    step()
                s.synchronize()
                ts.append(1e3 * (time.perf_counter() - t1))
            per.append(round(statistics.median(ts[4:]), 2))
        q.put({"kind": kind, "per_queue_ms": per, "before_ms": None, "after_ms": None, "timeline": []})
        return
    t0 = time.monotonic()
    rows = []
    while True:
        now = time.monotonic() - t0
        if now >= seconds:
            break
        ses = first if now < swap_at else home
        s = stream(ses)
        t1 = time.perf_counter()
        with torch.cuda.stream(s):
            step()
        s.synchronize()
        rows.append((now, 1e3 * (time.perf_counter() - t1)))
    before = [r for t, r in rows if 0.3 <= t < swap_at]
    after = [r for t, r in rows if t >= swap_at + 0.3]
    bins = {}
    for t, r in rows:
        bins.setdefault(int(t / 0.25), []).append(r)
    q.put({"kind": kind, "before_ms": round(statistics.median(before), 3) if before else None,
           "after_ms": round(statistics.median(after), 3) if after else None,
           "timeline": [[round(k * 0.25, 2), round(statistics.median(v), 2)] for k, v in sorted(bins.items())]})


def run_arm(arm, seconds, swap_at):
    ctx = mp.get_context("spawn")
    q, start = ctx.Queue(), ctx.Barrier(3)
    ps = [ctx.Process(target=_proc, args=(k, arm, seconds, swap_at, start, q)) for k in ("lat", "bulk")]
    for p in ps:
        p.start()
    start.wait(timeout=600)  # both processes warmed up
    out = {}
    for _ in ps:
        r = q.get(timeout=300)
        out[r["kind"]] = r
    for p in ps:
        p.join(timeout=60)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--swap-at", type=float, default=1.5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--arms", default="fixed,swap,lat-only,pre,fixed-graph,swap-graph")
    a = ap.parse_args()
    res = {}
    for rep in range(a.reps):
        for arm in a.arms.split(","):
            r = run_arm(arm, a.seconds, a.swap_at)
            res.setdefault(arm, []).append(r)
            print(f"[probe] {arm} rep {rep}: lat {r['lat']['before_ms']} -> {r['lat']['after_ms']} ms "
                  f"{r['lat'].get('per_queue_ms', '')}, "
                  f"bulk {r['bulk']['before_ms']} -> {r['bulk']['after_ms']} ms", file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
