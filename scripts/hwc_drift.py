"""Does device-counting sampling slow the GPU down over time, and why?

Round 3 measured the GPU ~11 % slower (solo GEMM and stream rates alike)
after the 8mix's ~38k rocprofiler device-counting samples in one counting
context, and no slowdown with modeled counters.  This probe separates the
candidate causes in one GPU call.  Each variant is a fresh process (the
counter service registers before HIP starts):

  none   the same load phases with the sampler off (thermal / workload control)
  sync   synchronous samples every 1 ms during the load phases (the bench's path)
  async  GPBS_HWC_ASYNC=1: ROCPROFILER_COUNTER_FLAG_ASYNC reads into a buffer
  fresh  solo rates only, no counter service (does a slowdown outlive the process?)

Per segment it records the solo GEMM and stream rates, the sample latency,
the GPU's clock / power / temperature / throttle residency
(pbs_amd/utils/gpustate.py) and every process thread's CPU time (a runtime
thread that burns more CPU per sample would starve the runners' host side).

    python scripts/hwc_drift.py --variants fresh,none,sync,fresh,async,fresh --load-s 10 --segs 4
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, %(root)r)
mode = %(mode)r
from pbs_amd.counters import hwc
if mode in ("sync", "async"):
    assert hwc.init()
import torch
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
if mode in ("sync", "async"):
    assert hwc.start()
from pbs_amd.runtime.gpu import GpuContext, Runner
from pbs_amd.utils.gpustate import GpuStateRecorder, device_bdf
rec = GpuStateRecorder(device_bdf(0), period_s=0.2).start()
ctx = GpuContext(0, nctx=4)
g = Runner(ctx, "gemm", 1, gate=False, engine_wake=False)
s = Runner(ctx, "stream", 2, gate=False, engine_wake=False, bytes=1 << 30)
Q = {id(g): 400, id(s): 120}

def pump(rs, secs):
    d0 = [r.stats().units_done for r in rs]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for r in rs:
            st = r.stats()
            if st.submitted - st.units_done < Q[id(r)]:
                r.submit(Q[id(r)])
        time.sleep(0.001)
    dt = time.perf_counter() - t0
    return [(r.stats().units_done - d) / dt for r, d in zip(rs, d0)]

def drain(rs):
    for r in rs:
        st = r.stats()
        r.cancel()
    for r in rs:
        r.wait(30)

def threads_cpu():
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
            comm = st[st.index("(") + 1:st.rindex(")")]
            fl = st[st.rindex(")") + 2:].split()
            out[f"{comm}:{tid}"] = (int(fl[11]) + int(fl[12])) / tck
        except (OSError, ValueError):
            pass
    return out

def solo():
    t0 = rec.now()
    rg = pump([g], %(solo_s)f)[0]
    drain([g])
    t1 = rec.now()
    rs = pump([s], %(solo_s)f)[0]
    drain([s])
    t2 = rec.now()
    return {"gemm": rg, "stream": rs, "gs_gemm": rec.window(t0, t1), "gs_stream": rec.window(t1, t2)}

out = {"mode": mode, "bdf": rec.bdf, "state_source": rec.source}
pump([g, s], 0.5); drain([g, s])
out["seg0"] = solo()
cpu_prev = threads_cpu()
segs = []
for i in range(%(segs)d):
    if mode in ("sync", "async"):
        ctx.set_hwc_duty(0)
        ctx.set_hwc_period(1000, 0)
        ctx.set_hwc(True)
        ctx.hwc_reset()
    t0 = rec.now()
    load = pump([g, s], %(load_s)f)
    drain([g, s])
    t1 = rec.now()
    seg = {"load_rates": load, "gs_load": rec.window(t0, t1)}
    if mode in ("sync", "async"):
        st = ctx.hwc_stats()
        seg["samples"] = st["samples"]
        seg["mean_sample_us"] = st["mean_sample_us"]
        seg["max_sample_us"] = st["max_sample_us"]
        ctx.set_hwc(False)
        if mode == "async":
            seg["async"] = hwc.async_stats()
    seg.update(solo())
    cpu = threads_cpu()
    seg["cpu_s"] = {k: round(v - cpu_prev.get(k, 0.0), 3) for k, v in cpu.items() if v - cpu_prev.get(k, 0.0) > 0.05}
    cpu_prev = cpu
    segs.append(seg)
    print("SEG " + json.dumps({"i": i, "gemm": seg["gemm"], "stream": seg["stream"],
                               "samples": seg.get("samples"), "us": seg.get("mean_sample_us"),
                               "clk": seg["gs_gemm"].get("gfxclk_mhz"), "pw": seg["gs_gemm"].get("power_w")}), flush=True)
out["segs"] = segs
if mode in ("sync", "async"):
    hwc.stop()
    out["after_stop"] = solo()
base = out["seg0"]
last = out.get("after_stop") or (segs[-1] if segs else base)
out["rel_last_seg"] = {k: round(segs[-1][k] / base[k], 4) for k in ("gemm", "stream")} if segs else {}
out["rel_after_stop"] = {k: round(last[k] / base[k], 4) for k in ("gemm", "stream")}
g.close(); s.close(); ctx.close(); rec.stop()
print("RESULT " + json.dumps(out), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="fresh,none,sync,fresh,async,fresh")
    ap.add_argument("--load-s", type=float, default=10.0)
    ap.add_argument("--segs", type=int, default=4)
    ap.add_argument("--solo-s", type=float, default=1.5)
    ap.add_argument("--out", default="")
    ap.add_argument("--timeout", type=float, default=200.0)
    args = ap.parse_args()
    res = []
    for v in args.variants.split(","):
        segs = 0 if v == "fresh" else args.segs
        mode = "none" if v == "fresh" else v
        env = dict(os.environ)
        if v == "async":
            env["GPBS_HWC_ASYNC"] = "1"
        code = CHILD % {"root": ROOT, "mode": mode, "segs": segs, "load_s": args.load_s, "solo_s": args.solo_s}
        t0 = time.time()
        # the child's SEG lines stream through (a long variant is never silent)
        p = subprocess.Popen([sys.executable, "-u", "-c", code], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             text=True, env=env)
        lines = []
        try:
            for ln in p.stdout:
                lines.append(ln)
                if ln.startswith("SEG "):
                    print(f"[{v}] {ln.strip()}", flush=True)
            p.wait(timeout=args.timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        line = [x for x in lines if x.startswith("RESULT ")]
        rec = {"variant": v, "rc": p.returncode, "wall_s": round(time.time() - t0, 1)}
        if line:
            rec.update(json.loads(line[-1][7:]))
        else:
            rec["err"] = "".join(lines)[-2500:]
        brief = {k: rec.get(k) for k in ("variant", "rc", "wall_s", "rel_last_seg", "rel_after_stop")}
        brief["seg0"] = {k: rec.get("seg0", {}).get(k) for k in ("gemm", "stream")}
        print(json.dumps(brief), flush=True)
        res.append(rec)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(res, f, indent=1)
        if p.returncode not in (0, 1):  # crash / abort / timeout: stop touching the GPU
            break


if __name__ == "__main__":
    main()
