"""What a live-counter sample costs the tenants, by counter set and period.

The PBS metric tick wants a fresh counter sample every 1 ms (the reference's
CSCHED_METRIC_TICK_PERIOD, X:xen/common/sched_credit.c:55).  A
rocprofiler-sdk device-counting sample is synchronous and perturbs the
kernels running on the GPU.  This script measures, for several counter sets
(one process each: the set is fixed when the counter service registers,
before the HIP runtime starts), a backlogged tenant's throughput alone with
the sampler off, at 4 ms and at 1 ms, plus the per-sample latency.

    python scripts/hwc_cost.py [--tenant gemm|stream] [--secs 1.0] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name -> counter spec (4 '|'-separated PBS slots, '+'-joined counters)
SPECS = {
    "full": "full",  # round-2 default: 7 SQ + 2 TCP + 1 TCC
    "lean": "lean",  # round-3 default: 5 SQ + 1 TCP + 1 TCC
    "sq2_tcp1_tcc1": "SQ_INSTS_VALU+SQ_INSTS_VALU_MFMA_MOPS_BF16|SQ_BUSY_CYCLES|TCP_TCC_READ_REQ|TCC_MISS",
    "sq1_tcc1": "SQ_INSTS_VALU|SQ_WAVES|TCC_REQ|TCC_MISS",
    "tcc2": "TCC_HIT|TCC_REQ|TCC_EA0_RDREQ|TCC_MISS",
    "sq1": "SQ_INSTS_VALU|SQ_WAVES|SQ_INSTS_SALU|SQ_INSTS_LDS",
    # refs from SQ memory instructions instead of TCP requests: 6 SQ + 1 TCC
    "lean2": "SQ_INSTS_VALU+SQ_INSTS_SALU+SQ_INSTS_VALU_MFMA_MOPS_BF16|SQ_BUSY_CYCLES|"
             "SQ_INSTS_VMEM_RD+SQ_INSTS_VMEM_WR|TCC_MISS",
}
DEFAULT_SET = "full,lean,lean2,sq1_tcc1"

CHILD = r"""
import json, sys, time
sys.path.insert(0, %(root)r)
from pbs_amd.counters import hwc
spec = %(spec)r
assert hwc.init(spec=spec or None)
import torch
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
assert hwc.start()
from pbs_amd.runtime.gpu import GpuContext, Runner
ctx = GpuContext(0, nctx=4)
kind = %(kind)r
r = Runner(ctx, "gemm", 1, gate=False, engine_wake=False) if kind == "gemm" else \
    Runner(ctx, "stream", 1, gate=False, engine_wake=False, bytes=1 << 30)
q = 400 if kind == "gemm" else 120
def rate(secs):
    st = r.stats(); d0 = st.units_done; t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        st = r.stats()
        if st.submitted - st.units_done < q:
            r.submit(q)
        time.sleep(0.001)
    return (r.stats().units_done - d0) / (time.perf_counter() - t0)
r.submit(q); rate(0.3)  # warm
out = {"spec": spec or "default", "kind": kind}
out["off"] = rate(%(secs)f)
ctx.set_hwc_duty(0)  # measure the raw period
for per in (4000, 1000):
    ctx.set_hwc_period(per, 0)   # fixed period, no back-off
    ctx.set_hwc(True)
    ctx.hwc_reset()
    out[f"p{per}"] = rate(%(secs)f)
    st = ctx.hwc_stats()
    out[f"p{per}_samples"] = st["samples"]; out[f"p{per}_mean_us"] = st["mean_sample_us"]
    out[f"p{per}_max_us"] = st["max_sample_us"]
    ctx.set_hwc(False)
out["off_again"] = rate(%(secs)f)
r.cancel(); r.wait(60); r.close(); ctx.close()
base = (out["off"] + out["off_again"]) / 2
for per in (4000, 1000):
    out[f"p{per}_rel"] = round(out[f"p{per}"] / base, 4)
print("RESULT " + json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tenant", default="gemm", choices=["gemm", "stream"])
    ap.add_argument("--secs", type=float, default=1.0)
    ap.add_argument("--specs", default=DEFAULT_SET)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    res = []
    for name in args.specs.split(","):
        code = CHILD % {"root": ROOT, "spec": SPECS[name], "kind": args.tenant, "secs": args.secs}
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
        rec = {"name": name, "rc": p.returncode}
        if line:
            rec.update(json.loads(line[-1][7:]))
        else:
            rec["err"] = (p.stdout + p.stderr)[-1500:]
        print(json.dumps(rec), flush=True)
        res.append(rec)
        if p.returncode not in (0, 1):  # a crash / abort: stop here
            break
    if args.out:
        with open(args.out, "w") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
