#!/usr/bin/env python3
"""Summarise a ``rocprofv3 --kernel-trace --marker-trace --output-format csv``
run of the bench: scheduler roctx ranges (gpbs:metric_tick, gpbs:publish,
gpbs:hwc_sample, gpbs:gang_epoch, gpbs:policy) and switch marks next to the
tenant kernels, as one text report.

    python scripts/roctx_summary.py DIR/run [--window-ms 2] > summary.txt

Sections: per-range duration percentiles; switch marks per partition; tenant
kernel stats; and a timeline excerpt (every scheduler event and tenant kernel
start/end in a short window of the steady state, on one clock).
"""
from __future__ import annotations

import argparse
import csv
import collections


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))] if xs else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="rocprofv3 output prefix, e.g. gpurun_out/roctx/run")
    ap.add_argument("--window-ms", type=float, default=2.0)
    ap.add_argument("--at", type=float, default=0.5, help="window start as a fraction of the policy range")
    a = ap.parse_args()
    marks = list(csv.DictReader(open(a.prefix + "_marker_api_trace.csv")))
    kerns = list(csv.DictReader(open(a.prefix + "_kernel_trace.csv")))
    t0 = min(int(r["Start_Timestamp"]) for r in marks + kerns)
    rng = collections.defaultdict(list)
    sw = collections.Counter()
    for r in marks:
        f = r["Function"]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if f.startswith("gpbs:switch"):
            sw[f.split(" ")[1]] += 1
        elif f.startswith("gpbs:gang_epoch"):
            rng["gpbs:gang_epoch"].append(d)
        else:
            rng[f].append(d)
    print("== scheduler roctx ranges (us)")
    print(f"{'range':28s} {'n':>7s} {'p50':>9s} {'p90':>9s} {'p99':>9s} {'max':>9s}")
    for f, ds in sorted(rng.items()):
        print(f"{f:28s} {len(ds):7d} {pct(ds, .5) / 1e3:9.1f} {pct(ds, .9) / 1e3:9.1f} {pct(ds, .99) / 1e3:9.1f} "
              f"{max(ds) / 1e3:9.1f}")
    print(f"\n== switch marks per partition (GPBS_ROCTX=1): {sum(sw.values())} total")
    print("  " + "  ".join(f"{k}:{v}" for k, v in sorted(sw.items())))
    ks = collections.defaultdict(list)
    for r in kerns:
        ks[r["Kernel_Name"].split("(")[0]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("\n== kernels (us)")
    for k, ds in sorted(ks.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:60]:60s} {len(ds):7d} p50 {pct(ds, .5) / 1e3:9.1f} max {max(ds) / 1e3:9.1f}")
    pol = [r for r in marks if r["Function"].startswith("gpbs:policy")]
    if pol:
        p0, p1 = int(pol[0]["Start_Timestamp"]), int(pol[0]["End_Timestamp"])
        w0 = p0 + int(a.at * (p1 - p0))
    else:
        w0 = t0 + int(0.5 * (max(int(r["End_Timestamp"]) for r in kerns) - t0))
    w1 = w0 + int(a.window_ms * 1e6)
    ev = []
    for r in marks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if w0 <= s <= w1 and not r["Function"].startswith("gpbs:policy"):
            ev.append((s, f"[sched] {r['Function']}" + (f" ({(e - s) / 1e3:.1f} us)" if e > s else "")))
    for r in kerns:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s <= w1 and e >= w0:
            name = r["Kernel_Name"].split("(")[0]
            ev.append((max(s, w0), f"[queue {r['Queue_Id']}] {name[:48]} {(e - s) / 1e3:.1f} us"))
    print(f"\n== timeline excerpt: {a.window_ms} ms at {(w0 - t0) / 1e6:.1f} ms (us from window start)")
    for s, txt in sorted(ev):
        print(f"{(s - w0) / 1e3:9.1f}  {txt}")


if __name__ == "__main__":
    main()
