"""Per-run migration churn from the engine trace rings the co-run bench dumps
(GPBS_DIAG_DIR=<dir> python bench.py --mix 8mix ... writes
trace_<policy>_NN.json.gz, pbs_amd/bench/corun.py).

Per run: the aggregate, and per tenant the STEAL / MIGRATE / SLEEP / WAKE
records of the timed window (after the last CLASS record of the layout),
plus the SLEEP records grouped in bursts (< 200 us apart): a burst that
coincides with a WAKE burst at a classify tick is the class tick sending
displaced slots home (engine.cpp classify_tick -> send_home), a lone one a
runner that drained and blocked its slots.

    python scripts/trace_storm.py gpurun_out/r4/diag [gpurun_out/r4/diag11 ...]
"""
from __future__ import annotations

import collections
import glob
import gzip
import json
import os
import sys

EVENTS = ("STEAL", "MIGRATE", "SLEEP", "WAKE")


def bursts(ts, gap_ns=200_000):
    out = []
    for t in ts:
        if out and t - out[-1][-1] < gap_ns:
            out[-1].append(t)
        else:
            out.append([t])
    return out


def analyse(path):
    d = json.load(gzip.open(path))
    recs = d["trace"]
    cls = [i for i, r in enumerate(recs) if r[1] == "CLASS"]
    recs = recs[cls[-1]:] if cls else recs
    names = {v: k for k, v in d["tid"].items()}
    cnt = {ev: collections.Counter() for ev in EVENTS}
    sleeps = collections.defaultdict(list)
    for r in recs:
        if r[1] in cnt:
            t = names.get(r[3], str(r[3]))
            cnt[r[1]][t] += 1
            if r[1] == "SLEEP":
                sleeps[t].append(r[0])
    span = (recs[-1][0] - recs[0][0]) / 1e6 if recs else 0.0
    return {"file": os.path.basename(path), "aggregate": round(d["aggregate"], 4), "span_ms": round(span, 1),
            "tenants": {t: {ev: cnt[ev].get(t, 0) for ev in EVENTS} | {"sleep_bursts": len(bursts(sleeps[t]))}
                        for t in d["tid"]}}


def main(dirs):
    for dd in dirs:
        for p in sorted(glob.glob(os.path.join(dd, "trace_*.json.gz"))):
            a = analyse(p)
            tot = {ev: sum(v[ev] for v in a["tenants"].values()) for ev in EVENTS}
            gemm = {t: (v["STEAL"], v["MIGRATE"], v["sleep_bursts"]) for t, v in a["tenants"].items()
                    if t.startswith("gemm")}
            print(f"{dd}/{a['file']}: agg {a['aggregate']:.3f} span {a['span_ms']} ms totals {tot} "
                  f"gemm (steal, migrate, sleep bursts) {gemm}")


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out/r4/diag"])
