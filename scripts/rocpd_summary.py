#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (the default output
format of rocprofv3 in ROCm 7: SQLite).  Prints calls, total/avg duration and
share of summed kernel time, plus busy-time union (kernels overlap when
tenants co-run, so the summed durations exceed wall time).

    python scripts/rocpd_summary.py gpurun_out/prof/run_results.db [-o out.txt]
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels"))
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    agg = {}
    for name, s, e in rows:
        k = short(name)
        n, tot, mx = agg.get(k, (0, 0, 0))
        agg[k] = (n + 1, tot + (e - s), max(mx, e - s))
    total = sum(v[1] for v in agg.values())
    # busy union
    iv = sorted((s, e) for _, s, e in rows)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    lines = [f"kernels: {len(rows)} dispatches, span {(t1 - t0) / 1e6:.1f} ms, busy union {busy / 1e6:.1f} ms, "
             f"summed durations {total / 1e6:.1f} ms (overlap {total / max(busy, 1):.2f}x)",
             f"{'kernel':60s} {'calls':>7s} {'total ms':>10s} {'avg us':>9s} {'max us':>9s} {'% sum':>6s}"]
    for k, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{k:60s} {n:7d} {tot / 1e6:10.2f} {tot / n / 1e3:9.1f} {mx / 1e3:9.1f} {100 * tot / total:6.2f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
