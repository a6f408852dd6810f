"""Summarise a bench.py --out JSON: per policy median/IQR aggregate and mean
slowdown, and per run the tenants' normalised throughput, contention classes
and hardware miss rates.

    python scripts/bench_summary.py gpurun_out/bench.json
"""
import json
import sys


def main(path):
    d = json.load(open(path))
    line = d["line"]
    print(f"headline gpbs value {line['value']}  mean slowdown {line['mean_slowdown_pct']}")
    for p, s in line["policies"].items():
        a, m = s["aggregate_all_gpus"], s["mean_slowdown_pct"]
        print(f"  {p:16s} agg {a['median']:.4f} (IQR {a['iqr']:.4f}, {a['min']:.3f}-{a['max']:.3f})  "
              f"slowdown {m['median']:.1f} (IQR {m['iqr']:.1f})")
    if "-v" in sys.argv:
        for p, rs in d["runs"].items():
            for r in rs:
                t, e = r["tenants"], r.get("engine", {})
                hw = e.get("hw_tenant", {})
                print(f"    {p:16s} {r['aggregate_all_gpus']:.3f}", {k: t[k]["norm_perf"] for k in t},
                      "cls", e.get("class"), "miss", {k: v.get("miss_rate") for k, v in hw.items()},
                      "mfrac", e.get("hwc", {}).get("metric_frac"))


if __name__ == "__main__":
    main(sys.argv[1])
