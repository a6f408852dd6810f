"""Summarise bench JSON runs for drift: per run aggregate, GPU clock / power /
PPT residency, sampler counts; the --resolo end/start solo ratio."""
import json
import sys

for path in sys.argv[1:]:
    line = None
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    if line is None:
        print(path, "no JSON line")
        continue
    print("==", path, "value", line["value"], "counters", line.get("counters"))
    for p, v in line["policies"].items():
        print("  ", p, "agg", v["aggregate_all_gpus"], "runs", v["runs"])
    print("   resolo", line["solo"].get("_end_over_start_rate"))
    eng = line.get("engine", {})
    h = eng.get("hwc", {})
    print("   hwc", {k: h.get(k) for k in ("samples", "burst_samples", "burst_denied", "model_fallback_periods",
                                          "clean_periods", "mean_period_us", "mean_sample_us", "budget_pct")})
    print("   mean_tslice", eng.get("mean_tslice_us"))
