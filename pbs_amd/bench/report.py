"""The driver-contract line of bench.py.

bench.py prints ONE JSON line on stdout that the driver parses from an 8 KB
tail, so the line carries the contract fields plus a per-mix digest only:
for each mix the {median, IQR} of gpbs, ``none``, ``static-se`` and the best
other policy (the strongest ablation), gpbs's PBS detector activity
(adapt inc / dec / rearm), how much of its metric came from clean hardware
windows vs the modeled fallback, and the fraction of metric periods its
tenants' quanta sat at a bound.  Everything else -- per-policy tables,
per-tenant rows, solo rates, drift, GPU state, every rank's pre-flight
record -- goes to the ``--out`` detail file.  ``compact_line`` is pure
Python (no torch), so a CPU test builds it from recorded runs and checks the
size bound at N = 8.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional

MAX_LINE_BYTES = 4096
# policies that are not ablations of the flagship (baselines reported on their own)
_BASELINES = ("gpbs", "none", "static", "static-se")


def _q(xs, f):
    xs = sorted(xs)
    k = (len(xs) - 1) * f
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def _mi(p: Optional[dict]) -> Optional[List[float]]:
    """[median, IQR] of a policy's aggregate (None when the policy did not run)."""
    if not p:
        return None
    a = p["aggregate_all_gpus"]
    return [a["median"], a["iqr"]]


def _hw_digest(runs: List[dict]) -> Optional[dict]:
    """Median over the gpbs runs of the clean / fallback shares of the metric
    periods (periods that fed the PBS metric: a clean hardware window or the
    calibrated modeled fallback), the worst throughput tenant's clean share,
    the mean hardware period and the one over intervals with a switch (the
    time-shared cadence)."""
    hw = [r.get("engine", {}).get("hwc") for r in runs]
    hw = [h for h in hw if h]
    if not hw:
        return None
    clean, fb, worst, period, skip = [], [], [], [], []
    for h in hw:
        c, f = h.get("clean_periods", 0), h.get("model_fallback_periods", 0)
        tot = c + f
        if tot:
            clean.append(c / tot)
            fb.append(f / tot)
            skip.append(h.get("skipped_periods", 0) / (tot + h.get("skipped_periods", 0)))
        pt = h.get("per_tenant_clean_frac")
        if pt:
            worst.append(min(pt.values()))
        if h.get("mean_period_us"):
            period.append(h["mean_period_us"] / 1e3)
    out = {}
    if clean:
        out["clean_frac"] = round(_q(clean, 0.5), 3)
        out["fallback_frac"] = round(_q(fb, 0.5), 3)
        out["skipped_frac"] = round(_q(skip, 0.5), 3)
    if worst:
        out["worst_tenant_clean_frac"] = round(_q(worst, 0.5), 3)
    if period:
        out["period_ms"] = round(_q(period, 0.5), 2)
    ts = [h.get("ts_period_us") for h in hw if h.get("ts_period_us")]
    if ts:
        out["ts_period_ms"] = round(_q(ts, 0.5) / 1e3, 2)
    return out or None


def _bound_digest(runs: List[dict]) -> Optional[dict]:
    """Median over gpbs runs of the fraction of metric periods the throughput
    tenants' quanta sat at min_us / max_us (engine ``at_bound`` records)."""
    lo, hi = [], []
    for r in runs:
        ab = r.get("engine", {}).get("at_bound")
        if not ab:
            continue
        fr = [v for v in ab.values() if v.get("periods")]
        if not fr:
            continue
        lo.append(sum(v["at_min"] for v in fr) / sum(v["periods"] for v in fr))
        hi.append(sum(v["at_max"] for v in fr) / sum(v["periods"] for v in fr))
    if not lo:
        return None
    return {"at_min": round(_q(lo, 0.5), 3), "at_max": round(_q(hi, 0.5), 3)}


def mix_digest(summary: dict, runs: Dict[str, List[dict]]) -> dict:
    """Compact per-mix record from bench.mix_summary's output and the raw runs."""
    pol = summary["policies"]
    g = pol["gpbs"]
    d = {"gpbs": _mi(g)}
    for p in ("none", "static-se"):
        if p in pol:
            d[p] = _mi(pol[p])
    abl = [(p, v) for p, v in pol.items() if p not in _BASELINES]
    if abl:
        p, v = max(abl, key=lambda kv: kv[1]["aggregate_all_gpus"]["median"])
        d["best_ablation"] = [p] + _mi(v)
        m = g["aggregate_all_gpus"]
        d["gpbs_minus_best_ablation"] = round(m["median"] - v["aggregate_all_gpus"]["median"], 4)
        d["beats_best_ablation_by_iqr"] = (m["median"] - v["aggregate_all_gpus"]["median"]) > \
            max(m["iqr"], v["aggregate_all_gpus"]["iqr"])
    if "adapt_inc" in g:
        d["adapt"] = [int(_q(g[k], 0.5)) for k in ("adapt_inc", "adapt_dec", "adapt_rearm")]
    if g.get("mean_tslice_us_by_class"):
        d["tslice_us_by_class"] = g["mean_tslice_us_by_class"]
    hw = _hw_digest(runs.get("gpbs", []))
    if hw:
        d["hw"] = hw
    b = _bound_digest(runs.get("gpbs", []))
    if b:
        d["quantum_at_bound"] = b
    if "idle_p50_ms" in g:
        d["lat_p50_ms"] = g["idle_p50_ms"]
    if "idle_p99_ms" in g and summary.get("slo"):
        # in-region latency tenant: p99 per policy against its target
        d["slo"] = {"target_ms": summary["slo"], **{p: v.get("idle_p99_ms") for p, v in pol.items()
                                                    if "idle_p99_ms" in v}}
    q = _dispatched(runs.get("gpbs", []))
    if q:
        d["dispatched_q_us"] = q
    return d


def _dispatched(runs: List[dict]) -> Optional[dict]:
    """Median over gpbs runs of the quantum each time-shared tenant was
    dispatched with (the s_timer quantum), us."""
    per: Dict[str, List[float]] = {}
    for r in runs:
        e = r.get("engine") or {}
        for n, q in (e.get("mean_tslice_us") or {}).items():
            if (e.get("shared") or {}).get(n):
                per.setdefault(n, []).append(q)
    return {n: int(_q(v, 0.5)) for n, v in sorted(per.items())} or None


def ranks_digest(ranks: List[dict]) -> dict:
    """Count plus per-rank failures only: a counted agent that is not the
    rank's device, a CU-map mismatch, an IPC self-test that failed, gang
    deadline misses."""
    fails = []
    for r in ranks:
        why = []
        ag = r.get("hwc_agent")
        if ag and r.get("device_bdf") and ag.get("bdf") and ag["bdf"] != r["device_bdf"]:
            why.append("agent_bdf")
        if r.get("cu_map_ok") is False:
            why.append("cu_map")
        if (r.get("pipes") or {}).get("ok") is False:
            why.append("pipes")
        for mix, m in (r.get("mixes") or {}).items():
            if m.get("ipc_selftest") == "failed":
                why.append(f"{mix}:ipc_selftest")
            g = m.get("gang") or {}
            if g.get("timeouts"):
                why.append(f"{mix}:gang_timeouts={g['timeouts']}")
        if why:
            fails.append({"rank": r.get("rank"), "why": why[:6]})
    coll = sorted({m.get("coll") for r in ranks for m in (r.get("mixes") or {}).values() if m.get("coll")})
    return {"n": len(ranks), "coll": coll, "failures": fails[:8]}


def compact_line(full: dict, digests: Dict[str, dict], detail_path: str = "") -> dict:
    """The stdout line: the contract fields of `full`, the per-mix digests
    and the ranks digest, at most MAX_LINE_BYTES.  An oversized line degrades
    step by step instead of failing (a raise on rank 0 before the final
    barrier would leave the other ranks waiting in it): the least
    important digest fields go first, then the per-rank failure list is cut,
    then the non-headline mixes keep only their policy medians; the contract
    fields always stay."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "mean_slowdown_pct", "counters")
    line = {k: full[k] for k in keep if k in full}
    line["reps"] = full.get("protocol", {}).get("reps")
    line["mixes"] = {m: dict(d) for m, d in digests.items()}
    line["ranks"] = ranks_digest(full.get("ranks") or [])
    if detail_path:
        line["detail"] = detail_path
    head = next(iter(line["mixes"]), None)

    def size() -> int:
        return len(json.dumps(line))

    steps = [
        lambda: [m.pop(k, None) for m in line["mixes"].values()
                 for k in ("tslice_us_by_class", "lat_p50_ms", "quantum_at_bound")],
        lambda: [m.pop(k, None) for n, m in line["mixes"].items() if n != head
                 for k in ("hw", "dispatched_q_us")],
        lambda: line["ranks"].update(failures=line["ranks"]["failures"][:2],
                                     n_failed=len(line["ranks"]["failures"])),
        lambda: [line["mixes"].__setitem__(n, {k: v for k, v in m.items()
                                               if k in ("gpbs", "none", "static-se", "best_ablation")})
                 for n, m in list(line["mixes"].items()) if n != head],
        lambda: line.update(data=str(line.get("data", ""))[:160], unit=str(line.get("unit", ""))[:160]),
        lambda: line["mixes"].__setitem__(head, {k: v for k, v in line["mixes"][head].items()
                                                 if k in ("gpbs", "none", "static-se", "best_ablation")})
        if head else None,
        lambda: line.update(mixes={head: line["mixes"][head]} if head else {}),
        lambda: line.update(ranks={"n": line["ranks"].get("n"), "n_failed": len(line["ranks"].get("failures", []))}),
    ]
    for st in steps:
        if size() <= MAX_LINE_BYTES:
            break
        st()
    return line
