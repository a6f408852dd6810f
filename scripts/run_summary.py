"""Summarise a bench.py --out detail file (round-5 fields): per mix and
policy the median / IQR aggregate, and for the scheduler policies the
counter sampler's record -- clean / fallback / skipped metric periods per
throughput tenant, switch-aligned samples, the time-shared sample period,
the in-run attribution kernel time -- the quantum-at-bound fractions, the PBS
detector activity, and the CU-masked queues held at once.

    python scripts/run_summary.py gpurun_out/bench_detail.json [-v]
"""
import json
import statistics
import sys


def q(xs, f):
    xs = sorted(xs)
    if not xs:
        return float("nan")
    k = (len(xs) - 1) * f
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def med(xs):
    return q(xs, 0.5)


def main(path, verbose=False):
    d = json.load(open(path))
    print("line:", json.dumps({k: d["line"].get(k) for k in ("value", "n_gpus", "steps", "warmup", "ms_per_step")}))
    for mix, r in d["results"].items():
        print(f"# {mix}")
        rows = []
        for pol, rs in r["runs"].items():
            a = [x["aggregate_all_gpus"] for x in rs]
            rows.append((med(a), pol, rs, a))
        for m, pol, rs, a in sorted(rows, reverse=True):
            mq = [x.get("masked_queues", {}) for x in rs]
            held = [x.get("held_max", 0) for x in mq]
            cross = [x.get("cross_key_shares", 0) for x in mq]
            print(f"  {pol:16s} {m:.4f} IQR {q(a, .75) - q(a, .25):.4f} runs {[round(x, 3) for x in a]}"
                  f"  queues held {held} cross {cross}")
            es = [x.get("engine") for x in rs if x.get("engine")]
            if not es:
                continue
            ab = {}
            for e in es:
                for n, v in (e.get("at_bound") or {}).items():
                    ab.setdefault(n, []).append(v)
            bounds = {n: (round(sum(v["at_min"] for v in vs) / max(1, sum(v["periods"] for v in vs)), 2),
                          round(sum(v["at_max"] for v in vs) / max(1, sum(v["periods"] for v in vs)), 2))
                      for n, vs in ab.items()}
            print(f"      adapt inc/dec/rearm {[e.get('adapt_inc') for e in es]} {[e.get('adapt_dec') for e in es]} "
                  f"{[e.get('adapt_rearm') for e in es]}  tslice {es[-1].get('mean_tslice_us')}")
            print(f"      at (min, max) {bounds}")
            hw = [e.get("hwc") for e in es if e.get("hwc")]
            if hw:
                h = hw[len(hw) // 2]
                print(f"      hw: samples {[x['samples'] for x in hw]} aligned {[x.get('align_samples') for x in hw]} "
                      f"(close {h.get('align_close')} long {h.get('align_long')} short {h.get('align_short')} "
                      f"denied {h.get('align_denied')}) ts_period_us {[x.get('ts_period_us') for x in hw]} "
                      f"mean_period_us {[x.get('mean_period_us') for x in hw]}")
                print(f"      clean {[x['clean_periods'] for x in hw]} fallback {[x['model_fallback_periods'] for x in hw]}"
                      f" skipped {[x.get('skipped_periods') for x in hw]}  attr kernel us {h.get('attr_kernel_us_mean')}"
                      f" / max {h.get('attr_kernel_us_max')} lag us {h.get('attr_harvest_lag_us')}")
                print(f"      per-tenant clean frac {h.get('per_tenant_clean_frac')}")
                if verbose:
                    print(f"      tenant periods {h.get('tenant_periods')}")
            kt = [x["kernel_trace"] for x in rs if x.get("kernel_trace")]
            if kt:  # in-process kernel trace (bench.py --kernel-trace): the median run by dispatches
                k = sorted(kt, key=lambda z: z["dispatches"])[len(kt) // 2]
                tot = sum(r[2] for r in k["kernels"]) or 1
                print(f"      kernel trace: {k['dispatches']} dispatches, span {k['span_ns'] / 1e6:.1f} ms, "
                      f"dropped {k['dropped']}")
                for name, calls, tns, mx in k["kernels"][:12]:
                    print(f"        {name[:58]:58s} {calls:7d} {tns / 1e6:9.2f} ms {tns / calls / 1e3:8.1f} us avg "
                          f"{mx / 1e3:8.1f} us max {100 * tns / tot:6.2f} %")
            if verbose:  # normalised shares and absolute rates (a slower solo kernel inflates the former)
                for x in rs:
                    print("       ", round(x["aggregate_all_gpus"], 4),
                          {n: t["norm_perf"] for n, t in x["tenants"].items()},
                          {n: t.get("units_per_ms") for n, t in x["tenants"].items() if "units_per_ms" in t})
        solo = d["line"].get("solo") if mix == list(d["results"])[0] else None
        if solo:
            print("  solo:", json.dumps(solo)[:400])


if __name__ == "__main__":
    main(sys.argv[1], "-v" in sys.argv)
