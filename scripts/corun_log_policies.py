"""Per-policy aggregates from a bench stderr log ([corun] <policy>: {...} lines):
median / IQR / runs, mean slowdown, GPU state, per-tenant norm, sampler stats."""
import json
import statistics
import sys


def q(xs, f):
    xs = sorted(xs)
    k = (len(xs) - 1) * f
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


runs = {}
for path in sys.argv[1:]:
    for l in open(path):
        if l.startswith("[corun] ") and ': {"policy"' in l:
            pol = l[len("[corun] "):l.index(":")]
            r = json.loads(l[l.index("{"):])
            mix = "+".join(sorted(r.get("tenants", {})))  # one log can hold several mixes: key by tenant set
            runs.setdefault((mix, pol), []).append(r)
mixes = sorted({k[0] for k in runs})
for (mix, pol), rs in sorted(runs.items(), key=lambda kv: (kv[0][0], -q([r["aggregate"] for r in kv[1]], 0.5))):
    if len(mixes) > 1:
        pol = f"[{'/'.join(t[:4] for t in mix.split('+'))}] {pol}"
    a = [r["aggregate"] for r in rs]
    e = [r.get("engine", {}) for r in rs]
    ten = {n: round(statistics.median(r["tenants"][n]["norm_perf"] for r in rs), 3) for n in rs[0]["tenants"]}
    hw = [x.get("hwc", {}) for x in e if x.get("hwc")]
    print(f"{pol:18s} med {q(a, .5):.4f} iqr {q(a, .75) - q(a, .25):.4f} min {min(a):.3f} max {max(a):.3f} "
          f"slow {q([r['mean_slowdown_pct'] for r in rs], .5):.0f}% runs {[round(x, 3) for x in a]}")
    print(f"{'':18s} norm {ten}")
    if e and e[0]:
        print(f"{'':18s} tslice {e[0].get('mean_tslice_us')} rearm {[x.get('adapt_rearm') for x in e]} "
              f"inc {[x.get('adapt_inc') for x in e]} dec {[x.get('adapt_dec') for x in e]}")
    if hw:
        print(f"{'':18s} hw samples {[h.get('samples') for h in hw]} fallback {[h.get('model_fallback_periods') for h in hw]}")
