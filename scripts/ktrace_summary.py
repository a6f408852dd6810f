"""Per-policy medians, per-tenant rates and scheduler-kernel table of a bench
--out file run with --kernel-trace (scheduler kernels: k_adapt,
k_partition_switch, k_hwc_attribute, k_counter_reduce, blits)."""
import json
import statistics as st
import sys

SCHED = ("k_adapt", "k_partition_switch", "k_hwc_attribute", "k_counter_reduce", "copyBuffer", "fillBuffer")


def main(paths):
    for path in paths:
        d = json.load(open(path))
        for mix, res in d["results"].items():
            print(f"== {path} {mix}")
            for pol, runs in res["runs"].items():
                ten = runs[0]["tenants"].keys()
                aggs = sorted(r["aggregate"] for r in runs)
                row = {n: round(st.median([r["tenants"][n].get("norm_perf", 0) for r in runs]), 3) for n in ten}
                print(f"{pol:14s} med {st.median(aggs):.4f} iqr {aggs[-1] - aggs[0]:.4f} {row}")
                tot = {}
                span = 0
                for r in runs:
                    kt = r.get("kernel_trace") or {}
                    span += kt.get("span_ns", 0)
                    for name, n, ns, mx in kt.get("kernels", []):
                        for k in SCHED:
                            if k in name:
                                t = tot.setdefault(k, [0, 0, 0])
                                t[0] += n
                                t[1] += ns
                                t[2] = max(t[2], mx)
                for k, (n, ns, mx) in tot.items():
                    print(f"     {k:20s} n={n:6d} per_s={n / max(span, 1) * 1e9:7.1f} mean_us={ns / max(n, 1) / 1e3:7.1f}"
                          f" max_us={mx / 1e3:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
