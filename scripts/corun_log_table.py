"""Per-run table from a bench.py log: policy, aggregate, per-tenant norm_perf,
classes, PBS quanta (mean_tslice_us), miss rates.  usage: corun_log_table.py LOG"""
import json
import sys


def main(path):
    for line in open(path):
        if not line.startswith("[corun] ") or ': {"policy"' not in line:
            continue
        d = json.loads(line[line.index(': {"policy"') + 2:])
        e = d.get("engine", {})
        np_ = {k: v["norm_perf"] for k, v in d["tenants"].items()}
        print(f'{d["policy"]:16s} agg {d["aggregate"]:.3f} {np_} cls {e.get("class")} '
              f'q {e.get("mean_tslice_us")} miss {e.get("miss_rate")}')


if __name__ == "__main__":
    main(sys.argv[1])
