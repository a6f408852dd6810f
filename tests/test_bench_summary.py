"""bench.py's per-mix summary on real run records (round-4 8mix, two
policies, tests/data/bench_runs_8mix_r4.json): medians / IQR, the drift
check (last five gpbs runs vs the first five), the per-class quantum and
the GPU-state record."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_mix_summary_fields():
    import bench
    with open(os.path.join(ROOT, "tests", "data", "bench_runs_8mix_r4.json")) as f:
        runs = json.load(f)
    s = bench.mix_summary("8mix", runs, {"gemm": {}}, 6)
    xs = sorted(r["aggregate_all_gpus"] for r in runs["gpbs"])
    assert s["value"] == round(bench.q(xs, 0.5), 4)
    p = s["policies"]["gpbs"]
    assert p["aggregate_all_gpus"]["iqr"] >= 0 and len(p["runs"]) == len(runs["gpbs"])
    d = s["drift"]
    assert d["n"] == 3 and "last_within_first_iqr" in d  # 6 runs: first three vs last three
    assert set(p["mean_tslice_us_by_class"]) <= {"0", "1"}
    assert s["gpu_state"]["first_run"]["gfxclk_mhz"] > 0
    assert "adapt_inc" in p and "adapt_dec" in p


def test_quantile_helper():
    import bench
    assert bench.q([1, 2, 3, 4], 0.5) == 2.5
    assert bench.summ([{"a": 1}, {"a": 3}], "a") == {"median": 2.0, "iqr": 1.0, "min": 1, "max": 3}
