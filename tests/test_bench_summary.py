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


def test_policy_tables_are_consistent():
    """Every policy the bench names (default lists per mix, sampler variants)
    has an engine row; every engine row's boot overrides are real boot keys;
    every sampler variant's keys are set_hwc_sampler arguments; every mix
    with a static split has one."""
    import inspect

    from pbs_amd.bench.corun import MIXES, POLICY_ENGINES, SAMPLER, STATIC_SE
    from pbs_amd.core.config import BOOT_KEYS
    from pbs_amd.runtime.gpu import GpuContext
    import bench
    src = inspect.getsource(bench)
    for pol in SAMPLER:
        assert pol in POLICY_ENGINES, pol
    args = set(inspect.signature(GpuContext.set_hwc_sampler).parameters) - {"self"}
    for pol, smp in SAMPLER.items():
        if smp != "model":
            assert set(smp) <= args, (pol, smp)
    for pol, (nctx, over, _, _) in POLICY_ENGINES.items():
        assert nctx >= 1
        assert set(over) <= set(BOOT_KEYS) | {"adapt", "atc"}, (pol, set(over) - set(BOOT_KEYS))
    # the per-mix default policy lists in bench.py
    start = src.index('default = {"4mix"')
    block = src[start:src.index("}[mix]", start)]
    for mix in ("4mix", "gemm2", "phase", "phase-ts", "8mix"):
        assert f'"{mix}"' in block and mix in MIXES, mix
    import re
    for lst in re.findall(r'"([a-z0-9,+\-]+)"', block):
        for pol in lst.split(","):
            if pol in MIXES:
                continue
            assert pol in POLICY_ENGINES or pol in ("none", "static", "static-se"), pol
    for mix in MIXES:
        if mix != "gemm2":
            assert mix in STATIC_SE, mix
