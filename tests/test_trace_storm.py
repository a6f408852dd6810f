"""scripts/trace_storm.py on a synthetic engine-trace dump (the layout
pbs_amd/bench/corun.py writes under GPBS_DIAG_DIR): per-tenant STEAL /
MIGRATE / SLEEP / WAKE counts after the last CLASS record, SLEEP bursts."""
import gzip
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def test_counts_and_bursts(tmp_path):
    import trace_storm
    t0 = 1_000_000_000
    recs = [[t0, "SWITCH", 0, 1, 1, 1000, 0],   # before the layout: not counted
            [t0 + 1, "STEAL", 0, 1, 0, 1, 0],
            [t0 + 10, "CLASS", 0, 1, 0, 16, 0]]
    # two SLEEP bursts of tenant 1 (3 records 50 us apart, then one 1 ms later), one steal of tenant 2
    for i in range(3):
        recs.append([t0 + 1_000_000 + i * 50_000, "SLEEP", 3, 1, i, 3, 0])
    recs.append([t0 + 2_000_000, "SLEEP", 4, 1, 3, 4, 0])
    recs.append([t0 + 2_100_000, "STEAL", 5, 2, 0, 6, 5])
    recs.append([t0 + 2_200_000, "MIGRATE", 5, 2, 0, 6, 5])
    p = tmp_path / "trace_gpbs_01.json.gz"
    with gzip.open(p, "wt") as f:
        json.dump({"tid": {"gemm": 1, "gemm_b": 2}, "aggregate": 1.25, "trace": recs}, f)
    a = trace_storm.analyse(str(p))
    assert a["aggregate"] == 1.25
    assert a["tenants"]["gemm"] == {"STEAL": 0, "MIGRATE": 0, "SLEEP": 4, "WAKE": 0, "sleep_bursts": 2}
    assert a["tenants"]["gemm_b"]["STEAL"] == 1 and a["tenants"]["gemm_b"]["MIGRATE"] == 1
    assert a["span_ms"] == 2.2  # from the CLASS record on
