"""Multi-GPU pre-flight record of bench.py (VERDICT r3 missing #3 / item 5):
every rank reports the agent it counts on (by PCI address, cross-checked
against its HIP device), whether its all-reduce tenant passed the IPC
self-test or fell back, its gang transport statistics and the node totals.
Checked on the committed 8-rank rehearsal (every rank on one MI355X,
``bench.py --rehearse-ipc``, profiles/r4/rehearse8_1gpu.json); the per-rank
fields are produced by bench.py and are the same at N = 8 on a node."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REHEARSAL = os.path.join(ROOT, "profiles", "r4", "rehearse8_1gpu.json")


def _line():
    if not os.path.exists(REHEARSAL):
        pytest.skip("no committed 8-rank rehearsal record")
    with open(REHEARSAL) as f:
        for ln in f:
            if ln.startswith("{"):
                return json.loads(ln)
    pytest.fail("no JSON line in the rehearsal record")


def test_every_rank_reports_its_preflight_fields():
    line = _line()
    ranks = line["ranks"]
    assert line["n_gpus"] == 8 and len(ranks) == 8
    assert sorted(r["rank"] for r in ranks) == list(range(8))
    for r in ranks:
        assert r["device_bdf"] and r["gpu_state_source"] in ("amdsmi", "sysfs", None)
        if r["counters"] == "hw":  # counted agent chosen by PCI address = the rank's device
            assert r["hwc_agent"]["bdf"] == r["device_bdf"], r
            assert r["hwc_agent"]["agent_index"] >= 0
        for mix, d in r["mixes"].items():
            assert d["coll"] in ("ipc", "rccl-fallback", "rccl", "gloo-cpu"), d
            assert d["ipc_selftest"] in ("ok", "failed"), d  # --rehearse-ipc runs the self-test
            g = d["gang"]
            assert g is not None and {"sync_p50_us", "sync_p99_us", "timeouts", "transport"} <= set(g), g
            assert g["timeouts"] == 0
            assert d.get("node_totals"), d
            for t in d["node_totals"].values():
                assert {"inst", "l2_misses", "miss_rate"} <= set(t)


def test_ranks_agree_on_node_totals():
    """node totals are the SUM over ranks of the cumulative counters at the
    last exchange: the ranks' records of the same mix agree (up to the last
    exchange each saw)."""
    line = _line()
    for mix in line["ranks"][0]["mixes"]:
        tots = [r["mixes"][mix]["node_totals"] for r in line["ranks"]]
        names = set(tots[0])
        assert all(set(t) == names for t in tots)
