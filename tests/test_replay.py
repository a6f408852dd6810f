"""Counter-trace replay: the PBS detector re-run on CPU
against counter deltas recorded from live MI355X hardware counters takes
exactly the decisions the engine took on the GPU (FakeCounterSource on a
simulated clock), and a synthetic trace exercises the same path without a
recording."""
import os

import pytest

from pbs_amd.core.config import MI355X_PROFILE
from pbs_amd.utils import replay

HERE = os.path.dirname(os.path.abspath(__file__))
TRACE = os.path.join(HERE, "data", "counter_trace_gpbs_ts.json")


def _synthetic(nper=400):
    """Two tenants: a steady memory-bound one and one that alternates
    between phases every 50 periods, plus an idle stretch."""
    prof = dict(MI355X_PROFILE)
    prof.update(class_split=2, idle_skip=1)
    metric = []
    for k in range(nper):
        t = k * 1_000_000
        metric.append([t, 0, 0, 0, 0])                       # Domain-0
        metric.append([t, 1, 4_000_000, 4_000_000 // 1, 0])  # memory-bound: 1e5 misses / 100k inst
        if 200 <= k < 240:
            metric.append([t, 2, 0, 0, 0])                   # idle stretch (Q14 skips it)
        else:
            hot = (k // 50) % 2
            metric.append([t, 2, 9_000_000, 9_000_000 // (3 if hot else 500), 0])
    return {"profile": prof, "partitions": [[0, x, c] for x in range(8) for c in range(4)],
            "tenants": [["Domain-0", 1], ["mem", 8], ["phased", 8]],
            "tids": {"Domain-0": 0, "mem": 1, "phased": 2}, "metric": metric, "adapt": [], "source": "synthetic"}


def test_replay_is_deterministic_and_adapts_on_a_synthetic_trace():
    doc = _synthetic()
    a = replay.replay(doc)
    b = replay.replay(doc)
    assert a == b
    assert a["periods"] == 400
    assert a["adapt"], a
    # the memory-bound tenant is driven up to the quantum ceiling, the phased
    # one moves both ways
    assert a["tslice"]["mem"] == MI355X_PROFILE["adapt"]["max_us"], a["tslice"]
    ph = [(old, new) for t, old, new, _ in a["adapt"] if t == 2]
    assert any(n > o for o, n in ph) and any(n < o for o, n in ph), ph


@pytest.mark.skipif(not os.path.exists(TRACE), reason="no recorded MI355X trace")
def test_recorded_mi355x_trace_reproduces_the_gpu_decisions():
    doc = replay.load(TRACE)
    per = replay.periods(doc)
    assert len(per) > 200 and doc["adapt"], doc["source"]
    # hardware-measured inputs: the memory-class tenants' misses per 100k
    # instructions are far above the compute tenant's in the recording
    tot = {}
    for p in per:
        for t, (i, m) in p.items():
            a = tot.setdefault(t, [0, 0])
            a[0] += i
            a[1] += m
    tid = {k: int(v) for k, v in doc["tids"].items()}
    rate = {n: tot[t][1] * 1e5 / tot[t][0] for n, t in tid.items() if t in tot and tot[t][0]}
    assert rate["hbm"] > 10 * rate["gemm"] and rate["coll"] > 5 * rate["gemm"], rate
    out = replay.replay(doc)
    rec = [a[1:] for a in doc["adapt"]]
    assert out["adapt"][:len(rec)] == rec, (len(out["adapt"]), len(rec))
