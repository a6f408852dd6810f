"""Counter-trace record and replay (FakeCounterSource).

A trace is what the engine's metric tick saw on a real MI355X: for every
metric period, every tenant's (instructions, L2 misses) deltas -- the
TRC_METRIC records -- plus the PBS decisions they produced (TRC_ADAPT).
``FakeCounterSource`` feeds the recorded deltas back through the engine's
counter backend on a simulated clock, one period per metric tick, so the
PBS detector can be re-run on CPU against recorded hardware behaviour:
``replay()`` returns the adapt decisions, which must equal the recorded ones
(the detector is a pure function of its inputs), and new policies can be
evaluated offline against real counter traces.

Trace document (JSON)::

    {"profile": {...engine kwargs...}, "partitions": [[gpu, xcd, ctx], ...],
     "tenants": [[name, nslots], ...], "tids": {name: id},
     "metric": [[t_ns, tenant, inst, miss, rate], ...],
     "adapt":  [[t_ns, tenant, old_us, new_us, phase_err], ...],
     "source": "..."}
"""
from __future__ import annotations

import ctypes as C
import json
from typing import Dict, List, Optional

from .. import _native as N


def capture(engine, profile: Dict, partitions: List, tenants: List, tids: Dict[str, int], source: str = "") -> Dict:
    """Build a trace document from an engine whose trace mask included
    METRIC and ADAPT for its whole life (``engine.trace_set_mask``)."""
    recs = engine.trace(max_records=1 << 21, from_start=True)
    if getattr(engine, "trace_lost", 0):
        raise RuntimeError(f"trace ring wrapped ({engine.trace_lost} records lost): record a shorter run")
    metric = [[r.t_ns, r.a[0], r.a[1], r.a[2], r.a[3]] for r in recs if r.event == "METRIC"]
    adapt = [[r.t_ns, r.a[0], r.a[1], r.a[2], r.a[3]] for r in recs if r.event == "ADAPT"]
    return {"profile": profile, "partitions": [list(p) for p in partitions], "tenants": [list(t) for t in tenants],
            "tids": dict(tids), "metric": metric, "adapt": adapt, "source": source}


def periods(doc: Dict) -> List[Dict[int, tuple]]:
    """Group the METRIC records into metric periods: one record per tenant
    per tick, emitted in tenant order, so a new period starts when a tenant
    id repeats."""
    out: List[Dict[int, tuple]] = []
    cur: Dict[int, tuple] = {}
    for _, t, inst, miss, _rate in doc["metric"]:
        if t in cur:
            out.append(cur)
            cur = {}
        cur[t] = (int(inst), int(miss))
    if cur:
        out.append(cur)
    return out


class FakeCounterSource:
    """Engine counter backend that replays recorded per-period deltas."""

    def __init__(self, per_period: List[Dict[int, tuple]]):
        self.per = per_period
        self.k = 0
        self._cb = N.COUNTER_TENANT_DELTAS(self._deltas)
        self.ops = N.CounterOps()
        self.ops.user = None
        self.ops.tenant_deltas = self._cb

    def _deltas(self, _user, n, ids, out):
        rec = self.per[self.k] if self.k < len(self.per) else {}
        self.k += 1
        for i in range(n):
            inst, miss = rec.get(ids[i], (0, 0))
            out[4 * i + 0] = inst
            out[4 * i + 1] = 0
            out[4 * i + 2] = 0
            out[4 * i + 3] = miss
        return 0


def replay(doc: Dict, periods_max: Optional[int] = None, **overrides) -> Dict:
    """Re-run the PBS detector of a fresh simulated-clock engine on the
    trace's counter deltas.  Returns {"adapt": [[tenant, old, new, phase_err]],
    "periods": n, "tslice": {tenant: final}} (engine overrides, e.g. another
    ``adapt`` dict, evaluate a different policy on the same trace)."""
    from ..core.engine import Engine
    prof = dict(doc["profile"])
    prof.update(overrides)
    prof["sim_clock"] = True
    e = Engine(**prof)
    try:
        for g, x, c in doc["partitions"]:
            e.pool_assign(0, e.partition_add(g, x, c))
        ids = {}
        for name, ns in doc["tenants"]:
            ids[name] = e.tenant_create(name, nslots=ns)
        if any(ids.get(k) != int(v) for k, v in doc["tids"].items()):
            raise RuntimeError(f"tenant ids differ from the recording: {ids} vs {doc['tids']}")
        per = periods(doc)
        if periods_max is not None:
            per = per[:periods_max]
        src = FakeCounterSource(per)
        e.trace_set_mask(["ADAPT"])
        e.set_counter_ops(src.ops)
        for name, t in ids.items():
            if name != "Domain-0":
                e.wake(t)
        period_ns = int(prof.get("metric_period_us", 1000)) * 1000
        t = 0
        while src.k < len(per):
            t += period_ns
            e.advance(t)
        e.set_counter_ops(None)
        recs = e.trace(max_records=1 << 20, from_start=True)
        adapt = [[r.a[0], r.a[1], r.a[2], r.a[3]] for r in recs if r.event == "ADAPT"]
        return {"adapt": adapt, "periods": src.k,
                "tslice": {name: e.tenant_info(t).tslice_us for name, t in ids.items()}}
    finally:
        e.close()


def load(path: str) -> Dict:
    with open(path) as f:
        return json.load(f)


def save(doc: Dict, path: str):
    with open(path, "w") as f:
        json.dump(doc, f)
