"""Scheduler-state snapshot / restore.

The reference saves domains (X:tools/libxc/xc_domain_save.c) but never the
scheduler state; a moved domain even loses its PBS fields (Q4).  gpbs
snapshots what a restarted daemon needs to resume scheduling identically:
pools (scheduler, partitions, tslice/ratelimit), tenants (pool, slots,
weight/cap, pause, per-slot affinity) and the PBS adaptation state (quantum,
phase, 5-sample window) of every tenant.  JSON, written atomically.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import tempfile
from typing import Any, Dict, Optional

from .. import _native as N

VERSION = 1


def _adapt_to_dict(s: N.AdaptState) -> Dict[str, Any]:
    return {"tslice_us": s.tslice_us, "tick_period_us": s.tick_period_us, "window_left": s.window_left,
            "stable_count": s.stable_count, "phase": s.phase, "last_err": s.last_err, "last_curr": s.last_curr,
            "last_win": s.last_win, "filter": [[f.spin, f.inst, f.miss] for f in s.filter]}


def _dict_to_adapt(d: Dict[str, Any]) -> N.AdaptState:
    s = N.AdaptState()
    for k in ("tslice_us", "tick_period_us", "window_left", "stable_count", "phase", "last_err", "last_curr",
              "last_win"):
        setattr(s, k, int(d[k]))
    for i, (sp, ins, mi) in enumerate(d["filter"]):
        s.filter[i].spin, s.filter[i].inst, s.filter[i].miss = sp, ins, mi
    return s


def slot_affinity(engine, sid: int):
    o = N.SlotInfo()
    engine.lib.gpbs_slot_info(engine.h, sid, C.byref(o))
    return [i for i in range(256) if (o.affinity[i // 64] >> (i % 64)) & 1]


def capture(engine, extra: Optional[Dict] = None) -> Dict[str, Any]:
    doc: Dict[str, Any] = {"version": VERSION, "now_ns": engine.now(), "pools": [], "tenants": [],
                           "extra": extra or {}}
    for p in engine.pools():
        info = engine.pool_info(p)
        ts, rl = engine.sched_params_get(p)
        ent = {"id": p, "name": info["name"], "sched": info["sched"], "cpus": info["cpus"],
               "tslice_us": ts, "ratelimit_us": rl}
        if info["sched"] == "arinc653":  # an installed ARINC 653 table (by tenant NAME: ids change on restore)
            a = engine.arinc653_get(p)
            if a["explicit"]:
                ent["arinc653"] = {"major_frame_us": a["major_frame_us"],
                                   "entries": [[engine.tenant_info(t).name, sl, rt] for t, sl, rt in a["entries"]]}
        doc["pools"].append(ent)
    for t in engine.tenants():
        i = engine.tenant_info(t)
        ent = {"id": t, "name": i.name, "pool": i.pool, "slots": i.nslots, "weight": i.weight, "cap": i.cap,
               "paused": i.paused, "affinity": [slot_affinity(engine, engine.slot_id(t, k)) for k in range(i.nslots)]}
        try:
            ent["adapt"] = _adapt_to_dict(engine.adapt_state(t))
        except Exception:
            pass
        doc["tenants"].append(ent)
    return doc


def save(engine, path: str, extra: Optional[Dict] = None) -> str:
    doc = capture(engine, extra)
    d = os.path.dirname(os.path.abspath(path))
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".gpbs-snap-")
    with os.fdopen(fd, "w") as f:
        json.dump(doc, f, indent=1)
    os.replace(tmp, path)
    return path


def restore(engine, path_or_doc) -> Dict[str, Any]:
    doc = path_or_doc
    if isinstance(path_or_doc, str):
        with open(path_or_doc) as f:
            doc = json.load(f)
    if doc.get("version") != VERSION:
        raise ValueError(f"unsupported snapshot version {doc.get('version')}")
    pool_map = {}
    existing = {engine.pool_info(p)["name"]: p for p in engine.pools()}
    # pools: recreate, then move partitions to their recorded pool
    for p in doc["pools"]:
        pid = existing.get(p["name"])
        if pid is None:
            pid = engine.pool_create(p["name"], p["sched"])
        pool_map[p["id"]] = pid
    for p in doc["pools"]:
        pid = pool_map[p["id"]]
        for c in p["cpus"]:
            if c >= engine.num_partitions:
                continue
            owner = engine.partition_info(c)["pool"]
            if owner == pid:
                continue
            if owner >= 0:
                try:
                    engine.pool_unassign(owner, c)
                except Exception:
                    continue
            engine.pool_assign(pid, c)
    for p in doc["pools"]:
        try:
            engine.sched_params_set(pool_map[p["id"]], p["tslice_us"], p["ratelimit_us"])
        except Exception:
            pass
    names = {engine.tenant_info(t).name: t for t in engine.tenants()}
    for t in doc["tenants"]:
        pid = pool_map.get(t["pool"], 0)
        tid = names.get(t["name"])
        if tid is None:
            tid = engine.tenant_create(t["name"], nslots=t["slots"], pool=pid)
        elif engine.tenant_info(tid).pool != pid:
            engine.tenant_move(tid, pid)
        engine.sched_credit_set(tid, t["weight"], t["cap"])
        for k, aff in enumerate(t.get("affinity", [])):
            if aff and len(aff) < 256 and k < engine.tenant_info(tid).nslots:
                valid = [c for c in aff if c < engine.num_partitions]
                if valid:
                    engine.pin(tid, k, valid)
        if "adapt" in t:
            try:
                engine.set_adapt_state(tid, _dict_to_adapt(t["adapt"]))
            except Exception:
                pass
        cur = engine.tenant_info(tid).paused
        for _ in range(max(0, t.get("paused", 0) - cur)):
            engine.pause(tid)
    names = {engine.tenant_info(t).name: t for t in engine.tenants()}
    for p in doc["pools"]:
        a = p.get("arinc653")
        if a:
            try:
                engine.arinc653_set(pool_map[p["id"]], a["major_frame_us"],
                                    [(names[n], sl, rt) for n, sl, rt in a["entries"] if n in names])
            except Exception:
                pass
    return doc
