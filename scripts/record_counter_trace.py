"""Record a counter trace of the PBS metric path on a real MI355X: the
per-period, per-tenant (instructions, L2 misses) deltas the engine's metric
tick received from the live, ownership-attributed CDNA4 counters, and the
adapt decisions it took (pbs_amd/utils/replay.py; replayed on CPU by
tests/test_replay.py).

    python scripts/record_counter_trace.py --policy gpbs-ts --steps 10 --out tests/data/trace.json
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPU_MAX_HW_QUEUES"] = str(max(8, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--policy", default="gpbs-ts")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from pbs_amd.counters import hwc
    assert hwc.init(gpu=0), "hardware counter init failed"
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    assert hwc.start(), "hardware counter start failed"
    from pbs_amd import build
    build.build_all()
    from pbs_amd.bench import corun as CR
    from pbs_amd.core.config import MI355X_PROFILE
    from pbs_amd.utils import replay
    cfg = CR.CorunConfig(steps=a.steps, warmup=a.warmup, policies=(a.policy,), hw_counters=True)
    c = CR.Corun(cfg, log=lambda *x: print(*x, file=sys.stderr, flush=True))
    c.calibrate()
    e = c.engines[a.policy]
    e.trace_set_mask(["METRIC", "ADAPT"])
    res = c.run_policy(a.policy, a.steps, a.warmup)
    nctx, over, _, table = CR.POLICY_ENGINES[a.policy]
    prof = dict(MI355X_PROFILE)
    prof.update(over)
    opts = table.split(",")
    slots = CR.SE8_SLOTS if "se8" in opts else CR.SE_SLOTS if "se" in opts else {}
    tenants = [("Domain-0", 1)] + [(n, slots.get(n, ns)) for n, ns in c.tenants]
    doc = replay.capture(e, prof, [(0, x, k) for x in range(8) for k in range(nctx)], tenants, c.tid,
                         source=f"MI355X, bench corun policy {a.policy}, {a.steps}+{a.warmup} steps of "
                                f"{cfg.step_ms} ms, live counters; aggregate {res['aggregate']:.3f}")
    c.close()
    replay.save(doc, a.out)
    print(f"recorded {len(doc['metric'])} metric records, {len(doc['adapt'])} adapt decisions -> {a.out}")


if __name__ == "__main__":
    main()
