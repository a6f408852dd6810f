#!/usr/bin/env python3
"""gpbs headline benchmark (driver contract).

    python bench.py --gpus N --steps K --warmup W

Runs the BASELINE.json metric — co-run slowdown vs solo + aggregate
throughput of the 4-tenant mix (MFMA GEMM + HBM stream + all-reduce + idle)
per MI355X — under the gpbs PBS adaptive credit scheduler, one rank per GPU
(weak scaling: every GPU hosts its own 4-tenant mix; the all-reduce tenant
spans all GPUs over RCCL/xGMI when N > 1).  Rank 0 prints ONE JSON line.

``value`` = aggregate normalized throughput summed over all GPUs
(sum over tenants of solo_time/co-run_time, "solo-equivalents"; higher is
better).  Comparison policies (none = default hardware sharing, static =
equal XCD split) are measured on the same box and reported alongside.
Data: synthetic random-init bf16 tensors of the named shapes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# one HW queue per tenant/scheduler stream (see pbs_amd/runtime/gpu.py)
os.environ["GPU_MAX_HW_QUEUES"] = str(max(8, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--policies", default="none,static,gpbs-ctx2,gpbs-spatial,gpbs", help="comma list; gpbs is the reported policy")
    ap.add_argument("--target-ms", type=float, default=30.0)
    ap.add_argument("--table", default="host", choices=["host", "device"])
    ap.add_argument("--out", default="")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank control-flow rehearsal on ONE GPU: every rank on cuda:0, gloo for the default "
                         "group and the all-reduce tenant (CPU tensors); numbers are not a measurement")
    ap.add_argument("--counters", default="model", choices=["model", "hw"],
                    help="PBS metric source: modeled per-tile counters, or live CDNA4 hardware counters "
                         "(rocprofiler-sdk device counting) attributed by the model")
    ap.add_argument("--mix", default="4mix", choices=["4mix", "gemm2"],
                    help="4mix: BASELINE config #3/#4 (headline); gemm2: config #2 (two 4096^2 GEMM tenants)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world == 1:
        print("bench.py: --gpus > 1 must be launched with torch.distributed.run (one rank per GPU)", file=sys.stderr)
        sys.exit(2)
    if args.rehearse:
        local = 0
    if args.counters == "hw":  # must register with rocprofiler before the HIP runtime starts
        from pbs_amd.counters import hwc
        if not hwc.init(gpu=local):
            print("bench.py: hardware counter init failed", file=sys.stderr)
            sys.exit(3)
    torch.cuda.set_device(local)
    if args.counters == "hw":
        torch.zeros(1, device="cuda")
        if not hwc.start():
            print("bench.py: hardware counter start failed", file=sys.stderr)
            sys.exit(3)
    groups = {}
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.rehearse:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        groups["ctrl"] = dist.new_group(backend="gloo")
        groups["gang"] = dist.new_group(backend="gloo")  # cross-GPU gang epochs (own thread)
        groups["coll"] = dist.new_group(backend="gloo" if args.rehearse else "nccl")

    from pbs_amd import build
    if rank == 0:  # one builder per node; the others wait (no concurrent relink)
        build.build_all()
    if world > 1:
        dist.barrier(group=groups["ctrl"])
    from pbs_amd.bench.corun import Corun, CorunConfig

    pols = tuple(p for p in args.policies.split(",") if p)
    if "gpbs" not in pols:
        pols = pols + ("gpbs",)
    cfg = CorunConfig(steps=args.steps, warmup=args.warmup, target_ms=args.target_ms, policies=pols,
                      table_mode=args.table, mix=args.mix, hw_counters=(args.counters == "hw"))
    if args.rehearse:
        cfg.coll_bytes = 4 << 20  # CPU gloo all-reduce stand-in
    log = (lambda *a: print(*a, file=sys.stderr, flush=True))
    c = Corun(cfg, rank=rank, world=world, device=local, groups=groups, log=log, coll_on_cpu=args.rehearse)
    c.calibrate()
    results = {}
    for p in pols:
        results[p] = c.run_policy(p, args.steps, args.warmup)
    g = results["gpbs"]
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    value = g["aggregate_all_gpus"]
    line = {
        "metric": base["metric"],
        "value": round(value, 4),
        "unit": "solo-equivalents (sum over GPUs and throughput tenants of solo_time/co-run_time)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(g["ms_per_step"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random-init bf16 tensors; 4096^3 GEMM, 1 GiB stream, 256 MiB reduce/all-reduce, "
                "8192^2 GEMV)",
        "config": {"model": ("4-tenant mix (MFMA GEMM + HBM-stream + all-reduce + idle)" if args.mix == "4mix"
                             else "2 bf16 4096^2 GEMM tenants"),
                   "global_batch": world * 4, "seq_len": 0, "parallelism": f"dp{world}" if world > 1 else "dp1",
                   "tenants_per_gpu": 4 if args.mix == "4mix" else 2, "policy": "gpbs-pbs-credit", "mix": args.mix},
        "mean_slowdown_pct": round(g["mean_slowdown_pct"], 2),
        "per_tenant": g["tenants"],
        "policies": {p: {"aggregate_all_gpus": round(r["aggregate_all_gpus"], 4),
                         "mean_slowdown_pct": round(r["mean_slowdown_pct"], 2),
                         "ms_per_step": round(r["ms_per_step"], 3)} for p, r in results.items()},
        "solo_unit_ms": {k: round(v, 4) for k, v in c.solo_unit_ms.items()},
        "engine": g.get("engine", {}),
    }
    c.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump({"line": line, "results": results}, f, indent=1)
    if world > 1:
        import torch.distributed as dist
        dist.barrier(group=groups["ctrl"])
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
