#!/usr/bin/env python3
"""gpbs headline benchmark (driver contract).

    python bench.py --gpus N --steps K --warmup W

Runs the BASELINE.json metric -- co-run slowdown vs solo + aggregate
throughput of the 4-tenant mix (MFMA GEMM + HBM stream + all-reduce + idle)
per MI355X -- under the gpbs PBS adaptive credit scheduler, one rank per GPU
(weak scaling: every GPU hosts its own mix; at N > 1 the all-reduce tenant
spans all GPUs over xGMI -- a gpbs kernel on IPC-mapped peer buffers, gated
per workgroup like every tenant, with RCCL as --coll rccl and as the fallback
when its one-unit self-test fails).  Rank 0 prints ONE JSON line.

``value`` = aggregate normalized throughput of the headline mix summed over
all GPUs (sum over throughput tenants of co-run rate / solo rate,
"solo-equivalents"; higher is better).  Solo rates are measured with the
same steady protocol as the co-run (backlogged, W + K windows, alone).
Comparison policies run on the same box, 5 randomized reps each: none
(default hardware sharing), static (equal XCD split), static-se (the
hand-picked shader-engine layout, no engine, no counters), the PBS ablations
(credit-fixed*: fixed quantum; gpbs-split: crowded class regions split by
XCD blocks instead of time-shared) and gpbs-lat (latency hold).

By default two more mixes run after the headline and are reported under
``mixes``: "phase" (a tenant alternating GEMM <-> stream every 300 ms and a
stream tenant stopping / starting every 500 ms: the counter-driven layout
must follow, a static one cannot) and "8mix" (config #4's 8 tenants on one
GPU: classes must time-share their shader engines, where PBS quanta apply).
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
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("GPBS_HWQ") or str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def q(xs, f):
    xs = sorted(xs)
    k = (len(xs) - 1) * f
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)



def summ(rs, key):
    xs = [r[key] for r in rs]
    return {"median": round(q(xs, 0.5), 4), "iqr": round(q(xs, 0.75) - q(xs, 0.25), 4),
            "min": round(min(xs), 4), "max": round(max(xs), 4)}


def mix_summary(mix, runs, solo, reps):
    gr = sorted(runs["gpbs"], key=lambda r: r["aggregate_all_gpus"])
    g = gr[(len(gr) - 1) // 2]  # headline run = the gpbs run with the median aggregate
    pol = {p: {"aggregate_all_gpus": summ(rs, "aggregate_all_gpus"),
               "mean_slowdown_pct": summ(rs, "mean_slowdown_pct"),
               "ms_per_step": round(q([r["ms_per_step"] for r in rs], 0.5), 3),
               "runs": [round(r["aggregate_all_gpus"], 4) for r in rs]} for p, rs in runs.items()}
    for p, rs in runs.items():
        eng = [r.get("engine") for r in rs if r.get("engine")]
        if eng:
            pol[p]["adapt_rearm"] = [e.get("adapt_rearm", 0) for e in eng]
            pol[p]["adapt_inc"] = [e.get("adapt_inc", 0) for e in eng]
            pol[p]["adapt_dec"] = [e.get("adapt_dec", 0) for e in eng]
            pol[p]["relayout"] = [e.get("relayout", 0) for e in eng]
            # the quantum each contention class ran with (class 0 compute, 1 memory)
            by = {}
            for e in eng:
                for n, ts in (e.get("mean_tslice_us") or {}).items():
                    c = (e.get("class") or {}).get(n, -1)
                    if n != "idle" and c >= 0:
                        by.setdefault(str(c), []).append(ts)
            pol[p]["mean_tslice_us_by_class"] = {c: round(q(v, 0.5), 1) for c, v in sorted(by.items())}
        if "idle" in rs[0]["tenants"]:
            pol[p]["idle_p50_ms"] = round(q([r["tenants"]["idle"]["p50_ms"] for r in rs], 0.5), 4)
            pol[p]["idle_p99_ms"] = round(q([r["tenants"]["idle"]["p99_ms"] for r in rs], 0.5), 4)
    # drift over the mix's runs (chronological): the last five gpbs runs
    # against the first five, and the GPU state of the first and last run
    xs = [r["aggregate_all_gpus"] for r in runs["gpbs"]]
    if len(xs) >= 6:
        k = min(5, len(xs) // 2)
        f, l = xs[:k], xs[-k:]
        out_drift = {"first_median": round(q(f, 0.5), 4), "last_median": round(q(l, 0.5), 4),
                     "first_iqr": round(q(f, 0.75) - q(f, 0.25), 4), "n": k}
        out_drift["last_within_first_iqr"] = abs(out_drift["last_median"] - out_drift["first_median"]) <= \
            max(out_drift["first_iqr"], 1e-9)
    else:
        out_drift = None
    gs = [r.get("gpu_state") for r in runs["gpbs"] if r.get("gpu_state")]
    if gs:
        pick = ("gfxclk_mhz", "power_w", "ppt_frac", "temp_hotspot_c_max")
        out_gs = {"first_run": {k: gs[0].get(k) for k in pick}, "last_run": {k: gs[-1].get(k) for k in pick}}
    else:
        out_gs = None
    out = {"value": round(q([r["aggregate_all_gpus"] for r in runs["gpbs"]], 0.5), 4),
           "mean_slowdown_pct": round(q([r["mean_slowdown_pct"] for r in runs["gpbs"]], 0.5), 2),
           "reps": max(1, reps), "policies": pol, "per_tenant": g["tenants"], "engine": g.get("engine", {}),
           "ms_per_step": round(g["ms_per_step"], 3), "solo": solo, "drift": out_drift, "gpu_state": out_gs}
    from pbs_amd.bench.corun import MIXES
    if MIXES.get(mix, {}).get("slo_p99_ms"):  # in-region latency tenant: its p99 target
        out["slo"] = MIXES[mix]["slo_p99_ms"]
        for p, v in pol.items():
            if "idle_p99_ms" in v:
                v["slo_met"] = v["idle_p99_ms"] <= out["slo"]
    if "static-se" in runs:
        a, b = pol["gpbs"]["aggregate_all_gpus"], pol["static-se"]["aggregate_all_gpus"]
        out["gpbs_vs_static_se"] = {"delta_median": round(a["median"] - b["median"], 4),
                                    "iqr_gpbs": a["iqr"], "iqr_static_se": b["iqr"],
                                    "beats_by_more_than_iqr": a["median"] - b["median"] > max(a["iqr"], b["iqr"])}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--policies", default="",
                    help="comma list for the headline mix (default: per-mix list below); gpbs is the reported policy")
    ap.add_argument("--keep-engines", action="store_true",
                    help="one engine per policy for the whole process (default: a fresh engine per timed run)")
    ap.add_argument("--reps", type=int, default=5,
                    help="timed runs per policy, in a randomized order per repetition (median and IQR reported)")
    ap.add_argument("--seed", type=int, default=20261016, help="policy-order shuffle seed (same on every rank)")
    ap.add_argument("--target-ms", type=float, default=30.0)
    ap.add_argument("--protocol", default="steady", choices=["steady", "quota"],
                    help="steady: tenants backlogged over common step windows (weighted speedup, default); "
                         "quota: round-1 fixed per-step quotas (early finishers idle)")
    ap.add_argument("--step-ms", type=float, default=80.0, help="steady protocol: step window length")
    ap.add_argument("--gang-transport", default="shm", choices=["shm", "dist", "xgmi"],
                    help="N > 1 gang epochs: native shared memory among the node's ranks, or the 'gang' process "
                         "group (gloo; RCCL over xGMI with --gang-rccl)")
    ap.add_argument("--gang-rccl", action="store_true", help="with --gang-transport dist: the gang group is RCCL")
    ap.add_argument("--gang-wait-driven", action="store_true",
                    help="N > 1: the all-reduce tenant gets aligned gang windows only while its K10 wait reports "
                         "(peer-arrival skew of its RCCL all-reduces) say its peers lag")
    ap.add_argument("--table", default="host", choices=["host", "device"])
    ap.add_argument("--coll", default="ipc", choices=["ipc", "rccl"],
                    help="N > 1 all-reduce tenant: ipc (gated gpbs kernel over IPC-mapped peer buffers, xGMI; "
                         "default) or rccl (torch.distributed all-reduce, not CU-confined)")
    ap.add_argument("--resolo", dest="resolo", action="store_true", default=True,
                    help="measure the solo rates again after each mix's runs (reported as "
                         "solo._end_over_start_rate, not used): a GPU that got slower over the runs shows here "
                         "(default on)")
    ap.add_argument("--no-resolo", dest="resolo", action="store_false")
    ap.add_argument("--out", default="")
    ap.add_argument("--no-cu-check", dest="cu_check", action="store_false",
                    help="skip the CU-mask layout check (scripts/cu_map_check.py) run before the bench")
    ap.add_argument("--rehearse-ipc", action="store_true",
                    help="like --rehearse (every rank on GPU 0, gloo) but with the gated IPC all-reduce tenant on "
                         "the GPU: rehearses the whole N > 1 path (IPC self-test, P2P-flag barrier, gang epochs, "
                         "agreed stop) on one GPU; numbers are not a measurement")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank control-flow rehearsal on ONE GPU: every rank on cuda:0, gloo for the default "
                         "group and the all-reduce tenant (CPU tensors); numbers are not a measurement")
    ap.add_argument("--counters", default="hw", choices=["model", "hw"],
                    help="PBS metric source: live CDNA4 hardware counters (rocprofiler-sdk device counting, "
                         "attributed to tenants by shader-engine ownership; default), or the modeled per-tile "
                         "counters of the tenant kernels (debug cross-check)")
    ap.add_argument("--mix", default="all", choices=["all", "4mix", "gemm2", "phase", "phase-ts", "8mix", "slo", "llm5"],
                    help="all (default): 4mix (headline, BASELINE config #3) + phase (phase-changing mix) + "
                         "phase-ts (the phase mix with a time-shared memory region, where the adaptive quantum "
                         "matters) + 8mix (config #4's 8 tenants on one GPU); gemm2: config #2 (two 4096^2 GEMM "
                         "tenants); "
                         "llm5: config #5 (Llama-3-8B fp8 decode + Llama-1B-shaped bf16 trainer, torch tenants "
                         "on the shim under gpbsd; not in the default run)")
    ap.add_argument("--reps-extra", type=int, default=5, help="reps of the non-headline mixes")
    ap.add_argument("--gemm-opts", type=int, default=-1,
                    help="GEMM tenant kernel variant bits (csrc/hip/tenant_kernels.hip g_gemm_opts; -1 = default)")
    ap.add_argument("--reduce-opts", type=int, default=-1,
                    help="reduce-copy tenant variant bits (g_reduce_opts; -1 = default)")
    ap.add_argument("--stream-opts", type=int, default=-1,
                    help="HBM-stream tenant variant bits (g_stream_opts; -1 = default)")
    ap.add_argument("--kernel-trace", action="store_true",
                    help="per-run kernel dispatch statistics from this process's own rocprofiler-sdk context "
                         "(the live counters stay on; rocprofv3 would take the SDK from them) -> --out")
    ap.add_argument("--hang-dump-s", type=float, default=0.0,
                    help="diagnostics: dump every thread's stack every this many seconds (0: off)")
    ap.add_argument("--llm5-warm-s", type=float, default=5.0, help="--mix llm5: untimed warm-up seconds")
    args = ap.parse_args()
    if args.mix == "llm5":  # its own process tree (daemon + torch tenants); nothing here touches HIP first
        return run_llm5(args)
    if args.hang_dump_s > 0:  # diagnostics: every thread's stack when a run stops progressing
        import faulthandler
        faulthandler.dump_traceback_later(args.hang_dump_s, repeat=True)

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # stdout carries exactly one line, rank 0's JSON: the process's fd 1 goes
    # to stderr until then (gloo prints its "[Gloo] Rank r is connected to N
    # peer ranks" banners to stdout from C++, one per group and rank)
    line_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.gpus > 1 and world == 1:
        print("bench.py: --gpus > 1 must be launched with torch.distributed.run (one rank per GPU)", file=sys.stderr)
        sys.exit(2)
    if args.rehearse_ipc:
        args.rehearse = True
    if args.rehearse:
        local = 0
    # the CU-mask layout every SE-exclusive policy assumes, checked on this
    # rank's device in a child process before this one touches the GPU
    # (scripts/cu_map_check.py; a rehearsal checks once, on rank 0)
    cu_map = None
    if args.cu_check and (not args.rehearse or rank == 0):
        import subprocess
        try:
            p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "cu_map_check.py"), "--device", str(local)],
                               capture_output=True, text=True, timeout=240)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            cu_map = json.loads(line[-1]) if line else {"ok": None, "rc": p.returncode, "err": p.stderr[-400:]}
        except subprocess.TimeoutExpired:
            cu_map = {"ok": None, "err": "timeout"}
        if cu_map.get("ok") is False:
            print(f"bench.py: rank {rank}: CU-mask bits do not map to shader engines as assumed: {cu_map}",
                  file=sys.stderr)
    counters = args.counters
    if counters == "hw":  # must register with rocprofiler before the HIP runtime starts
        from pbs_amd.counters import hwc
        if args.kernel_trace:
            hwc.trace_enable(True)
        if not hwc.init(gpu=local):
            print("bench.py: hardware counter init failed; falling back to modeled counters", file=sys.stderr)
            counters = "model"
    torch.cuda.set_device(local)
    if max(args.gemm_opts, args.reduce_opts, args.stream_opts) >= 0:  # tenant kernel variants (A/B runs)
        from pbs_amd.ops import kernels as _K
        _K.lib().gpbs_hip_set_gemm_opts(args.gemm_opts)  # -1 keeps
        _K.lib().gpbs_hip_set_reduce_opts(args.reduce_opts)
        _K.lib().gpbs_hip_set_stream_opts(args.stream_opts)
    if counters == "hw":
        torch.zeros(1, device="cuda")
        if not hwc.start():
            print("bench.py: hardware counter start failed; falling back to modeled counters", file=sys.stderr)
            counters = "model"
    # the GPU's clock / power / temperature / throttle residency over every
    # timed run (host thread, amdsmi or sysfs): tells a DVFS / power-state
    # drift from a queue / pipe effect
    from pbs_amd.utils.gpustate import GpuStateRecorder, bdf_mismatch, device_bdf
    bdf = device_bdf(local)
    gpustate = GpuStateRecorder(bdf, period_s=0.2).start()
    rank_diag = {"rank": rank, "local_rank": local, "device_bdf": bdf, "gpu_state_source": gpustate.source,
                 "counters": counters, "cu_map_ok": cu_map.get("ok") if cu_map else None}
    if counters == "hw":
        rank_diag["hwc_agent"] = hwc.agent()
        ag = rank_diag["hwc_agent"].get("bdf")
        if bdf_mismatch(ag, bdf):
            print(f"bench.py: rank {rank} counts on agent {rank_diag['hwc_agent']} but runs on {bdf}",
                  file=sys.stderr)
            if world == 1:
                sys.exit(3)
        elif not ag or not bdf:  # an unknown address is no evidence of a mismatch
            print(f"bench.py: rank {rank}: counted agent {ag} / device {bdf} not both known", file=sys.stderr)
    groups = {}
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.rehearse:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        groups["ctrl"] = dist.new_group(backend="gloo")
        # cross-GPU gang epochs (own thread); only used with --gang-transport dist
        groups["gang"] = dist.new_group(backend="nccl" if args.gang_rccl and not args.rehearse else "gloo")
        groups["coll"] = dist.new_group(backend="gloo" if args.rehearse else "nccl")
        # a rank counting on another GPU's agent fails the whole job, after
        # the rendezvous so no peer is left waiting in it
        bad = torch.tensor([1 if counters == "hw" and bdf_mismatch(rank_diag["hwc_agent"].get("bdf"), bdf) else 0])
        dist.all_reduce(bad, group=groups["ctrl"])
        if int(bad.item()):
            print(f"bench.py: {int(bad.item())} rank(s) count on the wrong agent", file=sys.stderr)
            dist.destroy_process_group()
            sys.exit(3)

    from pbs_amd import build
    if rank == 0:  # one builder per node; the others wait (no concurrent relink)
        build.build_all()
    if world > 1:
        dist.barrier(group=groups["ctrl"])
    # masked-queue pipe pre-flight: the burst of
    # CU-masked queues is made now -- after RCCL's communicators (one small
    # all-reduce on the coll group brings them up) -- and checked against
    # KFD's queue ids; a failed check is a rank failure in the line
    try:
        if world > 1 and not args.rehearse:
            import torch.distributed as dist
            dist.all_reduce(torch.ones(1, device="cuda"), group=groups["coll"])
            torch.cuda.synchronize()
        from pbs_amd.ops import kernels as _K
        from pbs_amd.utils.pipes import pipe_preflight
        rank_diag["pipes"] = pipe_preflight(_K.lib(), local)
    except Exception as ex:  # noqa: BLE001
        rank_diag["pipes"] = {"ok": False, "error": str(ex)[:200]}
    if not rank_diag["pipes"].get("ok"):
        print(f"bench.py: rank {rank}: masked-queue pipe pre-flight failed: {rank_diag['pipes']}", file=sys.stderr)
    from pbs_amd.bench.corun import MIXES, Corun, CorunConfig
    # gang epochs (N > 1): native shared-memory transport among the node's
    # ranks; the region name is a nonce from rank 0 so no stale region matches
    gang_base = ""
    if world > 1:
        nonce = torch.tensor([int.from_bytes(os.urandom(4), "little") if rank == 0 else 0], dtype=torch.int64)
        dist.broadcast(nonce, src=0, group=groups["ctrl"])
        gang_base = f"gpbs-gang-{int(nonce.item()):08x}"

    mixes = ["4mix", "phase", "phase-ts", "8mix", "slo"] if args.mix == "all" else [args.mix]
    log = (lambda *a: print(*a, file=sys.stderr, flush=True))
    import random

    def run_mix(mix, pols, reps):
        """Calibrate solo rates, then every policy `reps` times in a fresh
        random order per repetition (the same on every rank)."""
        if "gpbs" not in pols:
            pols = pols + ("gpbs",)
        cfg = CorunConfig(steps=args.steps, warmup=args.warmup, target_ms=args.target_ms, policies=pols,
                          table_mode=args.table, mix=mix, hw_counters=(counters == "hw"),
                          protocol=args.protocol, step_ms=args.step_ms, gang_transport=args.gang_transport,
                          gang_shm_base=f"{gang_base}-{mix}" if gang_base else "",
                          gang_wait_driven=args.gang_wait_driven, fresh_engine=not args.keep_engines,
                          coll_impl=args.coll, kernel_trace=args.kernel_trace and counters == "hw")
        if args.rehearse:
            cfg.coll_bytes = 4 << 20  # CPU gloo all-reduce stand-in
        c = Corun(cfg, rank=rank, world=world, device=local, groups=groups, log=log,
                  coll_on_cpu=args.rehearse and not args.rehearse_ipc)
        c.gpustate = gpustate
        c.calibrate()
        rng = random.Random(args.seed)
        runs = {p: [] for p in pols}
        order = []
        for _ in range(max(1, reps)):
            perm = list(pols)
            rng.shuffle(perm)
            order += perm
        for p in order:
            runs[p].append(c.run_policy(p, args.steps, args.warmup))
        solo = c.solo_report()
        if args.resolo:  # diagnostic: the solo rates again after the runs (drift over the mix)
            start = dict(c.solo_unit_ms)
            c.calibrate()
            solo["_end_over_start_rate"] = {k: round(start[k] / c.solo_unit_ms[k], 4) for k in start
                                            if k in c.solo_unit_ms and c.solo_unit_ms[k]}
            if counters == "hw" and mix == mixes[-1]:
                # the same with the device-counting context stopped and the GPU
                # idle for a second: a slowdown that survives it is not the
                # counter service's (queue state), one that goes away is
                import time as _t
                hwc.stop()
                _t.sleep(1.0)
                c.calibrate()
                solo["_end_over_start_rate_ctx_stopped"] = {
                    k: round(start[k] / c.solo_unit_ms[k], 4) for k in start
                    if k in c.solo_unit_ms and c.solo_unit_ms[k]}
            c.solo_unit_ms = start
        c.close()
        diag = dict(c.diag, gang=c.gang_stats or None)  # gang stats of the last run (recorded at its stop)
        last = [r for r in runs["gpbs"] if r.get("engine")]
        if last and last[-1]["engine"].get("node_totals"):
            diag["node_totals"] = last[-1]["engine"]["node_totals"]
        rank_diag.setdefault("mixes", {})[mix] = diag
        del c
        torch.cuda.empty_cache()
        return runs, order, solo

    results = {}
    for mix in mixes:
        # crowded mixes (phase-ts, 8mix, slo) carry the long-quantum
        # ablations on the flagship's layout: one 30 ms
        # quantum for all (credit-fixed-ts30), the class map with the 30 ms
        # floor (credit-classq-f), ATC -- and the layout ablation gpbs-ts
        # (crowded memory regions time-shared, round 6's quanta)
        default = {"4mix": "none,static-se,credit-fixed,gpbs-lat,gpbs",
                   "gemm2": "none,static,static-se,credit-fixed,gpbs",
                   "phase": "none,static-se,credit-fixed,gpbs",
                   "phase-ts": "none,static-se,credit-fixed-ts30,credit-classq-f,atc,gpbs-ts,gpbs",
                   "8mix": "none,static-se,credit-fixed-ts30,credit-classq-f,gpbs-split,atc,gpbs-ts,gpbs",
                   "slo": "none,static-se,credit-fixed-ts30,credit-classq-f,atc,gpbs-ts,gpbs"}[mix]
        spec = args.policies if (args.policies and mix == mixes[0]) else default
        pols = tuple(p for p in spec.split(",") if p)
        reps = args.reps if mix == mixes[0] else args.reps_extra
        runs, order, solo = run_mix(mix, pols, reps)
        results[mix] = {"runs": runs, "order": order, "summary": mix_summary(mix, runs, solo, reps)}

    head = mixes[0]
    hs = results[head]["summary"]
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    names = {"4mix": "4-tenant mix (MFMA GEMM + HBM-stream + all-reduce + idle)",
             "gemm2": "2 bf16 4096^2 GEMM tenants",
             "phase": "phase-changing mix (GEMM + GEMM<->stream phase tenant + on/off stream + idle)",
             "phase-ts": "time-shared phase mix (GEMM + GEMM<->stream phase tenant + on/off stream + stream + "
                         "reduce + idle)",
             "8mix": "8-tenant mix (3 GEMMs + 3 streams + all-reduce + idle)",
             "slo": "latency-SLO mix (GEMM + 2 HBM streams + MALL-resident stream + in-region latency tenant)"}
    line = {
        "metric": base["metric"],
        "value": hs["value"],
        "unit": ("solo-equivalents (sum over GPUs and throughput tenants of co-run throughput / solo throughput, "
                 "all tenants backlogged over common step windows; solo rates measured with the same protocol)"
                 if args.protocol == "steady" else
                 "solo-equivalents (sum over GPUs and throughput tenants of solo_time/co-run_time per quota step)"),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": hs["ms_per_step"],  # of the headline (median) gpbs run
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random-init bf16 tensors; 4096^3 GEMM, 1 GiB stream, 256 MiB reduce/all-reduce, "
                "8192^2 GEMV; the N=1 'all-reduce' tenant is a local reduce-copy kernel; at N>1 it is the gated "
                "all-reduce kernel over IPC-mapped peer buffers on xGMI, RCCL only as fallback or --coll rccl)",
        "config": {"model": names[head], "global_batch": world * 4, "seq_len": 0,
                   "parallelism": f"dp{world}" if world > 1 else "dp1",
                   "tenants_per_gpu": len(MIXES[head]["tenants"]),
                   "policy": "gpbs (counter-driven SE budgets, PBS credit, hw counters)", "mix": head},
        "mean_slowdown_pct": hs["mean_slowdown_pct"],
        "counters": counters,
        "protocol": {"kind": args.protocol, "step_ms": args.step_ms if args.protocol == "steady" else None,
                     "reps": max(1, args.reps), "order": "randomized per repetition", "seed": args.seed,
                     "statistic": "median over reps (IQR = q75 - q25)", "solo": "steady (same protocol, alone)"},
        "per_tenant": hs["per_tenant"],
        "policies": hs["policies"],
        "solo": hs["solo"],
        "engine": hs["engine"],
        "drift": hs["drift"],
        "gpu_state": hs["gpu_state"],
    }
    if "gpbs_vs_static_se" in hs:
        line["gpbs_vs_static_se"] = hs["gpbs_vs_static_se"]
    line["mixes"] = {m: {k: v for k, v in results[m]["summary"].items() if k not in ("per_tenant", "engine")}
                     for m in mixes[1:]}
    for m in mixes[1:]:
        line["mixes"][m]["per_tenant"] = {n: {k: v for k, v in t.items() if k != "step_norm_perf"}
                                          for n, t in results[m]["summary"]["per_tenant"].items()}
    # per-rank pre-flight record (agent / BDF, IPC self-test and fallback,
    # gang transport, node totals): a multi-GPU run diagnoses itself
    if world > 1:
        import torch.distributed as dist
        allr = [None] * world
        dist.all_gather_object(allr, rank_diag, group=groups["ctrl"])
    else:
        allr = [rank_diag]
    line["ranks"] = allr
    gpustate.stop()
    if rank == 0:
        # the detail record (every policy table, per-tenant rows, ranks, GPU
        # state) goes to --out; stdout gets the compact contract line, last
        from pbs_amd.bench.report import compact_line, mix_digest
        out = args.out or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
            with open(out, "w") as f:
                json.dump({"line": line, "results": {m: {"runs": r["runs"], "order": r["order"]}
                                                     for m, r in results.items()}}, f, indent=1)
        except OSError as ex:
            print(f"bench.py: detail record not written: {ex}", file=sys.stderr)
            out = ""
        digests = {m: mix_digest(results[m]["summary"], results[m]["runs"]) for m in mixes}
        sys.stdout.flush()
        os.dup2(line_fd, 1)
        print(json.dumps(compact_line(line, digests, os.path.relpath(out, ROOT) if out else "")), flush=True)
        os.dup2(2, 1)
    if world > 1:
        import torch.distributed as dist
        dist.barrier(group=groups["ctrl"])
        dist.destroy_process_group()

def run_llm5(args):
    """Config #5 in the bench contract: solo, none,
    static-se and gpbs (the daemon's demand-driven SE budgets on live
    counters; shim tenants on CU-masked queues chosen by measurement in
    every run -- remembering the choice across runs was measured harmful,
    runtime/tenant.py qprobe_load), --reps runs each; decode p50 / p99 and
    both tenants' shares per policy.  One JSON line (the driver contract's
    fields, config #5)."""
    import contextlib
    import tempfile

    from pbs_amd.bench import llm_corun
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        print("bench.py --mix llm5 runs on one GPU", file=sys.stderr)
        sys.exit(2)
    secs = max(4.0, args.steps * args.step_ms / 1e3)
    # untimed warm-up, the same for every policy: the trainer's first step
    # compiles for ~2 s, and a scheduler then needs ~1 s to classify and place
    # the arriving tenant (its 190 ms training steps run wherever they were
    # launched); steady state is what config #5 measures (s25 timelines:
    # profiles/r4/llm5_s25.txt)
    warm = max(args.llm5_warm_s, args.warmup * args.step_ms / 1e3)
    out = os.path.join(tempfile.mkdtemp(), "llm5.json")
    pols = args.policies or "solo,none,static-se,gpbs-budget"
    if "solo" not in pols.split(","):  # every share is over the solo rates
        pols = "solo," + pols
    with contextlib.redirect_stdout(sys.stderr):  # rank 0 prints ONE line: ours
        llm_corun.main(["--fp8", "--graph", "--seconds", str(secs), "--warmup", str(warm), "--reps", str(args.reps),
                        "--policies", pols, "--out", out])
    res = json.load(open(out))
    summ = res["summary"]
    g = summ.get("gpbs-budget") or next(iter(summ.values()))
    pol = {("gpbs" if p == "gpbs-budget" else p): {
        "aggregate": v["aggregate"], "mean_slowdown_pct": v["mean_slowdown_pct"],
        "decode_share": v["norm"].get("infer"), "trainer_share": v["norm"].get("train"),
        "decode_p50_ms": v["infer_p50_ms"], "decode_p99_ms": v["infer_p99_ms"],
        "runs": [r["aggregate"] for r in v["runs"]]} for p, v in summ.items()}
    ss = pol.get("static-se")
    line = {
        "metric": json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"],
        "value": g["aggregate"],
        "unit": "solo-equivalents (decode tokens/s + trainer tokens/s, each over its solo rate)",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": g["infer_p50_ms"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16 (decode weights fp8 e4m3fn)",
        "data": "synthetic tokens, random-init Llama-3-8B / Llama-3.2-1B-shaped weights",
        "config": {"model": "#5 Llama-3-8B fp8 decode (batch 8) + Llama-1B-shaped bf16 trainer (4 x 2048)",
                   "global_batch": 8, "seq_len": 2048, "parallelism": "dp1", "mix": "llm5",
                   "seconds_per_run": secs, "reps": args.reps},
        "mean_slowdown_pct": g["mean_slowdown_pct"],
        "policies": pol,
    }
    if ss and "gpbs" in pol:
        line["gpbs_vs_static_se"] = {
            "delta_aggregate": round(pol["gpbs"]["aggregate"] - ss["aggregate"], 4),
            "decode_p99_ratio": round(pol["gpbs"]["decode_p99_ms"] / ss["decode_p99_ms"], 3)
            if ss["decode_p99_ms"] else None}
    print(json.dumps(line), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"line": line, "raw": res}, f, indent=1)


if __name__ == "__main__":
    main()
