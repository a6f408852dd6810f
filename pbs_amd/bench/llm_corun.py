"""Config #5: Llama-3-8B inference co-located with a bf16 training tenant on
one MI355X, under default hardware sharing ("none") and under gpbsd
("gpbs": both are torch processes attached through the tenant shim, their
kernels confined to the CU partitions the scheduler hands them, classes and
quanta driven by the counters they publish).

    python -m pbs_amd.bench.llm_corun [--seconds 8] [--policies solo,none,gpbs]

Tenants (random-init weights of the real architectures, synthetic tokens):
  infer  Llama-3-8B greedy decode, batch 8, 1024-token prompt, KV cache 2048
  train  Llama-3.2-1B-shaped training step (bf16, fused AdamW), batch 4 x 2048

Per tenant: throughput (decode tokens/s, train tokens/s), decode-step
latency p50/p99; normalised to the solo run on the same box:
aggregate = sum of co-run/solo throughputs, slowdown = mean over tenants.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import statistics
import sys
import tempfile
import time
from typing import Dict, Optional

os.environ["GPU_MAX_HW_QUEUES"] = str(max(8, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def _kfd_queues(pid: int) -> Optional[int]:
    """Hardware queues KFD holds for process `pid` (sysfs; None where not exposed)."""
    try:
        return len(os.listdir(f"/sys/class/kfd/kfd/proc/{pid}/queues"))
    except OSError:
        return None


def _timeline(rows, t0: float, bin_s: float = 0.25):
    """Per-step rows (t, gate_ms, run_ms, key) -> per-bin summary: steps, mean
    gate wait, mean run time, the most frequent SE set."""
    bins: Dict[int, list] = {}
    for (t, g, r, k) in rows:
        bins.setdefault(int((t - t0) / bin_s), []).append((g, r, k))
    out = []
    for b in sorted(bins):
        xs = bins[b]
        keys: Dict[str, int] = {}
        for _, _, k in xs:
            keys[k] = keys.get(k, 0) + 1
        out.append([round(b * bin_s, 2), len(xs), round(statistics.mean(g for g, _, _ in xs), 3),
                    round(statistics.mean(r for _, r, _ in xs), 3), max(keys, key=keys.get)])
    return out


def _tenant(kind: str, seconds: float, warmup: float, socket: Optional[str], q, start_evt, args: dict):
    if args.get("tenant_hwq"):  # before anything initialises HIP in this process
        os.environ["GPU_MAX_HW_QUEUES"] = str(args["tenant_hwq"])
    import torch

    from ..models.llama import PRESETS, LlamaDecoder, LlamaTrainer
    torch.cuda.set_device(0)
    t = None
    if socket:
        from ..runtime.tenant import TenantClient
        t = TenantClient(kind, socket, slots=args.get("slots", 8), weight=args.get(f"{kind}_weight", 256),
                         spatial=args.get("spatial", False), priority=args.get(f"{kind}_prio", 0),
                         one_queue=bool(args.get("one_queue")), queue_probe=args.get("queue_probe", -1))
        if args.get("prestream") and t.se_mode:
            t.prepare_streams()
    if kind == "infer":
        w = LlamaDecoder(PRESETS[args["infer_model"]], batch=args["infer_batch"], context=args["context"],
                         fp8=args.get("fp8", False), graph=args.get("graph", False))
        prompt = torch.randint(0, w.cfg.vocab, (w.batch, args["prompt"]), device="cuda")
        nxt = w.prefill(prompt)
        nxt = w.decode_step(nxt)  # graph mode captures here, outside any tenant slice
        flops = 2.0 * w.cfg.n_params() * w.batch
        bytes_ = (1.0 if w.fp8 else 2.0) * w.cfg.n_params()  # weight bytes streamed per decode step

        def unit():
            nonlocal nxt
            nxt = w.decode_step(nxt)
        per_unit_tokens = w.batch
    else:
        w = LlamaTrainer(PRESETS[args["train_model"]], batch=args["train_batch"], seq=args["train_seq"])
        flops = w.flops_per_step()
        bytes_ = 16.0 * w.cfg.n_params()  # params + grads + fp32 Adam state traffic

        def unit():
            w.step()
        per_unit_tokens = w.tokens_per_step()
    prio_stream = None
    if t is None and args.get(f"{kind}_prio", 0):
        prio_stream = torch.cuda.Stream(priority=-abs(args[f"{kind}_prio"]))
    ses = args.get(f"{kind}_ses")
    swap_stream = None
    if t is None and ses is not None:  # static shader-engine split (se:I/T policies)
        from ..ops import kernels as K
        from ..runtime.tenant import se_cu_words
        if args.get("swap_s"):
            # +swapN: the first N seconds on the OTHER half (the swapped layout
            # the daemon's probe phase sometimes starts from), then this half
            other = tuple(sorted({0, 1, 2, 3} - set(ses)))
            swap_stream = torch.cuda.ExternalStream(K.cumask_stream(se_cu_words(other)))
        # +shiftN: N idle masked queues created first (kept), so the tenant's
        # own queue lands N places later in the hardware scheduler's queue
        # order (a probe of cross-process pipe coupling)
        pads = [K.cumask_stream(se_cu_words(ses)) for _ in range(args.get(f"{kind}_shift", 0))]
        prio_stream = torch.cuda.ExternalStream(K.cumask_stream(se_cu_words(ses)))
        args["_pads"] = pads
    torch.cuda.synchronize()
    start_evt.wait()
    lat = []
    rows = []
    halves: Dict[str, int] = {}
    t_start = time.monotonic()
    t_warm = t_start + warmup
    t_end = t_warm + seconds
    n = 0
    queues_mid = None
    while True:
        now = time.monotonic()
        if now >= t_end:
            break
        if queues_mid is None and now >= t_warm + seconds / 2:
            queues_mid = _kfd_queues(os.getpid())
        t0 = time.perf_counter()
        key = ""
        g_ms = 0.0
        if t is not None:
            with t.slice(timeout_s=30.0) as s_used:
                g_ms = 1e3 * (time.perf_counter() - t0)
                used = next((k for k, v in t._streams.items() if v is s_used), None)
                key = ",".join(str(h) for h in sorted({c for (_, c) in t.owned()})) + (
                    "|m" + "".join(str(x) for x in used[1:]) if used else "|u")
                halves[key] = halves.get(key, 0) + 1
                unit()
                torch.cuda.current_stream().synchronize()
            t.account(flops=flops, bytes_moved=bytes_, busy_ns=int((time.perf_counter() - t0) * 1e9))
        elif prio_stream is not None:
            st = swap_stream if swap_stream is not None and now < t_start + args["swap_s"] else prio_stream
            key = "swap" if st is swap_stream else ""
            with torch.cuda.stream(st):
                unit()
            st.synchronize()
        else:
            unit()
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rows.append((now, g_ms, 1e3 * dt - g_ms, key))
        if now >= t_warm:
            lat.append(dt)
            n += 1
    if t is not None:
        t.close(destroy=False)  # keep it registered for the daemon's dump
    span = sum(lat)
    timed = [r for r in rows if r[0] >= t_warm]
    q.put({"kind": kind, "units": n, "tokens_per_s": n * per_unit_tokens / span if span else 0.0,
           "p50_ms": 1e3 * statistics.median(lat) if lat else 0.0,
           "p99_ms": 1e3 * sorted(lat)[int(0.99 * (len(lat) - 1))] if lat else 0.0, "halves": halves,
           "gate_p50_ms": round(statistics.median(r[1] for r in timed), 3) if timed else 0.0,
           "run_p50_ms": round(statistics.median(r[2] for r in timed), 3) if timed else 0.0,
           "kfd_queues": queues_mid, "hwq": os.environ.get("GPU_MAX_HW_QUEUES"),
           "timeline": _timeline(rows, t_start)})


def parse_se_policy(policy: str):
    """'se:I/T' -> (infer SEs, trainer SEs): the decode tenant on the top I
    shader engines of every XCD, the trainer on the bottom T."""
    i, t = (int(x) for x in policy.split(":", 1)[1].split("/"))
    if not (1 <= i <= 4 and 1 <= t <= 4):
        raise ValueError(policy)
    return tuple(range(4 - i, 4)), tuple(range(t))


_HWC = {"on": False}
# Names shared with bench.py's mixes: "static-se" is the hand-picked static
# shader-engine split (decode on SEs {2,3}, trainer on {0,1} of every XCD, the
# best static point of profiles/llm5/frontier_explore_r2.md).
ALIASES = {"static-se": "se:2/2"}


def _hwc_setup():
    """Register the hardware-counter sampler in this (daemon) process before
    anything initialises HIP here; tenants are separate processes."""
    from ..counters import hwc
    _HWC["on"] = hwc.init(gpu=0)
    return _HWC["on"]


def run(policy: str, kinds, args: dict, seconds: float, warmup: float) -> Dict[str, dict]:
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    start = ctx.Event()
    daemon = None
    sock = None
    args = dict(args, spatial=policy == "gpbs-spatial")
    # variant suffixes: +prio (high-priority decode queue), +hwqN (tenant
    # GPU_MAX_HW_QUEUES=N), +pre (both SE-half streams created at registration),
    # +nohwc (daemon on modeled counters), +swapN (static split: the first N s
    # on the swapped halves), +one (one masked queue per shim tenant), +qpK
    # (K masked queues per half, chosen by measured slice time), +nox (no
    # cross-class steals by idle partitions), +ishiftN / +tshiftN (static
    # split: N idle masked queues created before the decode / trainer queue)
    policy, *mods = policy.split("+")
    policy = ALIASES.get(policy, policy)
    base = policy.split("@")[0]
    if base.startswith("se:"):  # static SE split; "se:I/T@solo" runs the given kinds alone on their masks
        args["infer_ses"], args["train_ses"] = parse_se_policy(base)
    for m in mods:
        if m == "prio":
            args["infer_prio"] = 1
        elif m.startswith("hwq"):
            args["tenant_hwq"] = int(m[3:])
        elif m == "pre":
            args["prestream"] = True
        elif m == "one":  # shim tenants: one masked queue, class home half only
            args["one_queue"] = True
        elif m.startswith("qp"):  # shim tenants: K masked queues per half, the fastest by measurement
            args["queue_probe"] = int(m[2:])
        elif m == "nohwc":
            args["nohwc"] = True
        elif m == "nox":  # budget layout without cross-class steals (boot class_steal=0)
            args["class_steal"] = 0
        elif m.startswith("swap"):
            args["swap_s"] = float(m[4:])
        elif m.startswith("ishift"):  # static split: the decode tenant's queue N places later
            args["infer_shift"] = int(m[6:])
        elif m.startswith("tshift"):  # ... the trainer's
            args["train_shift"] = int(m[6:])
        elif m.startswith("slow"):  # daemon sampler: steady-layout back-off period N ms ([runtime] slow_us)
            args["slow_us"] = int(m[4:]) * 1000
        else:
            raise ValueError(f"unknown policy variant +{m}")
    if policy in ("gpbs", "gpbs-spatial"):
        from ..runtime.daemon import Daemon
        sock = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
        daemon = Daemon(sock, gpus=[0], nctx=2, sim=False, profile="mi355x").start()
    elif policy in ("gpbs-se", "gpbs-budget"):
        if args.get("slow_us"):  # the daemon's GpuContext reads [runtime] from GPBS_CONFIG
            cfgp = os.path.join(tempfile.mkdtemp(), "gpbs.toml")
            with open(cfgp, "w") as f:
                f.write(f"[runtime]\nslow_us = {int(args['slow_us'])}\n")
            os.environ["GPBS_CONFIG"] = cfgp
        else:
            os.environ.pop("GPBS_CONFIG", None)
        # SE-exclusive class split driven by LIVE hardware counters: the daemon
        # owns the GPU actuator + rocprofiler-sdk sampler; the tenants' kernels
        # run on streams masked to the shader engines they own, so the per-SE
        # counters are attributed to them by ownership (no declared counters).
        from ..runtime.daemon import Daemon
        sock = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
        over = {"class_split": 2, "idle_skip": 1, "class_dwell": 8}
        if policy == "gpbs-budget":
            # the round-3 runner flagship's layout: demand-driven SE budgets
            # (probe layout until both tenants are classified, then compute
            # SEs {0,1} / memory SEs {2,3}), surplus slots offline
            over.update(class_budget=1, present_us=10000)
            if "class_steal" in args:
                over["class_steal"] = args["class_steal"]
        daemon = Daemon(sock, gpus=[0], nctx=4, sim=False, profile="mi355x", attach_gpu=True, se_mode=True,
                        hw_counters=_HWC["on"] and not args.get("nohwc"), overrides=over).start()
        args["slots"] = 16
        args["spatial"] = True
    ps = [ctx.Process(target=_tenant, args=(k, seconds, warmup, sock, q, start, args)) for k in kinds]
    for p in ps:
        p.start()
    time.sleep(0.5)
    start.set()
    out = {}
    hw_early = None
    try:
        for _ in ps:
            r = q.get(timeout=900)
            out[r["kind"]] = r
            if hw_early is None and daemon is not None and daemon.gpu_ctx is not None and daemon.hw_counters:
                # every tenant still registered: the first to finish is reaped
                # soon after its process exits
                e = daemon.engine
                hw_early = {"_daemon_kfd_queues": _kfd_queues(os.getpid())}
                for t in e.tenants():
                    att, _ = daemon.gpu_ctx.hwc_tenant(t)
                    hw_early[e.tenant_info(t).name] = {
                        "inst": round(att[0]), "miss_rate": round(att[3] * 1e5 / att[0]) if att[0] else None,
                        "class": e.lib.gpbs_tenant_class(e.h, t), "owned_s": daemon.gpu_ctx.ownership(t)}
    finally:
        for p in ps:
            p.join(timeout=120)
        if daemon is not None:
            e = daemon.engine
            if daemon.gpu_ctx is not None and daemon.hw_counters:
                hw = {}
                for t in e.tenants():
                    att, _ = daemon.gpu_ctx.hwc_tenant(t)
                    if att[0]:
                        hw[e.tenant_info(t).name] = {"inst": round(att[0]), "miss_rate": round(att[3] * 1e5 / att[0]),
                                                     "cpi_x1000": round(att[1] * 1e3 / att[0])}
                out["_hw"] = {"tenant": hw, "at_first_finish": hw_early, "stats": daemon.gpu_ctx.hwc_stats(),
                              "owned_s": {e.tenant_info(t).name: daemon.gpu_ctx.ownership(t) for t in e.tenants()}}
            out["_engine"] = {"z": e.debug_keys("z")[-3000:], "tenants": {
                e.tenant_info(t).name: {"tslice_us": e.tenant_info(t).tslice_us, "phase": e.tenant_info(t).phase,
                                        "class": e.lib.gpbs_tenant_class(e.h, t), "run_ns": e.tenant_info(t).run_ns}
                for t in e.tenants()}, "perfc": {
                k: v for k, v in daemon.engine.perfc().items() if v and k in ("sched_ctx", "metric_tick",
                                                                              "report_rx", "adapt_inc",
                                                                              "adapt_dec")}}
            daemon.stop()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    ap.add_argument("--policies", default="solo,none,gpbs")
    ap.add_argument("--infer-model", default="llama3-8b")
    ap.add_argument("--train-model", default="llama3-1b")
    ap.add_argument("--infer-batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=1024)
    ap.add_argument("--context", type=int, default=2048)
    ap.add_argument("--train-batch", type=int, default=4)
    ap.add_argument("--train-seq", type=int, default=2048)
    ap.add_argument("--fp8", action="store_true", help="decode tenant streams e4m3fn weights (fp8 MFMA linears)")
    ap.add_argument("--graph", action="store_true", help="with --fp8: decode step replayed from a HIP graph")
    ap.add_argument("--reps", type=int, default=1, help="repetitions of every co-run policy (median reported)")
    ap.add_argument("--tenant-hwq", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES of the tenant processes (default: inherit, >= 8)")
    ap.add_argument("--prestream", action="store_true",
                    help="shim tenants create both SE-half masked streams at registration")
    ap.add_argument("--daemon-hwq", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES of this (daemon) process (default: >= 8)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    if a.daemon_hwq:  # before anything initialises HIP in this process
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.daemon_hwq)
    args = {"infer_model": a.infer_model, "train_model": a.train_model, "infer_batch": a.infer_batch,
            "prompt": a.prompt, "context": a.context, "train_batch": a.train_batch, "train_seq": a.train_seq,
            "infer_weight": 512, "train_weight": 256, "fp8": a.fp8, "graph": a.graph and a.fp8,
            "tenant_hwq": a.tenant_hwq, "prestream": a.prestream}
    res = {}
    pols = [p for p in a.policies.split(",") if p]
    if any(p.split("+")[0] in ("gpbs-se", "gpbs-budget") for p in pols):  # variants (+hwq2, +nox ...) too
        _hwc_setup()
    if a.out and os.path.exists(a.out):
        raise SystemExit(f"{a.out} exists: results are never overwritten")
    if "solo" in pols:
        res["solo"] = {}
        for k in ("infer", "train"):
            res["solo"].update(run("solo", [k], args, a.seconds, a.warmup))
            print(f"[llm] solo {k}: {json.dumps(res['solo'][k])}", file=sys.stderr, flush=True)
    reps = {p: [] for p in pols if p != "solo"}
    for rep in range(max(1, a.reps)):
        for p in pols:
            if p == "solo":
                continue
            if p.endswith("@solo"):  # each tenant alone on its SE mask
                r = {}
                for k in ("infer", "train"):
                    r.update(run(p, [k], args, a.seconds, a.warmup))
            else:
                r = run(p, ["infer", "train"], args, a.seconds, a.warmup)
            reps[p].append(r)
            brief = {k: {kk: vv for kk, vv in v.items() if kk != "timeline"} for k, v in r.items() if not k.startswith('_')}
            print(f"[llm] {p} rep {rep}: {json.dumps(brief)}",
                  file=sys.stderr, flush=True)
            if a.out:  # every finished run survives a time limit
                with open(a.out + ".partial", "w") as f:
                    json.dump({"solo": res.get("solo"), "reps": reps}, f)
            if "_hw" in r:
                print(f"[llm] {p} rep {rep} hw: {json.dumps(r['_hw'])}", file=sys.stderr, flush=True)
    summary = {}
    if "solo" in res:
        for p, rs in reps.items():
            runs = []
            for r in rs:
                norm = {k: r[k]["tokens_per_s"] / res["solo"][k]["tokens_per_s"] for k in ("infer", "train")
                        if res["solo"][k]["tokens_per_s"]}
                runs.append({"aggregate": round(sum(norm.values()), 4),
                             "mean_slowdown_pct": round(statistics.mean((1 / v - 1) * 100 for v in norm.values()), 2),
                             "norm": {k: round(v, 4) for k, v in norm.items()},
                             "infer_p99_ms": round(r["infer"]["p99_ms"], 3),
                             "infer_p50_ms": round(r["infer"]["p50_ms"], 3)})
            med = lambda xs: round(statistics.median(xs), 4)
            summary[p] = {"aggregate": med([x["aggregate"] for x in runs]),
                          "mean_slowdown_pct": med([x["mean_slowdown_pct"] for x in runs]),
                          "norm": {k: med([x["norm"][k] for x in runs]) for k in runs[0]["norm"]},
                          "infer_p50_ms": med([x["infer_p50_ms"] for x in runs]),
                          "infer_p99_ms": med([x["infer_p99_ms"] for x in runs]), "runs": runs}
    res.update({p: rs for p, rs in reps.items()})
    line = {"config": "#5 Llama-3-8B decode + Llama-1B bf16 training, 1x MI355X", "data": "synthetic tokens, "
            "random-init weights", "dtype": "bf16" + (" (decode weights fp8 e4m3fn)" if a.fp8 else ""), "summary": summary, "raw": res}
    print(json.dumps(line))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
