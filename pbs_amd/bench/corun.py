"""Co-run benchmark: the BASELINE.json headline metric.

"co-run slowdown (%) vs solo + aggregate throughput, 4-tenant mix at
1/2/4/8 GPU" (SURVEY §6 protocol; config #3 per GPU, weak scaling).

Per GPU rank, four tenants share one MI355X:

* ``gemm``  bf16 4096^3 MFMA GEMM (compute-bound)            native runner
* ``hbm``   1 GiB float4 copy (HBM-bound)                     native runner
* ``coll``  all-reduce tenant: RCCL all-reduce over xGMI when N > 1, the
            reduce-copy traffic kernel on one GPU             native runner / thread
* ``idle``  latency tenant: one 8192^2 GEMV request every 2 ms native runner

A *step* gives every throughput tenant a fixed quota of units, sized so that
each quota takes ``target_ms`` when the tenant runs alone on the whole GPU
(calibrated during warmup), and lets the idle tenant issue its requests; the
step ends when every quota is done.  With t_i the time tenant i needed inside
the step and T_i its solo time for the same quota:

  slowdown_i  = t_i / T_i - 1                 (per tenant, %)
  norm_perf_i = T_i / t_i                     (idle tenant: solo/co-run p50 latency)
  aggregate   = sum_i norm_perf_i over the throughput tenants (weighted speedup)

``value`` = aggregate summed over all GPUs (whole-job, solo-equivalents).
Policies: ``none`` (default hardware sharing: all tenants launch ungated full
-GPU grids), ``static`` (equal static XCD split), ``gpbs`` (the PBS adaptive
credit scheduler driving XCD ownership from device counters) — the flagship.
"""
from __future__ import annotations

import json
import os
import statistics
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..core.engine import Engine
from ..runtime.gpu import GpuContext, Runner

THROUGHPUT = ("gemm", "hbm", "coll")


@dataclass
class CorunConfig:
    steps: int = 20
    warmup: int = 3
    target_ms: float = 30.0
    policies: tuple = ("none", "static", "gpbs")
    gemm_n: int = 4096
    hbm_bytes: int = 1 << 30
    coll_bytes: int = 256 << 20
    idle_rows: int = 8192
    idle_period_ms: float = 2.0
    sched: str = "credit"
    tslice_us: int = 100
    depth: int = 2
    table_mode: str = "host"
    calib_units: int = 8
    threshold: int = 20000  # PBS miss-rate threshold for modeled GPU counters (per 100k inst)


class CollTenant:
    """All-reduce tenant for N > 1: RCCL all-reduce over xGMI on its own
    process group and stream, launch-gated on XCD ownership (RCCL kernels
    themselves are not CU-confined)."""

    def __init__(self, ctx: GpuContext, engine: Optional[Engine], tenant: int, nbytes: int, group):
        self.ctx, self.engine, self.tenant, self.group = ctx, engine, tenant, group
        self.buf = torch.randn(nbytes // 2, device="cuda", dtype=torch.bfloat16)
        self.stream = torch.cuda.Stream(priority=0)
        self.gate = True
        self.work_per_unit = float(nbytes) * 2.0  # ring all-reduce: ~2x bytes per rank
        self.reset_stats()

    def reset_stats(self):
        self.units_done = 0
        self.last_done_ns = 0
        self.busy_ns = 0

    def _owns(self):
        return (not self.gate) or self.tenant in self.ctx.owners()

    def run_units(self, n: int):
        import torch.distributed as dist
        if self.engine is not None and self.gate:
            self.engine.wake(self.tenant)
        t0 = time.monotonic_ns()
        with torch.cuda.stream(self.stream):
            for _ in range(n):
                while not self._owns():
                    time.sleep(20e-6)
                dist.all_reduce(self.buf, group=self.group)
                self.buf.mul_(0.5)
            self.stream.synchronize()
        t = time.monotonic_ns()
        self.units_done += n
        self.last_done_ns = t
        self.busy_ns += t - t0
        if self.engine is not None and self.gate:
            self.engine.block(self.tenant)


def _pct(xs, q):
    if not xs:
        return 0.0
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


class Corun:
    def __init__(self, cfg: CorunConfig, rank: int = 0, world: int = 1, device: int = 0, groups=None, log=print):
        self.cfg, self.rank, self.world, self.device = cfg, rank, world, device
        self.groups = groups or {}
        self.log = log if rank == 0 else (lambda *a, **k: None)
        torch.cuda.set_device(device)
        self.engine = Engine(sched=cfg.sched, tslice_us=cfg.tslice_us,
                             adapt={"threshold": cfg.threshold})
        for x in range(8):
            pid = self.engine.partition_add(rank, x)
            self.engine.pool_assign(0, pid)
        self.dom0 = self.engine.tenant_create("Domain-0", nslots=1)
        self.tid = {}
        for name, ns in (("gemm", 8), ("hbm", 8), ("coll", 8), ("idle", 1)):
            self.tid[name] = self.engine.tenant_create(name, nslots=ns)
        self.ctx = GpuContext(device, self.engine, part_base=0, table_mode=cfg.table_mode)
        self.runners: Dict[str, object] = {}
        self.runners["gemm"] = Runner(self.ctx, "gemm", self.tid["gemm"], depth=cfg.depth, M=cfg.gemm_n,
                                      N=cfg.gemm_n, K=cfg.gemm_n)
        self.runners["hbm"] = Runner(self.ctx, "stream", self.tid["hbm"], depth=cfg.depth, bytes=cfg.hbm_bytes)
        if world > 1:
            self.runners["coll"] = CollTenant(self.ctx, self.engine, self.tid["coll"], cfg.coll_bytes,
                                              self.groups.get("coll"))
        else:
            self.runners["coll"] = Runner(self.ctx, "reduce", self.tid["coll"], depth=cfg.depth,
                                          bytes=cfg.coll_bytes)
        self.runners["idle"] = Runner(self.ctx, "gemv", self.tid["idle"], depth=1, priority=1, M=cfg.idle_rows,
                                      K=cfg.idle_rows)
        self.quota: Dict[str, int] = {}
        self.solo_unit_ms: Dict[str, float] = {}
        self.solo_lat_ms = 0.0
        self.engine_started = False

    # ------------------------------------------------------------- policy
    def set_policy(self, policy: str):
        native = [r for r in self.runners.values() if isinstance(r, Runner)]
        if policy == "gpbs":
            if not self.engine_started:
                self.engine.start()
                self.engine_started = True
            for r in native:
                r.set_gate(True)
                r.set_engine_wake(True)
            self.runners["coll"].gate = True if not isinstance(self.runners["coll"], Runner) else None
        else:
            if self.engine_started:
                self.engine.stop()
                self.engine_started = False
            if policy == "none":
                for r in native:
                    r.set_gate(False)
                    r.set_engine_wake(False)
                if not isinstance(self.runners["coll"], Runner):
                    self.runners["coll"].gate = False
            elif policy == "static":
                # equal XCD split, 2 XCDs per tenant (ARINC-653-like static partitions)
                order = ["gemm", "hbm", "coll", "idle"]
                owners = [self.tid[order[x // 2]] for x in range(8)]
                self.ctx.set_owners(owners)
                for r in native:
                    r.set_gate(True)
                    r.set_engine_wake(False)
                if not isinstance(self.runners["coll"], Runner):
                    self.runners["coll"].gate = True
            elif policy == "solo":
                for r in native:
                    r.set_gate(False)
                    r.set_engine_wake(False)
                if not isinstance(self.runners["coll"], Runner):
                    self.runners["coll"].gate = False
            else:
                raise ValueError(policy)
        if policy == "gpbs" and not isinstance(self.runners["coll"], Runner):
            self.runners["coll"].gate = True

    # ---------------------------------------------------------- primitives
    def _barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier(group=self.groups.get("ctrl"))
        torch.cuda.synchronize()

    def _run_units(self, name: str, n: int):
        r = self.runners[name]
        if isinstance(r, Runner):
            r.submit(n)
            r.wait(120.0)
        else:
            r.run_units(n)

    def calibrate(self):
        """Solo time per unit for each throughput tenant (whole GPU, ungated)."""
        self.set_policy("solo")
        cfg = self.cfg
        for name in THROUGHPUT:
            self._barrier()
            self._run_units(name, 2)  # warm
            self._barrier()
            t0 = time.perf_counter()
            self._run_units(name, cfg.calib_units)
            self._barrier()
            dt = (time.perf_counter() - t0) * 1e3 / cfg.calib_units
            self.solo_unit_ms[name] = self._allmax(dt)
            self.quota[name] = max(1, int(round(cfg.target_ms / self.solo_unit_ms[name])))
        # idle tenant solo latency (p50)
        r = self.runners["idle"]
        r.latencies(clear=True)
        for _ in range(20):
            r.submit(1)
            r.wait(10.0)
            time.sleep(cfg.idle_period_ms / 1e3)
        lats = r.latencies(clear=True)
        self.solo_lat_ms = _pct(lats, 0.5) / 1e6
        self.log(f"[corun] solo unit ms: {self.solo_unit_ms}  quota/step: {self.quota}  "
                 f"idle p50 {self.solo_lat_ms:.3f} ms")

    def _allmax(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.groups.get("ctrl"))
        return float(t.item())

    def _allsum(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.groups.get("ctrl"))
        return float(t.item())

    def step(self) -> Dict[str, float]:
        """One co-run step; returns per-tenant completion times (ms) in the step."""
        cfg = self.cfg
        t0 = time.monotonic_ns()
        done = {}
        threads = []
        for name in THROUGHPUT:
            r = self.runners[name]
            if isinstance(r, Runner):
                r.submit(self.quota[name])
            else:
                th = threading.Thread(target=r.run_units, args=(self.quota[name],))
                th.start()
                threads.append(th)
        # idle tenant: closed loop of requests with think time until the
        # throughput tenants finish (at least one request per step).
        idle = self.runners["idle"]
        nreq = 0
        while True:
            idle.submit(1)
            idle.wait(30.0)
            nreq += 1
            busy = any(self.runners[n].stats().units_done < self._target[n] for n in THROUGHPUT
                       if isinstance(self.runners[n], Runner)) or any(t.is_alive() for t in threads)
            if not busy:
                break
            time.sleep(cfg.idle_period_ms / 1e3)
        for name in THROUGHPUT:
            r = self.runners[name]
            if isinstance(r, Runner):
                r.wait(120.0)
        for th in threads:
            th.join()
        for name in THROUGHPUT:
            r = self.runners[name]
            last = r.stats().last_done_ns if isinstance(r, Runner) else r.last_done_ns
            done[name] = (last - t0) / 1e6
        done["_step"] = (time.monotonic_ns() - t0) / 1e6
        done["_nreq"] = nreq
        return done

    def run_policy(self, policy: str, steps: int, warmup: int) -> Dict:
        self.set_policy(policy)
        self._target = {}
        for _ in range(warmup):
            self._sync_targets()
            self.step()
        self.runners["idle"].latencies(clear=True)
        if policy == "gpbs":
            self.engine.perfc_reset()
        per = {n: [] for n in THROUGHPUT}
        step_ms = []
        self._barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            self._sync_targets()
            d = self.step()
            for n in THROUGHPUT:
                per[n].append(d[n])
            step_ms.append(d["_step"])
        self._barrier()
        wall_ms = (time.perf_counter() - t0) * 1e3
        wall_ms = self._allmax(wall_ms)
        lats = [x / 1e6 for x in self.runners["idle"].latencies(clear=True)]
        res = {"policy": policy, "wall_ms": wall_ms, "ms_per_step": wall_ms / steps, "tenants": {}}
        agg = 0.0
        slows = []
        for n in THROUGHPUT:
            t_i = statistics.mean(per[n])
            T_i = self.quota[n] * self.solo_unit_ms[n]
            perf = T_i / t_i if t_i > 0 else 0.0
            agg += perf
            slows.append((t_i / T_i - 1.0) * 100.0)
            res["tenants"][n] = {"corun_ms": round(t_i, 3), "solo_ms": round(T_i, 3), "norm_perf": round(perf, 4),
                                 "slowdown_pct": round((t_i / T_i - 1.0) * 100.0, 2)}
        p50 = _pct(lats, 0.5)
        p99 = _pct(lats, 0.99)
        idle_perf = self.solo_lat_ms / p50 if p50 > 0 else 0.0
        slows.append((p50 / self.solo_lat_ms - 1.0) * 100.0 if self.solo_lat_ms > 0 else 0.0)
        res["tenants"]["idle"] = {"p50_ms": round(p50, 4), "p99_ms": round(p99, 4),
                                  "solo_p50_ms": round(self.solo_lat_ms, 4), "norm_perf": round(idle_perf, 4),
                                  "slowdown_pct": round(slows[-1], 2), "requests": len(lats)}
        res["aggregate"] = agg
        res["aggregate_all_gpus"] = self._allsum(agg)
        res["mean_slowdown_pct"] = statistics.mean(slows)
        if policy == "gpbs":
            pc = self.engine.perfc()
            res["engine"] = {k: pc[k] for k in ("sched_ctx", "acct_run", "metric_tick", "adapt_inc", "adapt_dec",
                                                 "adapt_rearm", "migrate_queued", "vcpu_wake_runnable")}
            res["engine"]["gpu"] = self.ctx.stats()
            res["engine"]["tslice_us"] = {n: self.engine.tenant_info(self.tid[n]).tslice_us for n in self.tid}
            res["engine"]["phase"] = {n: self.engine.tenant_info(self.tid[n]).phase for n in self.tid}
            res["engine"]["miss_rate"] = {n: self.engine.tenant_info(self.tid[n]).cache_miss_rate for n in self.tid}
        self.log(f"[corun] {policy}: " + json.dumps(res))
        return res

    def _sync_targets(self):
        for n in THROUGHPUT:
            r = self.runners[n]
            if isinstance(r, Runner):
                self._target[n] = r.stats().units_done + self.quota[n]

    def close(self):
        if self.engine_started:
            self.engine.stop()
        for r in self.runners.values():
            if isinstance(r, Runner):
                r.close()
        self.ctx.close()
        self.engine.close()
