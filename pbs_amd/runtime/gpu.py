"""GPU runtime: one GpuContext per MI355X, bound to the engine of that rank.

* ``GpuContext`` owns the partition table (XCD -> tenant), the per-tenant
  software counter blocks, and installs the GPU actuator + device counter
  backend on the engine (``gpbs_gpu_attach``).
* ``Runner`` is a native (C++) tenant worker: it owns a HIP stream and keeps
  units of its workload in flight while its tenant owns XCDs.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

# One hardware queue per stream: every tenant runner stream plus the scheduler
# stream (partition-table updates, counter reduce).  With the HIP default of 4
# queues, streams share queues round-robin and a table update can sit behind
# a parked tenant kernel on the same queue until its park bound expires.
# Round 4: 12, not 8 -- the 8mix (8 runners plus the scheduler's streams) ran
# ~+0.006 higher and hit its masked-queue slow mode in 1 of 32 runs instead of
# 3 of 32; 4 and 2 made that mode far more frequent
# (profiles/r4/hip_queues_s40.txt, _s41.txt, _s42.txt).  GPBS_HWQ overrides.
# Must be set before the HIP runtime initialises (first device call).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("GPBS_HWQ") or str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))

import torch  # noqa: E402

from .. import _native as N
from ..ops import hipabi
from ..ops.kernels import lib as hiplib

XCDS = 8
CTX = 4  # issue contexts per XCD in the partition table (SMT-sibling analog)


class GpuContext:
    def __init__(self, device: int = 0, engine=None, part_base: int = 0, table_mode: str = "host",
                 device_counters: bool = True, device_adapt: bool = False, nctx: int = 1,
                 params: Optional[Dict[str, int]] = None):
        """``params``: runtime parameters by name (gpbs.toml ``[runtime]``,
        see :meth:`param`); None applies the loaded configuration's."""
        self.L = hiplib()
        self.device = device
        self.part_base = part_base
        self.nctx = nctx
        h = self.L.gpbs_gpu_ctx_create(device, part_base, 1 if table_mode == "device" else 0, nctx)
        if not h:
            raise RuntimeError(f"gpbs_gpu_ctx_create failed on device {device}")
        self.h = C.c_void_p(h)
        if params is None:
            from ..core.config import load
            params = load(os.environ.get("GPBS_CONFIG") or None).get("runtime", {})
        for k, v in params.items():
            self.param(k, int(v))
        if table_mode == "bar":
            self.set_table_mode("bar")
        self.engine = None
        if engine is not None:
            self.attach(engine, device_counters, device_adapt)

    def param(self, name: str, value: int = -1) -> int:
        """Set a runtime parameter (value >= 0) and return its previous value:
        sampler period_us / slow_us / duty_pct / burst_ms / budget_pct /
        bucket / clean_pct / device_attr / fallback / stale_us / watch /
        align / guard_us / long_us, class-share share / probe_every /
        probe_len (csrc/hip/runtime.cpp gpbs_gpu_param)."""
        r = self.L.gpbs_gpu_param(self.h, name.encode(), int(value))
        if r == -22:
            raise KeyError(f"unknown runtime parameter {name!r}")
        return r

    def attach(self, engine, device_counters=True, device_adapt=False, nctx=None):
        """Bind the GPU actuator + counter backend to ``engine`` (whose
        partitions are (xcd, ctx) pairs numbered xcd*nctx + ctx)."""
        self.engine = engine
        if nctx is not None:
            self.nctx = nctx
        self.L.gpbs_gpu_set_nctx(self.h, self.nctx)
        rc = self.L.gpbs_gpu_attach(self.h, engine.h, int(device_counters), int(device_adapt))
        if rc:
            raise RuntimeError("gpbs_gpu_attach failed")

    def attach_mux(self, engine, device_counters: bool = True, nctx: Optional[int] = None):
        """Register this GPU as one backend of a multi-GPU engine: it serves the
        partitions [part_base, part_base + 8 * nctx) (one engine spanning
        several GPUs, gpbs_backend_mux_add).  Clear the engine's mux before
        closing the context."""
        self.engine = engine
        if nctx is not None:
            self.nctx = nctx
        self.L.gpbs_gpu_set_nctx(self.h, self.nctx)
        a, k = N.ActuatorOps(), N.CounterOps()
        if self.L.gpbs_gpu_backend_ops(self.h, engine.h, C.byref(a), C.byref(k), int(device_counters)):
            raise RuntimeError("gpbs_gpu_backend_ops failed")
        return engine.mux_add(self.part_base, self.part_base + XCDS * self.nctx, a, k)

    @property
    def table(self):
        return C.c_void_p(self.L.gpbs_gpu_table(self.h))

    @property
    def counters(self):
        return C.c_void_p(self.L.gpbs_gpu_counters(self.h))

    def set_owners(self, owners: List[int]):
        """owners: 8 entries (one tenant per XCD, other contexts idle), 16
        ((xcd, ctx) major, two contexts per XCD) or XCDS*CTX entries."""
        if len(owners) % XCDS or not 1 <= len(owners) // XCDS <= CTX:
            raise ValueError(f"owners: need a multiple of {XCDS} entries, at most {XCDS * CTX}")
        per = len(owners) // XCDS
        owners = [owners[x * per + c] if c < per else -1 for x in range(XCDS) for c in range(CTX)]
        arr = (C.c_int * (XCDS * CTX))(*owners)
        return self.L.gpbs_gpu_set_owners(self.h, arr)

    def owners(self) -> List[int]:
        """XCDS*CTX entries: tenant on (xcd, ctx), (xcd, ctx) major, -1 idle."""
        arr = (C.c_int * (XCDS * CTX))()
        self.L.gpbs_gpu_get_owners(self.h, arr)
        return list(arr)

    def read_counters(self, tenant: int, per_xcd=False):
        out = (C.c_uint64 * 4)()
        px = (C.c_uint64 * 32)()
        rc = self.L.gpbs_gpu_read_counters(self.h, tenant, out, px)
        if rc:
            raise RuntimeError("read_counters failed")
        if per_xcd:
            return [tuple(px[x * 4:(x + 1) * 4]) for x in range(XCDS)]
        return tuple(out)

    def set_hold(self, on: bool) -> int:
        """Latency-request hold: while a priority (latency) runner's unit is in
        flight, memory-class runners pause at their next unit boundary
        (GATE_HOLD; host and BAR table modes).  Returns the number of holds
        raised so far."""
        n = C.c_uint64(0)
        self.L.gpbs_gpu_set_hold(self.h, 1 if on else 0, C.byref(n))
        return int(n.value)

    def hold_raises(self) -> int:
        n = C.c_uint64(0)
        self.L.gpbs_gpu_set_hold(self.h, -1, C.byref(n))
        return int(n.value)

    TABLE_MODES = {"host": 0, "device": 1, "bar": 2}

    def set_table_mode(self, mode: str):
        """'host': pinned host table polled over PCIe; 'device': device copy
        refreshed by the partition_switch kernel, polled on chip; 'bar': a
        fine-grained VRAM table the host writes directly through the BAR
        (no kernel or queue on the switch path), polled on chip."""
        if mode not in self.TABLE_MODES:
            raise ValueError(f"table mode {mode!r}: one of {sorted(self.TABLE_MODES)}")
        rc = self.L.gpbs_gpu_set_table_mode(self.h, self.TABLE_MODES[mode])
        if rc:
            raise RuntimeError(f"set_table_mode({mode!r}) failed: {rc}")

    def table_mode(self) -> str:
        m = self.L.gpbs_gpu_table_mode(self.h)
        return {v: k for k, v in self.TABLE_MODES.items()}[m]

    def set_hwc(self, on: bool):
        """Drive the PBS metric with live hardware counters (requires
        pbs_amd.counters.hwc.init() before HIP init, then hwc.start())."""
        rc = self.L.gpbs_gpu_set_hwc(self.h, 1 if on else 0)
        if rc:
            raise RuntimeError(f"set_hwc failed ({rc}): hardware counters not initialised/started")

    def hwc_stats(self):
        n, ns = C.c_uint64(0), C.c_uint64(0)
        r = (C.c_double * 4)()
        self.L.gpbs_gpu_hwc_stats(self.h, C.byref(n), C.byref(ns), r)
        mx, sem = C.c_uint64(0), C.c_int(0)
        u = (C.c_double * 4)()
        self.L.gpbs_gpu_hwc_quality(self.h, C.byref(mx), u, C.byref(sem))
        cf = (C.c_double * 4)()
        pct = self.L.gpbs_gpu_hwc_clean(self.h, -1, cf)
        slow = C.c_uint64(0)
        self.L.gpbs_gpu_hwc_period(self.h, -1, -1, C.byref(slow))
        la, bs, ho = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        dev = self.L.gpbs_gpu_hwc_attr_stats(self.h, C.byref(la), C.byref(bs), C.byref(ho))
        mp = C.c_uint64(0)
        duty = self.L.gpbs_gpu_hwc_duty(self.h, -1, C.byref(mp))
        tr, bsm = C.c_uint64(0), C.c_uint64(0)
        self.L.gpbs_gpu_hwc_bursts(self.h, C.byref(tr), C.byref(bsm))
        bud = (C.c_uint64 * 6)()
        self.L.gpbs_gpu_hwc_budget_stats(self.h, bud)
        al = (C.c_uint64 * 8)()
        align = self.L.gpbs_gpu_hwc_align(self.h, -1, -1, -1, al)
        at = (C.c_uint64 * 4)()
        self.L.gpbs_gpu_hwc_attr_timing(self.h, at)
        return {"budget_pct": bud[0], "burst_denied": bud[1], "model_fallback_periods": bud[2],
                "clean_periods": bud[3], "skipped_periods": al[7], "metric_periods": bud[2] + bud[3],
                "align": bool(align), "align_samples": al[0], "align_close": al[1], "align_long": al[2],
                "align_short": al[3], "align_denied": al[4], "ts_period_us": round(al[5] / 1e3, 1),
                "measure_requests": int(self.L.gpbs_gpu_hwc_measure_reqs(self.h)),
                "attr_device": bool(dev), "attr_kernel_launches": la.value, "attr_busy_skips": bs.value,
                "attr_host": ho.value, "attr_harvested": at[0], "attr_kernel_us_mean": round(at[1] / 1e3, 2),
                "attr_kernel_us_max": round(at[2] / 1e3, 2), "attr_harvest_lag_us": round(at[3] / 1e3, 1),
                "duty_cap_pct": duty, "mean_period_us": round(mp.value / 1e3, 1),
                "burst_triggers": tr.value, "burst_samples": bsm.value,
                "samples": n.value, "slow_samples": slow.value, "mean_sample_us": round(ns.value / 1e3, 1), "max_sample_us": round(mx.value / 1e3, 1),
                "hw_over_model": [round(x, 4) for x in r],
                "unattributed_frac": [round(x, 4) for x in u],
                "attribution": "exact-se" if sem.value & 1 else "xcd-time-share",
                # exclusive-ownership windows: share of the counts that reached the PBS metric
                "clean_pct": pct, "metric_frac": [round(x, 4) for x in cf]}

    def hwc_tenant_periods(self, tenant: int) -> dict:
        """A tenant's metric periods since the last hwc reset: clean window,
        calibrated model fallback, skipped (no clean window), sliver (the edge
        of another tenure); and its hardware/model calibration."""
        o = (C.c_uint64 * 4)()
        cal = (C.c_double * 4)()
        self.L.gpbs_gpu_hwc_tenant_periods(self.h, int(tenant), o, cal)
        cd = (C.c_int64 * 6)()
        self.L.gpbs_gpu_hwc_tenant_cadence(self.h, int(tenant), cd)
        # model: 1 ms ticks from the calibrated model; delivered: metric periods
        # with any delivery; period_ms: mean time between those (the effective
        # metric period of the tenant)
        return {"clean": o[0], "fallback": o[1], "skipped": o[2], "sliver": o[3],
                "cal": [round(x, 4) for x in cal], "model": int(cd[0]), "delivered": int(cd[1]),
                "period_ms": round(cd[2] / 1e6, 2), "cadence": bool(cd[3]), "moved": int(cd[4]),
                "ticks": int(cd[5])}

    def switch_cost(self, tenant: int) -> dict:
        """The tenant's measured switch cost (round 6): EWMA revocation drain
        (publish -> its interrupted unit's grid gone) and re-entry ramp
        (publish -> its next launch), us, and how many of each were measured.
        drain + ramp is what the engine floors its time-shared quantum on."""
        o = (C.c_int64 * 4)()
        self.L.gpbs_gpu_switch_cost(self.h, int(tenant), o)
        return {"drain_us": round(o[0] / 1e3, 1), "ramp_us": round(o[1] / 1e3, 1), "n_drain": int(o[2]),
                "n_ramp": int(o[3])}

    def set_hwc_sampler(self, budget_pct: int = -1, align: int = -1, fallback: int = -1, duty: int = -1,
                        slow_us: int = -1, guard_us: int = -1, long_us: int = -1, stale_us: int = -1):
        """Sampler policy: `budget_pct` caps the time all hardware samples may
        take (token bucket; 0: no budget); `align`: switch-aligned samples (a
        sample one drain guard of `guard_us` after an owner change that closes
        or opens a tenure window; tenures of `long_us` or more open one at
        every switch); `fallback`: a tenant without a clean window for
        `stale_us` reports its modeled deltas scaled by its hardware/model
        ratio; `duty`: the background cadence's duty-cycle cap
        (set_hwc_duty); `slow_us`: the back-off period once no owner has
        changed for 20 ms (0: none).  -1 keeps."""
        self.L.gpbs_gpu_hwc_sampler(self.h, int(budget_pct), int(align), int(fallback))
        self.L.gpbs_gpu_hwc_align(self.h, int(guard_us), int(long_us), int(stale_us), None)
        if duty >= 0:
            self.set_hwc_duty(duty)
        if slow_us >= 0:
            self.set_hwc_period(-1, int(slow_us))

    def hwc_sampler(self) -> dict:
        """The current sampler policy (set_hwc_sampler's arguments)."""
        bud = (C.c_uint64 * 6)()
        self.L.gpbs_gpu_hwc_budget_stats(self.h, bud)
        return {"budget_pct": int(bud[0]), "align": int(bud[4]), "fallback": int(bud[5]),
                "duty": int(self.L.gpbs_gpu_hwc_duty(self.h, -1, None)),
                "slow_us": int(self.L.gpbs_gpu_hwc_period(self.h, -1, -1, None))}

    def set_hwc_duty(self, pct: int) -> int:
        """Sampler duty-cycle cap: the period stretches so that sampling takes
        at most `pct` % of the time (0: off).  Returns the old cap."""
        return self.L.gpbs_gpu_hwc_duty(self.h, int(pct), None)

    def set_hwc_device(self, on: bool) -> bool:
        """Attribute counter snapshots on the GPU (k_hwc_attribute, default)
        or on the host (the reference implementation); returns the old setting."""
        return bool(self.L.gpbs_gpu_set_hwc_device(self.h, 1 if on else 0))

    def set_hwc_period(self, fast_us: int = -1, slow_us: int = -1):
        """Counter sampler cadence: every fast_us while the partition table is
        changing, every slow_us once no owner has changed for 20 ms (0: no
        back-off).  Each device-counting sample perturbs the tenants."""
        self.L.gpbs_gpu_hwc_period(self.h, int(fast_us), int(slow_us), None)

    def set_share(self, on: bool) -> int:
        """Class-share mode (SE mode): co-resident full-GPU grids while every
        partition owner is of one contention class, with periodic exclusive
        probe windows (needs the live-counter sampler).  Returns the old value."""
        return self.L.gpbs_gpu_set_share(self.h, 1 if on else 0, None)

    def share_ns(self) -> int:
        """Time spent in class-share mode since the last hwc reset (ns)."""
        v = C.c_int64(0)
        self.L.gpbs_gpu_set_share(self.h, -1, C.byref(v))
        return v.value

    def set_hwc_clean(self, pct: int) -> int:
        """Exclusive-ownership window: a partition's counter delta reaches the
        PBS metric only when one tenant owned it >= pct % of the sample
        interval (0: split every interval pro rata).  Returns the old value."""
        return self.L.gpbs_gpu_hwc_clean(self.h, int(pct), None)

    def hwc_tenant(self, tenant: int):
        """Cumulative hardware counts attributed to `tenant` since the last
        reset, and its modeled counts: (att[4], model[4]) over the PBS slots
        INST, CYCLES, LLC_REFS (L2 requests), LLC_MISSES (L2 misses)."""
        a, m = (C.c_double * 4)(), (C.c_double * 4)()
        self.L.gpbs_gpu_hwc_tenant(self.h, tenant, a, m)
        return list(a), list(m)

    def hwc_tenant_metric(self, tenant: int):
        """Cumulative counts of `tenant` that reached the PBS metric (the
        exclusive-ownership windows) since the last reset."""
        m = (C.c_double * 4)()
        self.L.gpbs_gpu_hwc_tenant_metric(self.h, tenant, m)
        return list(m)

    def hwc_reset(self):
        self.L.gpbs_gpu_hwc_reset(self.h)

    def hwc_poll(self) -> int:
        """Attribute the newest counter snapshot now (engine-less use)."""
        return self.L.gpbs_gpu_hwc_poll(self.h)

    def set_se_mode(self, on: bool, pool: bool = True):
        """SE-exclusive partitions: the 4 partitions of each XCD are its shader
        engines, each owned by one tenant at a time (GATE_SE gating).
        ``pool``: make the process's CU-masked queue burst now (False in a
        process that runs no tenant kernel, e.g. gpbsd)."""
        rc = self.L.gpbs_gpu_set_se_mode(self.h, (1 if pool else 2) if on else 0)
        if rc:
            raise RuntimeError("set_se_mode failed")

    def set_waveprio(self, on: bool):
        """Latency-class runners (priority > 0) raise their waves' SIMD issue
        priority (s_setprio 3) under gated policies."""
        rc = self.L.gpbs_gpu_set_waveprio(self.h, 1 if on else 0)
        if rc:
            raise RuntimeError("set_waveprio failed")

    def set_lat_half(self, half: int):
        """Latency lane: ungated latency-class runners launch on a stream
        CU-masked to class half `half` (0: SEs {0,1}, 1: SEs {2,3}; -1: off)."""
        rc = self.L.gpbs_gpu_set_lat_half(self.h, int(half))
        if rc:
            raise RuntimeError("set_lat_half failed")

    def set_spatial(self, on: bool):
        """Spatial partitions: the two partitions of an XCD are CU halves
        (shader engines 0-1 / 2-3) -- runners launch on half-masked streams
        and workgroups gate on their CU's half -- instead of co-resident
        issue contexts."""
        rc = self.L.gpbs_gpu_set_spatial(self.h, 1 if on else 0)
        if rc:
            raise RuntimeError("set_spatial failed")

    def ownership(self, tenant: int, clear: bool = False):
        """Seconds `tenant` held each issue context (summed over XCDs)."""
        out = (C.c_int64 * CTX)()
        self.L.gpbs_gpu_ownership(self.h, tenant, out, int(clear))
        return [x / 1e9 for x in out]

    def switch_latency(self, iters: int = 200, nwg: int = 1024) -> List[int]:
        """End-to-end actuation latency in ns per iteration: publish of a new
        assignment -> every workgroup of an nwg-workgroup probe grid observed
        it (the context's table mode; no engine may be attached)."""
        out = (C.c_int64 * iters)()
        n = self.L.gpbs_gpu_switch_latency(self.h, iters, nwg, out)
        if n < 0:
            raise RuntimeError(f"switch_latency failed ({n})")
        return list(out[:n])

    def stats(self):
        out = (C.c_uint64 * 4)()
        self.L.gpbs_gpu_stats(self.h, out)
        ca, la, bu = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        self.L.gpbs_gpu_adapt_stats(self.h, C.byref(ca), C.byref(la), C.byref(bu))
        mp = (C.c_uint64 * 5)()
        self.L.gpbs_gpu_masked_pool(mp, 0)
        return {"switches": out[0], "flushes": out[1], "metric_calls": out[2], "metric_ns": out[3],
                "adapt_device_calls": ca.value, "adapt_device_late": la.value, "adapt_device_busy": bu.value,
                "masked_queues_created": mp[0], "masked_queues_free": mp[1],
                "masked_cross_key_shares": mp[2], "masked_queues_held_max": mp[3],
                "masked_pipe_shared_other": mp[4]}

    def masked_pool_reset(self):
        """Restart the held-queues high-water mark (per timed run)."""
        self.L.gpbs_gpu_masked_pool(None, 1)

    def close(self):
        if getattr(self, "h", None):
            self.L.gpbs_gpu_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class RunnerStats:
    units_done: int
    launches: int
    relaunches: int
    waits_owner: int
    submitted: int
    busy_ns: int
    wait_owner_ns: int
    first_start_ns: int
    last_done_ns: int
    lat_sum_ns: int
    lat_max_ns: int
    lat_count: int
    units_alt: int = 0
    drain_sum_ns: int = 0   # revocation drain (publish -> interrupted unit's grid gone)
    drain_max_ns: int = 0
    drain_count: int = 0


class Runner:
    """Native tenant worker.  ``kind`` in {gemm, stream, reduce, gemv}.

    ``alt`` (optional): a second workload ``dict(kind=..., **shape)`` for a
    phase-changing tenant; ``set_phase(1)`` makes every fresh unit run it
    (``stats().units_alt`` counts them)."""

    def __init__(self, ctx: GpuContext, kind: str, tenant: int, *, gate: bool = True, priority: int = 0,
                 depth: int = 2, grid: int = 0, engine_wake: bool = True, alt: Optional[dict] = None, **shape):
        self.ctx = ctx
        self.L = ctx.L
        self.kind = kind
        self.tenant = tenant
        dev = torch.device("cuda", ctx.device)
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + tenant)
        cfg = hipabi.RunnerCfg()
        cfg.tenant = tenant
        cfg.gate = int(gate)
        cfg.priority = priority
        cfg.depth = depth
        cfg.grid = grid
        cfg.engine_wake = int(engine_wake)
        self.buffers = []
        w = self._workload(kind, shape, dev, g)
        cfg.kind, cfg.M, cfg.N, cfg.K, cfg.chunk_bytes, cfg.bytes = w["kind"], w["M"], w["N"], w["K"], w["chunk"], w["bytes"]
        cfg.a, cfg.b, cfg.c = w["a"], w["b"], w["c"]
        self.work_per_unit, self.unit_name = w["work"], w["unit"]
        self.alt_kind = None
        if alt:
            alt = dict(alt)
            self.alt_kind = alt.pop("kind")
            v = self._workload(self.alt_kind, alt, dev, g)
            cfg.alt_kind, cfg.alt_M, cfg.alt_N, cfg.alt_K = v["kind"], v["M"], v["N"], v["K"]
            cfg.alt_chunk_bytes, cfg.alt_bytes = v["chunk"], v["bytes"]
            cfg.alt_a, cfg.alt_b, cfg.alt_c = v["a"], v["b"], v["c"]
            self.alt_work_per_unit = v["work"]
        torch.cuda.synchronize(dev)
        self.cfg = cfg
        h = self.L.gpbs_runner_create(ctx.h, C.byref(cfg))
        if not h:
            raise RuntimeError(f"runner_create failed for {kind}")
        self.h = C.c_void_p(h)

    def _workload(self, kind, shape, dev, g) -> dict:
        """Device buffers + ABI fields of one workload kind."""
        M = Nn = K = chunk = nbytes = 0
        b = None
        if kind == "gemm":
            M, Nn, K = shape.get("M", 4096), shape.get("N", 4096), shape.get("K", 4096)
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            b = torch.randn(Nn, K, device=dev, dtype=torch.bfloat16, generator=g)
            c = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
            work, unit = 2.0 * M * Nn * K, "FLOP"
        elif kind in ("stream", "reduce"):
            nbytes = int(shape.get("bytes", 1 << 30))
            chunk = int(shape.get("chunk_bytes", 1 << 19))
            n = nbytes // 2
            a = torch.randn(n, device=dev, dtype=torch.bfloat16, generator=g)
            b = torch.randn(n, device=dev, dtype=torch.bfloat16, generator=g) if kind == "reduce" else None
            c = torch.empty(n, device=dev, dtype=torch.bfloat16)
            work, unit = float(nbytes * (2 if kind == "stream" else 3)), "B"  # bytes moved
        elif kind == "allreduce":  # IPC all-reduce tenant: buffers live in the IpcColl
            coll = shape["coll"]
            nbytes, chunk = coll.nbytes, int(shape.get("chunk_bytes", 1 << 19))
            M, Nn, K = coll.world, coll.rank, int(shape.get("timeout_ms", 5000))
            # bytes moved per unit by this rank: world reads + world writes of its slice
            work, unit = float(2 * nbytes), "B"
            return {"kind": hipabi.KIND[kind], "M": M, "N": Nn, "K": K, "chunk": chunk, "bytes": nbytes,
                    "a": coll.desc, "b": None, "c": None, "work": work, "unit": unit}
        elif kind == "gemv":
            M, K = shape.get("M", 8192), shape.get("K", 8192)
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            b = torch.randn(K, device=dev, dtype=torch.bfloat16, generator=g)
            c = torch.empty(M, device=dev, dtype=torch.float32)
            work, unit = float(M * K * 2), "B"
        else:
            raise ValueError(kind)
        for t in (a, b, c):
            if t is not None:
                self.buffers.append(t)
        return {"kind": hipabi.KIND[kind], "M": M, "N": Nn, "K": K, "chunk": chunk, "bytes": nbytes,
                "a": a.data_ptr(), "b": b.data_ptr() if b is not None else None, "c": c.data_ptr(),
                "work": work, "unit": unit}

    def set_phase(self, alt: int) -> int:
        """Phase-changing tenant: fresh units run the alternate workload (1)
        or the primary one (0); returns the previous phase."""
        rc = self.L.gpbs_runner_set_phase(self.h, int(alt))
        if rc < 0:
            raise RuntimeError("set_phase: runner has no alternate workload")
        return rc

    def submit(self, units: int = 1):
        self.L.gpbs_runner_submit(self.h, units)

    def wait(self, timeout_s: float = 0.0) -> int:
        rc = self.L.gpbs_runner_wait(self.h, int(timeout_s * 1e9))
        if rc == -110:
            raise TimeoutError(f"runner {self.kind} (tenant {self.tenant}) timed out")
        if rc:
            raise RuntimeError(f"runner {self.kind} failed rc={rc}")
        return rc

    def queue_index(self) -> int:
        """The process pool's CU-masked queue this runner launches on (-1: its own stream)."""
        return int(self.L.gpbs_runner_queue(self.h))

    def stats(self) -> RunnerStats:
        s = hipabi.RunnerStats()
        self.L.gpbs_runner_stats(self.h, C.byref(s))
        return RunnerStats(**{k: getattr(s, k) for k, _ in s._fields_})

    def latencies(self, clear=False) -> List[int]:
        n = self.L.gpbs_runner_latencies(self.h, None, 0, 0)
        arr = (C.c_int64 * max(1, n))()
        n = self.L.gpbs_runner_latencies(self.h, arr, n, int(clear))
        return list(arr[:n])

    def reset_stats(self):
        self.L.gpbs_runner_reset_stats(self.h)

    def cancel(self) -> int:
        """Drop the units not launched yet (in-flight ones complete)."""
        return int(self.L.gpbs_runner_cancel(self.h))

    def set_gate(self, gate):
        """False: run anywhere; True: leave revoked XCDs; "park": sleep on them."""
        self.L.gpbs_runner_set_gate(self.h, 2 if gate == "park" else int(bool(gate)))

    def set_engine_wake(self, on: bool):
        self.L.gpbs_runner_set_engine_wake(self.h, int(on))

    def close(self):
        if getattr(self, "h", None):
            self.L.gpbs_runner_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
