"""Pythonic handle on the native engine (libgpbs.so).

``Engine`` is the in-process scheduler instance (one per GPU rank).  Every
method is a thin wrapper over the C ABI in csrc/include/gpbs/gpbs.h; policy
logic lives in C++ (csrc/core), never here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional

from .. import _native as N
from .errors import GpbsError

TRACE_EVENTS = {1: "SWITCH", 2: "WAKE", 3: "SLEEP", 4: "ACCT", 5: "ADAPT", 6: "GANG_EPOCH", 7: "REPORT",
                8: "MIGRATE", 9: "PARK", 10: "STEAL", 11: "METRIC", 12: "DEAD", 13: "POOL", 14: "FAULT", 15: "ATC",
                16: "CLASS", 17: "GANG_TIMEOUT"}
EVENT_CODES = {v: k for k, v in TRACE_EVENTS.items()}

PMC_NAMES = ("INST_RETIRED", "CPU_CLK_UNHALTED", "LLC_REFERENCES", "LLC_MISSES")


def boot_params(**kw) -> N.BootParams:
    """Boot parameters with reference defaults; keyword overrides.

    Nested policy constants: ``adapt={'threshold':..}``, ``atc={...}``.
    """
    lib = N.load_core()
    p = N.BootParams()
    lib.gpbs_boot_defaults(C.byref(p))
    for k, v in kw.items():
        if k == "sched":
            p.sched = v.encode()
        elif k in ("adapt", "atc"):
            sub = getattr(p, k)
            for kk, vv in v.items():
                setattr(sub, kk, int(vv))
        else:
            setattr(p, k, int(v))
    return p


@dataclass
class TenantInfo:
    id: int
    name: str
    pool: int
    nslots: int
    weight: int
    cap: int
    paused: int
    alive: bool
    active_slots: int
    tslice_us: int
    tick_period_us: int
    phase: int
    window_left: int
    last_err: int
    last_curr: int
    last_win: int
    pmc: tuple
    cache_miss_rate: int
    cpi: int
    spin_latency: int
    report_count: int
    pending_requests: int
    sched_count: int
    run_ns: int
    shutdown: int = 0
    online_slots: int = 0
    budget_ctx: int = 0      # class_budget: shader engines of every XCD the layout gave the tenant (bit c)
    budget_shared: bool = False
    target_tslice_us: int = 0  # the policy's quantum target (PBS: adaptive); tslice_us is the dispatched one
    switch_cost_us: int = 0    # measured switch cost (drain + ramp) the engine holds
    slo_us: int = 0            # latency target (0: none)
    last_dispatch_us: int = 0  # quantum of its last dispatch


@dataclass
class TraceRec:
    t_ns: int
    event: str
    cpu: int
    a: tuple


class Engine:
    def __init__(self, sched: str = "credit", sim_clock: bool = False, partitions: Optional[Iterable] = None,
                 params: Optional[N.BootParams] = None, **kw):
        self.lib = N.load_core()
        if params is None:
            params = boot_params(sched=sched, sim_clock=int(sim_clock), **kw)
        self.params = params
        self.sim = bool(params.sim_clock)
        h = self.lib.gpbs_engine_create(C.byref(params))
        if not h:
            raise GpbsError(-22, "engine creation failed")
        self.h = C.c_void_p(h)
        self._keep = []  # ctypes callbacks kept alive
        self._trace_cursor = C.c_uint64(0)
        if partitions is not None:
            for part in partitions:
                pid = self.partition_add(*part)  # (gpu, xcd) or (gpu, xcd, ctx)
                self.pool_assign(0, pid)

    # ------------------------------------------------------------ lifecycle
    # Every ABI call goes through ``h``: once closed it raises instead of
    # handing a NULL engine to C (a late reaper / RPC call after close()).
    @property
    def h(self):
        h = self.__dict__.get("_h")
        if h is None:
            raise GpbsError(-19, "engine is closed")
        return h

    @h.setter
    def h(self, v):
        self.__dict__["_h"] = v

    @property
    def closed(self) -> bool:
        return self.__dict__.get("_h") is None

    def close(self):
        h = self.__dict__.get("_h")
        if h is not None:
            self.__dict__["_h"] = None
            self.lib.gpbs_engine_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc, what=""):
        return N.check(rc, what)

    # ------------------------------------------------------ topology/pools
    def partition_add(self, gpu: int, xcd: int, ctx: int = 0) -> int:
        return self._chk(self.lib.gpbs_partition_add_ctx(self.h, gpu, xcd, ctx), "partition_add")

    @property
    def num_partitions(self) -> int:
        return self.lib.gpbs_num_partitions(self.h)

    def pool_create(self, name: str, sched: str = "") -> int:
        return self._chk(self.lib.gpbs_pool_create(self.h, name.encode(), sched.encode()), "pool_create")

    def pool_destroy(self, pool: int):
        return self._chk(self.lib.gpbs_pool_destroy(self.h, pool), "pool_destroy")

    def pool_rename(self, pool: int, name: str):
        return self._chk(self.lib.gpbs_pool_rename(self.h, pool, name.encode()), "pool_rename")

    def pool_find(self, name: str) -> int:
        return self._chk(self.lib.gpbs_pool_find(self.h, name.encode()), f"pool '{name}'")

    def pool_assign(self, pool: int, part: int):
        return self._chk(self.lib.gpbs_pool_assign(self.h, pool, part), "pool_assign")

    def pool_unassign(self, pool: int, part: int):
        return self._chk(self.lib.gpbs_pool_unassign(self.h, pool, part), "pool_unassign")

    def pools(self) -> List[int]:
        n = self.lib.gpbs_pool_list(self.h, None, 0)
        arr = (C.c_int * max(n, 1))()
        n = self.lib.gpbs_pool_list(self.h, arr, n)
        return list(arr[:n])

    def pool_info(self, pool: int) -> Dict:
        name = C.create_string_buffer(64)
        sched = C.create_string_buffer(32)
        mask = (C.c_uint64 * 4)()
        nt = C.c_int(0)
        self._chk(self.lib.gpbs_pool_info(self.h, pool, name, 64, sched, 32, mask, C.byref(nt)), "pool_info")
        cpus = [i for i in range(256) if (mask[i // 64] >> (i % 64)) & 1]
        return {"id": pool, "name": name.value.decode(), "sched": sched.value.decode(), "cpus": cpus,
                "n_tenants": nt.value}

    def partition_info(self, part: int) -> Dict:
        o = N.PartitionInfo()
        self._chk(self.lib.gpbs_partition_info(self.h, part, C.byref(o)), "partition_info")
        return {k: getattr(o, k) for k, _ in o._fields_}

    # ------------------------------------------------------ tenants/slots
    def tenant_create(self, name: str, nslots: int = 1, pool: int = 0, weight: int = -1, cap: int = -1) -> int:
        return self._chk(self.lib.gpbs_tenant_create(self.h, name.encode(), pool, nslots, weight, cap),
                         f"tenant_create({name})")

    def tenant_destroy(self, t: int):
        return self._chk(self.lib.gpbs_tenant_destroy(self.h, t), "tenant_destroy")

    def tenant_find(self, name: str) -> int:
        return self._chk(self.lib.gpbs_tenant_find(self.h, name.encode()), f"tenant '{name}'")

    def tenants(self) -> List[int]:
        n = self.lib.gpbs_tenant_list(self.h, None, 0)
        arr = (C.c_int * max(n, 1))()
        n = self.lib.gpbs_tenant_list(self.h, arr, n)
        return list(arr[:n])

    def tenant_move(self, t: int, pool: int):
        return self._chk(self.lib.gpbs_tenant_move(self.h, t, pool), "tenant_move")

    def pause(self, t: int):
        return self._chk(self.lib.gpbs_tenant_pause(self.h, t), "pause")

    def unpause(self, t: int):
        return self._chk(self.lib.gpbs_tenant_unpause(self.h, t), "unpause")

    def set_nslots(self, t: int, n: int):
        return self._chk(self.lib.gpbs_tenant_set_nslots(self.h, t, n), "slot-set")

    def slot_id(self, t: int, idx: int) -> int:
        return self._chk(self.lib.gpbs_slot_id(self.h, t, idx), "slot_id")

    def wake(self, t: int, idx: int = -1):
        return self._chk(self.lib.gpbs_slot_wake(self.h, t, idx), "wake")

    def block(self, t: int, idx: int = -1):
        return self._chk(self.lib.gpbs_slot_block(self.h, t, idx), "block")

    def yield_(self, t: int, idx: int = -1):
        return self._chk(self.lib.gpbs_slot_yield(self.h, t, idx), "yield")

    def pin(self, t: int, idx: int, parts: Iterable[int]):
        m = (C.c_uint64 * 4)()
        for p in parts:
            m[p // 64] |= 1 << (p % 64)
        return self._chk(self.lib.gpbs_slot_pin(self.h, t, idx, m), "slot-pin")

    def tenant_vpmu(self, t: int) -> Dict[str, int]:
        """Cumulative counters the scheduler measured and attributed to the
        tenant (the vPMU mirror's source): INST, CYCLES, LLC refs, LLC misses."""
        a = (C.c_uint64 * 4)()
        self._chk(self.lib.gpbs_tenant_vpmu(self.h, t, a), "tenant_vpmu")
        return dict(zip(PMC_NAMES, list(a)))

    def tenant_info(self, t: int) -> TenantInfo:
        o = N.TenantInfo()
        self._chk(self.lib.gpbs_tenant_info(self.h, t, C.byref(o)), "tenant_info")
        return TenantInfo(id=o.id, name=o.name.decode(), pool=o.pool, nslots=o.nslots, weight=o.weight, cap=o.cap,
                          paused=o.paused, alive=bool(o.alive), active_slots=o.active_slots, tslice_us=o.tslice_us,
                          tick_period_us=o.tick_period_us, phase=o.phase, window_left=o.window_left,
                          last_err=o.last_err, last_curr=o.last_curr, last_win=o.last_win, pmc=tuple(o.pmc),
                          cache_miss_rate=o.cache_miss_rate, cpi=o.cpi, spin_latency=o.spin_latency,
                          report_count=o.report_count, pending_requests=o.pending_requests,
                          sched_count=o.sched_count, run_ns=o.run_ns, shutdown=o.shutdown,
                          online_slots=o.online_slots, budget_ctx=o.budget_ctx, budget_shared=bool(o.budget_shared),
                          target_tslice_us=o.target_tslice_us, switch_cost_us=o.switch_cost_us, slo_us=o.slo_us,
                          last_dispatch_us=o.last_dispatch_us)

    def slot_info(self, sid: int) -> Dict:
        o = N.SlotInfo()
        self._chk(self.lib.gpbs_slot_info(self.h, sid, C.byref(o)), "slot_info")
        d = {k: getattr(o, k) for k, _ in o._fields_ if k not in ("pmc", "affinity")}
        d["pmc"] = tuple(o.pmc)
        return d

    def adapt_state(self, t: int) -> N.AdaptState:
        s = N.AdaptState()
        self._chk(self.lib.gpbs_tenant_adapt_state(self.h, t, C.byref(s), 0), "adapt_state")
        return s

    def set_adapt_state(self, t: int, s: N.AdaptState):
        return self._chk(self.lib.gpbs_tenant_adapt_state(self.h, t, C.byref(s), 1), "set_adapt_state")

    FAULT_KINDS = ("counter_drop", "counter_reset", "heartbeat_drop", "actuate_delay", "timer_jitter", "rank_hang",
                   "torn_page")

    def fault_set(self, spec: str) -> int:
        """Arm fault injection: "kind=ppm[:param],...,seed=N" (see gpbs.h)."""
        return self.lib.gpbs_fault_set(self.h, spec.encode())

    def fault_hits(self) -> Dict[str, int]:
        arr = (C.c_uint64 * len(self.FAULT_KINDS))()
        n = self.lib.gpbs_fault_hits(self.h, arr, len(self.FAULT_KINDS))
        return {k: arr[i] for i, k in enumerate(self.FAULT_KINDS[:n])}

    GANG_NONE, GANG_FAVOUR, GANG_EXCLUDE = 0, 1, 2

    def gang_set(self, t: int, state: int, until_ns: int):
        """Cross-GPU gang window for tenant t (0 none, 1 favoured, 2 excluded)
        until `until_ns` on this engine's clock."""
        return self._chk(self.lib.gpbs_gang_set(self.h, t, int(state), int(until_ns)), "gang_set")

    def heartbeat(self, t: int):
        return self._chk(self.lib.gpbs_tenant_heartbeat(self.h, t), "heartbeat")

    # ------------------------------------------------------ sched control
    def sched_credit_get(self, t: int):
        w, c = C.c_int(), C.c_int()
        self._chk(self.lib.gpbs_sched_credit_get(self.h, t, C.byref(w), C.byref(c)), "sched_credit_get")
        return w.value, c.value

    def sched_credit_set(self, t: int, weight: int = -1, cap: int = -1):
        return self._chk(self.lib.gpbs_sched_credit_set(self.h, t, weight, cap), "sched_credit_set")

    def sched_ext_get(self, t: int) -> Dict[str, int]:
        """Scheduler-specific parameters (credit2: weight; sedf: period_us,
        slice_us, latency_us, extratime, weight), plus the slot-0 credit."""
        x = N.SchedExt()
        self._chk(self.lib.gpbs_sched_ext(self.h, t, 0, C.byref(x)), "sched_ext_get")
        return {k: getattr(x, k) for k, _ in N.SchedExt._fields_}

    def sched_ext_set(self, t: int, weight: int = 0, period_us: int = 0, slice_us: int = 0, latency_us: int = -1,
                      extratime: int = -1):
        """xl sched-credit2 -w / sched-sedf -p -s -l -e -w (0 / -1 = unset)."""
        x = N.SchedExt(weight, period_us, slice_us, latency_us, extratime, 0)
        self._chk(self.lib.gpbs_sched_ext(self.h, t, 1, C.byref(x)), "sched_ext_set")
        return {k: getattr(x, k) for k, _ in N.SchedExt._fields_}

    def atc_sync(self, pool: int = 0, global_min_us: int = 0) -> int:
        """ATC pool across GPUs: apply a node-wide minimum slice (> 0) and
        return this pool's local minimum (us) of its last apply."""
        return self._chk(self.lib.gpbs_atc_sync(self.h, pool, int(global_min_us)), "atc_sync")

    def arinc653_set(self, pool: int, major_frame_us: float, entries):
        """Install an ARINC 653 table on an arinc653 pool: entries =
        [(tenant, slot or -1, runtime_us), ...] (a653sched_adjust_global put)."""
        s = N.ArincSchedule()
        s.major_frame_ns = int(major_frame_us * 1000)
        s.num_entries = len(entries)
        if len(entries) > 64:
            raise GpbsError(-22, "at most 64 ARINC 653 entries")
        for i, (t, slot, rt) in enumerate(entries):
            s.entries[i].tenant, s.entries[i].slot, s.entries[i].runtime_ns = int(t), int(slot), int(rt * 1000)
        self._chk(self.lib.gpbs_arinc653_set(self.h, pool, C.byref(s)), "arinc653_set")

    def arinc653_get(self, pool: int = 0) -> Dict:
        s = N.ArincSchedule()
        self._chk(self.lib.gpbs_arinc653_get(self.h, pool, C.byref(s)), "arinc653_get")
        return {"major_frame_us": s.major_frame_ns / 1000, "explicit": bool(s.is_explicit),
                "entries": [(s.entries[i].tenant, s.entries[i].slot, s.entries[i].runtime_ns / 1000)
                            for i in range(s.num_entries)]}

    def sched_params_get(self, pool: int = 0):
        ts, rl = C.c_int(), C.c_int()
        self._chk(self.lib.gpbs_sched_params_get(self.h, pool, C.byref(ts), C.byref(rl)), "sched_params_get")
        return ts.value, rl.value

    def sched_params_set(self, pool: int, tslice_us: int, ratelimit_us: int):
        return self._chk(self.lib.gpbs_sched_params_set(self.h, pool, tslice_us, ratelimit_us), "sched_params_set")

    def sched_name(self, pool: int = 0) -> str:
        b = C.create_string_buffer(32)
        self._chk(self.lib.gpbs_sched_name(self.h, pool, b, 32), "sched_name")
        return b.value.decode()

    # ------------------------------------------------ paravirtual channel
    def report_wait(self, t: int, wait_ns: int, kind: int = 1):
        return self._chk(self.lib.gpbs_report_wait(self.h, t, int(wait_ns), kind), "report_wait")

    def report_requests(self, t: int, n: int):
        return self._chk(self.lib.gpbs_report_requests(self.h, t, n), "report_requests")

    # ------------------------------------------------------- backends
    def set_counter_ops(self, ops: Optional[N.CounterOps]):
        if ops is not None:
            self._keep.append(ops)
        return self.lib.gpbs_set_counter_ops(self.h, C.byref(ops) if ops is not None else None)

    def set_actuator_ops(self, ops: Optional[N.ActuatorOps]):
        if ops is not None:
            self._keep.append(ops)
        return self.lib.gpbs_set_actuator_ops(self.h, C.byref(ops) if ops is not None else None)

    def fault_fire(self, kind: str) -> int:
        """Injection point outside the engine: the kind's param (>= 0) when it
        fires this time, -1 otherwise (GPBS_FAULT / fault_set)."""
        return int(self.lib.gpbs_fault_fire(self.h, kind.encode()))

    def gang_timeout(self, epoch: int, rank: int, waited_us: int):
        """This rank missed a gang deadline: clear all cross-GPU windows,
        count it and trace GANG_TIMEOUT (scheduling continues locally)."""
        return self.lib.gpbs_gang_timeout(self.h, epoch & 0xFFFFFFFF, rank, min(int(waited_us), 0xFFFFFFFF))

    def mux_add(self, part_lo: int, part_hi: int, act: Optional[N.ActuatorOps] = None,
                ctr: Optional[N.CounterOps] = None) -> int:
        """Add a per-GPU backend serving partitions [part_lo, part_hi): one
        engine spanning several GPUs drives one actuator + counter backend
        per GPU (gpbs_backend_mux_add)."""
        for o in (act, ctr):
            if o is not None:
                self._keep.append(o)
        rc = self.lib.gpbs_backend_mux_add(self.h, part_lo, part_hi, C.byref(act) if act is not None else None,
                                           C.byref(ctr) if ctr is not None else None)
        return self._chk(rc, "backend_mux_add")

    def mux_clear(self):
        return self.lib.gpbs_backend_mux_clear(self.h)

    def mux_count(self) -> int:
        return self.lib.gpbs_backend_mux_count(self.h)

    def set_pmc(self, slot_id: int, pmc):
        arr = (C.c_uint64 * 4)(*[int(x) for x in pmc])
        return self._chk(self.lib.gpbs_slot_set_pmc(self.h, slot_id, arr), "set_pmc")

    # ------------------------------------------------------------ time
    def now(self) -> int:
        return self.lib.gpbs_now(self.h)

    def advance(self, t_ns: int):
        return self._chk(self.lib.gpbs_advance(self.h, int(t_ns)), "advance")

    def advance_us(self, dt_us: float):
        return self.advance(self.now() + int(dt_us * 1000))

    def start(self):
        return self._chk(self.lib.gpbs_start(self.h), "start")

    def stop(self):
        return self.lib.gpbs_stop(self.h)

    def poll(self):
        return self.lib.gpbs_poll(self.h)

    # --------------------------------------------------- observability
    def debug_keys(self, keys: str) -> str:
        """Run keyhandlers (r, q, z, p, P, c, h); output also goes to dmesg."""
        size = 1 << 21
        buf = C.create_string_buffer(size)
        self.lib.gpbs_debug_keys(self.h, keys.encode(), buf, size)
        return buf.value.decode()

    def dmesg(self, clear: bool = False) -> str:
        size = 1 << 21
        buf = C.create_string_buffer(size)
        self.lib.gpbs_dmesg(self.h, buf, size, int(clear))
        return buf.value.decode()

    def trace(self, max_records: int = 65536, from_start: bool = False) -> List[TraceRec]:
        if from_start:
            self._trace_cursor = C.c_uint64(0)
        arr = (N.TraceRecord * max_records)()
        lost = C.c_uint64(0)
        n = self.lib.gpbs_trace_read(self.h, C.byref(self._trace_cursor), arr, max_records, C.byref(lost))
        self.trace_lost = lost.value
        return [TraceRec(r.t_ns, TRACE_EVENTS.get(r.event, str(r.event)), r.cpu, tuple(r.a)) for r in arr[:n]]

    def trace_set_mask(self, events: Optional[Iterable[str]] = None):
        mask = (1 << 64) - 1 if events is None else sum(1 << EVENT_CODES[e] for e in events)
        return self.lib.gpbs_trace_set_mask(self.h, mask)

    def trace_emit(self, event: str, cpu: int, *a):
        a = list(a) + [0] * (4 - len(a))
        return self.lib.gpbs_trace_emit(self.h, EVENT_CODES[event], cpu, *[int(x) & 0xFFFFFFFF for x in a[:4]])

    def perfc(self) -> Dict[str, int]:
        n = self.lib.gpbs_perfc_count()
        arr = (C.c_uint64 * n)()
        self.lib.gpbs_perfc_read(self.h, arr, n)
        return {self.lib.gpbs_perfc_name(i).decode(): arr[i] for i in range(n)}

    def perfc_reset(self):
        return self.lib.gpbs_perfc_reset(self.h)

    def bound_stats(self, t: int, reset: bool = False) -> Dict[str, int]:
        """Metric periods the tenant was measured in and, of those, the ones
        its quantum sat at the adapt bounds (min_us / max_us)."""
        o = (C.c_uint64 * 3)()
        rc = self.lib.gpbs_tenant_bound_stats(self.h, t, o, int(reset))
        if rc < 0:
            return {"periods": 0, "at_min": 0, "at_max": 0}
        return {"periods": int(o[0]), "at_min": int(o[1]), "at_max": int(o[2])}

    def measure(self, t: int, us: int = -1) -> int:
        """Ask for a measurement tenure of at least `us` for the tenant's next
        tenure (0 cancels; -1 only reads).  Returns the tenures extended so far."""
        return int(self.lib.gpbs_tenant_measure(self.h, t, 0xFFFFFFFF if us < 0 else int(us)))

    def switch_cost(self, t: int, ns: int) -> int:
        """Measured cost of one switch of the tenant's partitions (ns): its
        per-tenant quantum floor in a time-shared region (boot switch_floor_x)."""
        return int(self.lib.gpbs_tenant_switch_cost(self.h, t, int(ns)))

    def set_slo(self, t: int, us: int) -> int:
        """Latency target of a tenant (us, 0 = none): with boot slo_cap, its
        co-sharers' quanta are capped to it."""
        return int(self.lib.gpbs_tenant_slo(self.h, t, int(us)))

    def perfc_prometheus(self, prefix: str = "gpbs") -> str:
        """perfc counters in the Prometheus text exposition format."""
        lines = [f"# TYPE {prefix}_perfc_total counter"]
        lines += [f'{prefix}_perfc_total{{name="{k}"}} {v}' for k, v in self.perfc().items()]
        lp = self.lockprof()
        lines.append(f"# TYPE {prefix}_lock_seconds_total counter")
        lines.append(f'{prefix}_lock_seconds_total{{lock="engine",kind="hold"}} {lp["time_hold_ns"] / 1e9:.9f}')
        lines.append(f'{prefix}_lock_seconds_total{{lock="engine",kind="block"}} {lp["time_block_ns"] / 1e9:.9f}')
        return "\n".join(lines) + "\n"

    def lockprof(self, reset: bool = False) -> Dict[str, int]:
        """Engine-mutex lock profile (xenlockprof analog)."""
        o = N.LockProf()
        self.lib.gpbs_lockprof(self.h, C.byref(o), int(reset))
        return {k: getattr(o, k) for k, _ in o._fields_}

    def watchdog(self, t: int, wid: int = 0, timeout_ms: int = 0) -> int:
        """SCHEDOP_watchdog: wid 0 allocates (returns the id), else re-arm
        (timeout_ms > 0) or free (0)."""
        return self._chk(self.lib.gpbs_watchdog(self.h, t, wid, timeout_ms), "watchdog")

    def check(self) -> str:
        buf = C.create_string_buffer(1 << 16)
        self.lib.gpbs_check_invariants(self.h, buf, 1 << 16)
        return buf.value.decode()
