"""Cross-GPU gang scheduling: epoch-synchronised windows over the per-GPU
engines of a node (SURVEY §2.6 C16 -- the reference co-schedules nothing; its
spin-latency channel P2 only measures the lock-holder-preemption symptom that
gang scheduling removes).

Every rank (one process per GPU) runs one ``GangCoordinator`` thread bound to
its GPU's engine.  Each epoch it all-reduces (MIN) a small vector over the
gang process group: per gang tenant "has demand here", plus a "keep going"
flag.  The collective's return is the common epoch boundary on every rank --
no clock synchronisation is needed -- and the window decision is a pure
function of the reduced vector and the epoch counter, so all ranks agree
without a second message.  Gang tenants (e.g. the all-reduce tenant whose
RCCL ranks span the GPUs) take ``share`` of the epochs, round-robin among
those with demand on every rank; in their epoch they are favoured on every
partition that holds one of their slots, otherwise excluded
(``Engine.gang_set``), so their ranks never run half-scheduled and a
collective never waits on a descheduled peer.

The vector is a few int32 (<= 4 KiB for any tenant count): latency-bound, so
the default group is node-local gloo (shared-memory/TCP loopback, ~50-100 us);
an RCCL group can be passed instead (``device="cuda"``) to ride xGMI.
Stopping is collective too: a rank that wants to stop contributes 0 to the
flag and every rank leaves at the same epoch.

The same epoch carries two node-level exchanges of the reference's
intra-host traffic:

* ``atc_pool``: the pool's local ATC minimum slice rides the MIN vector and
  the node-wide minimum is applied on every GPU (sched_credit_atc.c applies
  the global minimum to every domain each 21 ms period);
* ``metric_tenants``: every ``metric_every`` epochs the tenants' last-period
  counter deltas (INST, CYCLES, L2 refs, L2 misses) are SUM-reduced, so every
  rank sees node-wide per-tenant metrics (``node_metrics``) -- the master's
  cross-CPU pmc gather of csched_dom_metric_update, without a master.
Transports (``transport=``):

* ``shm`` -- all ranks of one node meet in a POSIX shared-memory region
  (csrc/comm/gang_shm.cpp): microseconds per epoch, no kernel launch, no CU
  time and no xGMI traffic next to the tenants' own RCCL all-reduce.  The
  default for the one-node bench.
* ``gloo`` -- node-local gloo (shared memory / TCP loopback, ~50-100 us).
* ``rccl`` -- an RCCL group over xGMI (``device="cuda:N"``): the cross-node
  capable path; latency-bound 4 KiB all-reduces cost tens of us and occupy
  CUs for their kernels.

Wait-driven windows (``wait_driven=True``): the vector also
carries each gang tenant's wait reported on this GPU since the last epoch
(RCCL-collective waits timed by runtime/waitprobe.py), MAX-reduced.  A gang
tenant then gets aligned windows only while its worst rank waits on peers
(EWMA >= ``wait_on_frac`` of the epoch) and is scheduled locally otherwise --
gang scheduling driven by the lock-holder-preemption symptom P2 measures.

Every epoch has a deadline (``deadline_ms``).  A rank that misses it -- one
rank hung (GPBS_FAULT ``rank_hang``), descheduled or dead -- makes the others'
exchange time out: they record GANG_TIMEOUT (trace + perfc ``gang_timeout``),
clear every gang window and go on scheduling locally instead
of stalling every GPU's gang thread.  With ``reform=True`` (shm transport)
the survivors then re-form: the first to claim the next view generation
waits a join window and publishes the member set and a common first epoch
(csrc/comm/gang_shm.cpp), so gang windows continue among the members; the
laggard finds the view changed when it returns and asks to rejoin (the
members join that view at their next exchange); a rank dropped twice stays
local (C12: the reference moves the pool master's timers to a surviving CPU).  Epoch-start skew across ranks (the
spread of the previous epoch's return time, on the node's shared monotonic
clock) rides the exchange and is reported in ``stats()``.
"""
from __future__ import annotations

import ctypes as C
import threading
import time
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..utils import roctx

FAVOUR, EXCLUDE, NONE = 1, 2, 0
NO_ATC = 1 << 30  # MIN-neutral stand-in for "no ATC pool on this rank"


class _DistTransport:
    """gloo / RCCL: asynchronous collectives polled against the deadline."""

    def __init__(self, group, device):
        self.group = group
        self.dev = torch.device(device) if device else torch.device("cpu")
        if self.dev.type == "cuda":
            torch.cuda.set_device(self.dev)

    def _run(self, vals, op, deadline_ns):
        buf = torch.tensor(vals, dtype=torch.int64, device=self.dev)
        work = dist.all_reduce(buf, op=op, group=self.group, async_op=True)
        while not work.is_completed():
            if time.monotonic_ns() > deadline_ns:
                return None  # left pending: this group is abandoned by the caller
            time.sleep(20e-6)
        work.wait()
        return buf.tolist()

    def reduce_min(self, vals, deadline_ns):
        return self._run(vals, dist.ReduceOp.MIN, deadline_ns)

    def reduce_sum(self, vals, deadline_ns):
        return self._run(vals, dist.ReduceOp.SUM, deadline_ns)

    def close(self):
        pass


class _ShmTransport:
    """One-node ranks: native shared-memory all-gather (csrc/comm/gang_shm.cpp),
    with elastic re-formation of the member set after a missed deadline."""

    def __init__(self, name: str, rank: int, world: int, nvals: int):
        from .. import _native as N
        self.lib = N.load_core()
        self.world, self.nvals = world, nvals
        self.h = self.lib.gpbs_gang_shm_open(name.encode(), rank, world, nvals)
        if not self.h:
            raise RuntimeError(f"gang shm region {name!r} could not be opened")
        self.seq = 0
        self.members = list(range(world))
        self.excluded = False  # the gang re-formed without this rank
        self.why = ""          # why the last exchange returned None: timeout / excluded / view

    def _gather(self, vals, deadline_ns):
        n = self.nvals
        vals = list(vals) + [0] * (n - len(vals))
        self.seq += 1
        src = (C.c_int64 * n)(*vals)
        out = (C.c_int64 * (n * self.world))()
        rc = self.lib.gpbs_gang_shm_allgather(C.c_void_p(self.h), self.seq, src, out, deadline_ns)
        if rc == -110:
            self.why = "timeout"
            return None
        if rc == -116:  # a view was published without us: we were the laggard
            self.excluded, self.why = True, "excluded"
            return None
        if rc == -117:  # a newer view is being formed (a rank asked to rejoin): join it
            self.why = "view"
            return None
        if rc:
            raise RuntimeError(f"gang shm all-gather failed ({rc})")
        return [list(out[r * n:(r + 1) * n]) for r in self.members]

    def reform(self, join_ms: float, deadline_ms: float) -> Optional[int]:
        """After a missed deadline, an exclusion (rejoin request) or a view
        change: join the next view.  Returns the first epoch of the new view
        (the same on every member) when this rank is a member, None when it
        was left out, has used up its rejoins, or no view appeared."""
        m, base = C.c_uint64(0), C.c_uint64(0)
        now = time.monotonic_ns()
        rc = self.lib.gpbs_gang_shm_reform(C.c_void_p(self.h), int(join_ms * 1e6),
                                           now + int((join_ms + deadline_ms) * 1e6), C.byref(m), C.byref(base))
        if rc:
            self.excluded = self.excluded or rc == -1
            return None
        self.excluded = False
        self.members = [r for r in range(self.world) if (m.value >> r) & 1]
        self.seq = base.value - 1
        return base.value

    def reduce_min(self, vals, deadline_ns):
        rows = self._gather(vals, deadline_ns)
        return None if rows is None else [min(c) for c in zip(*rows)][:len(vals)]

    def reduce_sum(self, vals, deadline_ns):
        rows = self._gather(vals, deadline_ns)
        return None if rows is None else [sum(c) for c in zip(*rows)][:len(vals)]

    def close(self):
        if self.h:
            self.lib.gpbs_gang_shm_close(C.c_void_p(self.h))
            self.h = None


class _XgmiTransport:
    """Device-side epoch exchange over xGMI: every rank's board
    in uncached VRAM, IPC-mapped by every peer; one exchange is one 64-lane
    kernel that writes this rank's values and sequence number into every
    peer's board and waits for every peer's (csrc/hip/coll_kernels.hip
    ``k_gang_exchange``).  Handles are swapped once, at start-up, over the
    host group; no host collective runs per epoch.  A missed deadline
    degrades the rank to local scheduling (no re-formation: the view is the
    rank set the boards were mapped for)."""

    def __init__(self, rank: int, world: int, nvals: int, device: int, gather: Callable):
        from ..ops.kernels import lib as hiplib
        self.L = hiplib()
        self.world, self.nvals = world, nvals
        h = self.L.gpbs_gangx_create(device, rank, world, nvals)
        if not h:
            raise RuntimeError("gpbs_gangx_create failed")
        self.h = C.c_void_p(h)
        nb = self.L.gpbs_gangx_handle_bytes()
        buf = (C.c_char * nb)()
        if self.L.gpbs_gangx_export(self.h, buf) != nb:
            self.close()
            raise RuntimeError("hipIpcGetMemHandle (gang board) failed")
        for peer, hb in enumerate(gather(bytes(buf))):
            if peer != rank and self.L.gpbs_gangx_open(self.h, peer, (C.c_char * nb).from_buffer_copy(hb)):
                self.close()
                raise RuntimeError(f"hipIpcOpenMemHandle of rank {peer}'s gang board failed")
        if self.L.gpbs_gangx_finalize(self.h):
            self.close()
            raise RuntimeError("gpbs_gangx_finalize failed")
        self.seq = 0
        self.members = list(range(world))
        self.excluded = False
        self.why = ""

    def _gather(self, vals, deadline_ns):
        n = self.nvals
        vals = list(vals) + [0] * (n - len(vals))
        self.seq += 1
        src = (C.c_longlong * n)(*vals)
        out = (C.c_longlong * (n * self.world))()
        rc = self.L.gpbs_gangx_exchange(self.h, self.seq, src, n, out, int(deadline_ns))
        if rc == -110:
            self.why = "timeout"
            return None
        if rc:
            raise RuntimeError(f"gang xGMI exchange failed ({rc})")
        return [list(out[r * n:(r + 1) * n]) for r in range(self.world)]

    def reduce_min(self, vals, deadline_ns):
        rows = self._gather(vals, deadline_ns)
        return None if rows is None else [min(c) for c in zip(*rows)][:len(vals)]

    def reduce_sum(self, vals, deadline_ns):
        rows = self._gather(vals, deadline_ns)
        return None if rows is None else [sum(c) for c in zip(*rows)][:len(vals)]

    def stats(self) -> Dict[str, int]:
        o = (C.c_uint64 * 3)()
        self.L.gpbs_gangx_stats(self.h, o)
        return {"exchanges": o[0], "relaunches": o[1], "timeouts": o[2]}

    def close(self):
        if self.h:
            self.L.gpbs_gangx_destroy(self.h)
            self.h = None


class GangCoordinator:
    def __init__(self, engine, group, tenants: List[int], epoch_ms: float = 4.0, share: float = 0.5,
                 device: Optional[str] = None, demand: Optional[Callable[[int], bool]] = None,
                 slack_ms: float = 1.0, atc_pool: Optional[int] = None,
                 metric_tenants: Optional[List[int]] = None, metric_every: int = 5,
                 transport: str = "dist", shm_name: Optional[str] = None, rank: Optional[int] = None,
                 world: Optional[int] = None, deadline_ms: float = 200.0, wait_driven: bool = False,
                 wait_on_frac: float = 0.02, wait_hold_epochs: int = 64, reform: bool = False,
                 join_ms: Optional[float] = None, start_grace_ms: float = 2000.0,
                 native: Optional[bool] = None):
        self.engine = engine
        # the epoch loop as a C++ thread (csrc/comm/gang_coord.cpp) on the shm
        # transport with the engine's own demand; the Python loop stays for the
        # dist/xgmi transports and custom demand callables
        can_native = transport == "shm" and demand is None and engine is not None and hasattr(engine, "h")
        self.native = can_native if native is None else bool(native)
        if self.native and not can_native:
            raise ValueError("native gang coordinator needs transport='shm', an Engine and the engine demand")
        self._nc = None   # native coordinator handle
        self._ntr = None  # its shm transport (owned here)
        self.group = group
        self.tenants = list(tenants)
        self.epoch_ns = int(epoch_ms * 1e6)
        self.share = float(share)
        self.device = device
        self.demand = demand or self._engine_demand
        self.slack_ns = int(slack_ms * 1e6)
        self.epoch = 0
        self.state: Dict[int, int] = {t: NONE for t in self.tenants}
        self._history: List[tuple] = []  # (epoch, {tenant: state}) -- bounded
        self.lat_ns: List[int] = []
        self.skew_ns: List[int] = []
        self._want_stop = False
        self._th: Optional[threading.Thread] = None
        self.error: Optional[BaseException] = None
        self.atc_pool = atc_pool
        self.atc_global_us = 0
        self.metric_tenants = list(metric_tenants or [])
        self.metric_every = max(1, int(metric_every))
        self._node_metrics: Dict[int, Dict[str, int]] = {}
        # node-wide cumulative counters (SUM over ranks of gpbs_tenant_vpmu)
        # at the last metric exchange: exact run totals
        self._node_totals: Dict[int, Dict[str, int]] = {}
        self.metric_syncs = 0
        self.transport = transport
        self.shm_name = shm_name
        self.rank = rank if rank is not None else (dist.get_rank() if dist.is_initialized() else 0)
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.deadline_ns = int(deadline_ms * 1e6)
        self.start_ns = int(max(deadline_ms, start_grace_ms) * 1e6)  # first exchange: start-up skew
        self.timeouts = 0
        self.degraded = False
        # elastic re-formation (shm transport): after a missed deadline the
        # survivors form a new view without the laggard and keep their gang
        # windows; False = degrade to local scheduling for good
        self.reform = bool(reform)
        # join window: the master waits at most this long for the ranks that
        # published the failed epoch (it stops early once they all joined)
        self.join_ms = float(join_ms if join_ms is not None else 2 * deadline_ms)
        self.reforms = 0
        self.members: List[int] = list(range(self.world))
        # K10 -> gang decision: a gang tenant gets aligned windows only while
        # its ranks report waiting on peers (wait reports: runtime/waitprobe.py)
        self.wait_driven = bool(wait_driven)
        self.wait_on_frac = float(wait_on_frac)
        self.wait_hold = int(wait_hold_epochs)
        self.gang_on: Dict[int, bool] = {t: not self.wait_driven for t in self.tenants}
        self._on_since: Dict[int, int] = {t: 0 for t in self.tenants}
        self.wait_ewma_us: Dict[int, int] = {t: 0 for t in self.tenants}
        self._wait_prev: Dict[int, int] = {}
        self.gang_switches = 0

    # ------------------------------------------------------------ demand
    def _engine_demand(self, t: int) -> bool:
        """Tenant has a runnable or running slot on this GPU's engine."""
        try:
            info = self.engine.tenant_info(t)
            for k in range(info.nslots):
                si = self.engine.slot_info(self.engine.slot_id(t, k))
                if si["is_running"] or si.get("runstate", 3) <= 1:
                    return True
        except Exception:
            return False
        return False

    # ----------------------------------------------------------- decision
    def _local_wait_us(self, t: int) -> int:
        """Wait (us) this GPU's tenant reported since the previous epoch."""
        try:
            cur = int(self.engine.tenant_info(t).spin_latency)
        except Exception:
            return 0
        prev = self._wait_prev.get(t, cur)
        self._wait_prev[t] = cur
        return max(0, cur - prev) // 1000

    def update_gang_on(self, epoch: int, max_wait_us: List[int]):
        """Wait-driven gang switch, a pure function of the reduced vector and
        its own history (identical on every rank): on when the EWMA of the
        worst rank's per-epoch wait reaches ``wait_on_frac`` of the epoch; off
        after ``wait_hold`` epochs on if it fell below a quarter of that."""
        on_us = self.wait_on_frac * self.epoch_ns / 1e3
        for t, w in zip(self.tenants, max_wait_us):
            ew = (3 * self.wait_ewma_us[t] + int(w)) // 4
            self.wait_ewma_us[t] = ew
            if not self.gang_on[t] and ew >= on_us:
                self.gang_on[t], self._on_since[t] = True, epoch
                self.gang_switches += 1
            elif self.gang_on[t] and epoch - self._on_since[t] >= self.wait_hold and ew < on_us / 4:
                self.gang_on[t] = False
                self.gang_switches += 1

    def decide(self, epoch: int, demand_all: List[int]) -> Dict[int, int]:
        """Pure function of (epoch, all-rank demand): identical on every rank."""
        eligible = [t for t, d in zip(self.tenants, demand_all) if d and self.gang_on.get(t, True)]
        out = {t: NONE for t in self.tenants}
        if not eligible:
            return out
        period = 8
        gang_slots = max(1, min(period, int(round(self.share * period))))
        pos = epoch % period
        if pos < gang_slots:  # spread one period's gang slots over the eligible tenants
            winner = eligible[(pos + epoch // period) % len(eligible)]
        else:
            winner = None
        for t in eligible:
            out[t] = FAVOUR if t == winner else EXCLUDE
        return out

    # --------------------------------------------------------------- loop
    def _make_transport(self, nvals: int):
        if self.transport == "xgmi":
            dev = torch.device(self.device) if self.device else torch.device("cuda", torch.cuda.current_device())
            group = self.group

            def gather(obj):
                out = [None] * self.world
                dist.all_gather_object(out, obj, group=group)
                return out
            return _XgmiTransport(self.rank, self.world, max(nvals, 8 * len(self.metric_tenants)),
                                  dev.index or 0, gather)
        if self.transport == "shm":
            if not self.shm_name:
                raise ValueError("transport 'shm' needs shm_name (the same fresh name on every rank)")
            return _ShmTransport(self.shm_name, self.rank, self.world, max(nvals, 8 * len(self.metric_tenants)))
        return _DistTransport(self.group, self.device)

    def _timeout(self, waited_ns: int):
        """Deadline missed: degrade this rank to local scheduling."""
        self.timeouts += 1
        self.degraded = True
        if self.engine is not None:
            self.engine.gang_timeout(self.epoch, self.rank, waited_ns // 1000)

    def _loop(self):
        tr = None
        try:
            nt = len(self.tenants)
            tr = self._make_transport(2 * nt + 4)
            t_prev = 0
            while True:
                hang = self.engine.fault_fire("rank_hang") if self.engine is not None else -1
                if hang >= 0:  # GPBS_FAULT rank_hang=ppm:ms -- this rank stalls before the exchange
                    time.sleep(max(hang, 1) / 1e3)
                t0 = time.monotonic_ns()
                vec = [1 if self.demand(t) else 0 for t in self.tenants]
                vec += [-self._local_wait_us(t) for t in self.tenants]  # MIN of -w = -(max over ranks)
                vec += [self._atc_local(), 0 if self._want_stop else 1, t_prev, -t_prev]
                # the first exchange also absorbs the ranks' start-up skew
                dl = self.deadline_ns if self.epoch else self.start_ns
                with roctx.range(f"gpbs:gang_epoch {self.epoch}"):
                    red = tr.reduce_min(vec, t0 + dl)
                t1 = time.monotonic_ns()
                if red is None:
                    why = getattr(tr, "why", "timeout")
                    if why == "timeout":
                        self._timeout(t1 - t0)
                    if self._reform(tr):
                        continue
                    if why != "timeout":  # excluded for good: recorded like a missed deadline
                        self._timeout(t1 - t0)
                    break
                t_prev = t1
                self.lat_ns.append(t1 - t0)
                if red[-2] > 0:  # spread of the previous epoch's return time over the ranks
                    self.skew_ns.append(-red[-1] - red[-2])
                for lst in (self.lat_ns, self.skew_ns):
                    if len(lst) > 4096:
                        del lst[:2048]
                if not red[-3]:
                    break
                if self.atc_pool is not None and 0 < red[-4] < NO_ATC:
                    self.atc_global_us = red[-4]
                    self.engine.atc_sync(self.atc_pool, red[-4])
                if self.metric_tenants and self.epoch % self.metric_every == 0:
                    if not self._sync_metrics(tr):
                        why = getattr(tr, "why", "timeout")
                        if why == "timeout":
                            self._timeout(time.monotonic_ns() - t1)
                        if self._reform(tr):
                            continue
                        if why != "timeout":
                            self._timeout(time.monotonic_ns() - t1)
                        break
                if self.wait_driven:
                    self.update_gang_on(self.epoch, [-x for x in red[nt:2 * nt]])
                dec = self.decide(self.epoch, red[:nt])
                until = self.engine.now() + self.epoch_ns + self.slack_ns
                for t, st in dec.items():
                    self.engine.gang_set(t, st, until)
                self.state = dec
                self._history.append((self.epoch, dict(dec)))
                if len(self._history) > 8192:
                    del self._history[:4096]
                self.epoch += 1
                rest = self.epoch_ns - (time.monotonic_ns() - t1)
                if rest > 0:
                    time.sleep(rest / 1e9)
        except BaseException as e:  # pragma: no cover - surfaced via .error
            self.error = e
        finally:
            if tr is not None and not self.degraded:
                tr.close()
            for t in self.tenants:
                try:
                    self.engine.gang_set(t, NONE, 0)
                except Exception:
                    pass

    def _reform(self, tr) -> bool:
        """Elastic re-formation after a missed deadline (shm transport): the
        survivors agree on a new member set and a common epoch; the gang
        windows resume among them.  False: stay degraded (local scheduling)."""
        if not self.reform or not hasattr(tr, "reform"):
            return False
        with roctx.range("gpbs:gang_reform"):
            base = tr.reform(self.join_ms, self.deadline_ns / 1e6)
        if base is None:
            return False
        self.reforms += 1
        self.degraded = False
        self.members = list(tr.members)
        self.epoch = int(base)  # decisions are a function of the epoch: same on every member
        return True

    def _atc_local(self) -> int:
        if self.atc_pool is None:
            return NO_ATC
        try:
            v = self.engine.atc_sync(self.atc_pool, 0)
        except Exception:
            return NO_ATC
        return v if v > 0 else NO_ATC

    def _sync_metrics(self, tr) -> bool:
        """SUM-reduce the metric tenants' last-period counter deltas (node
        metrics) and their cumulative counters (exact node-wide run totals)."""
        vals, cum = [], []
        for t in self.metric_tenants:
            try:
                vals += [int(x) for x in self.engine.tenant_info(t).pmc]
            except Exception:
                vals += [0, 0, 0, 0]
            try:
                v = self.engine.tenant_vpmu(t)
                cum += [int(v[k]) for k in v]
            except Exception:
                cum += [0, 0, 0, 0]
        red = tr.reduce_sum(vals + cum, time.monotonic_ns() + self.deadline_ns)
        if red is None:
            return False
        out = {}
        for i, t in enumerate(self.metric_tenants):
            inst, cyc, ref, miss = red[4 * i:4 * i + 4]
            out[t] = {"inst": inst, "cycles": cyc, "l2_refs": ref, "l2_misses": miss,
                      "miss_rate": miss * 100000 // inst if inst else 0}
        self._node_metrics = out
        nm = len(self.metric_tenants)
        for i, t in enumerate(self.metric_tenants):
            inst, cyc, ref, miss = red[4 * nm + 4 * i:4 * nm + 4 * i + 4]
            self._node_totals[t] = {"inst": inst, "cycles": cyc, "l2_refs": ref, "l2_misses": miss,
                                    "miss_rate": miss * 100000 // inst if inst else 0}
        self.metric_syncs += 1
        return True

    # ------------------------------------------------------ native loop
    def _start_native(self):
        from .. import _native as N
        nt, nm = len(self.tenants), len(self.metric_tenants)
        if nt > 32 or nm > 32:
            raise ValueError("native gang coordinator: at most 32 gang / metric tenants")
        nvals = max(2 * nt + 4, 8 * nm)
        self._ntr = _ShmTransport(self.shm_name, self.rank, self.world, nvals)
        cfg = N.GangCfg()
        cfg.rank, cfg.ntenants, cfg.nmetric, cfg.metric_every = self.rank, nt, nm, self.metric_every
        for i, t in enumerate(self.tenants):
            cfg.tenants[i] = t
        for i, t in enumerate(self.metric_tenants):
            cfg.metric_tenants[i] = t
        cfg.epoch_ns, cfg.slack_ns, cfg.deadline_ns = self.epoch_ns, self.slack_ns, self.deadline_ns
        cfg.start_ns, cfg.join_ns = self.start_ns, int(self.join_ms * 1e6)
        cfg.share = self.share
        cfg.atc_pool = -1 if self.atc_pool is None else int(self.atc_pool)
        cfg.wait_driven, cfg.wait_on_frac, cfg.wait_hold_epochs = int(self.wait_driven), self.wait_on_frac, self.wait_hold
        cfg.reform = int(self.reform)
        hip = N._hip
        if hip is not None:  # marker ranges on rocprofv3 timelines, as the Python loop's roctx.range
            cfg.roctx_push = C.cast(hip.gpbs_roctx_push, C.c_void_p).value
            cfg.roctx_pop = C.cast(hip.gpbs_roctx_pop, C.c_void_p).value
        self._cfg = cfg  # the thread copies it; keep the function pointers' owner alive anyway
        lib = self.engine.lib
        h = lib.gpbs_gang_coord_start(self.engine.h, C.c_void_p(self._ntr.h), self.world, nvals, C.byref(cfg))
        if not h:
            self._ntr.close()
            raise RuntimeError("gpbs_gang_coord_start failed")
        self._nc = C.c_void_p(h)

    def _pull(self):
        """Refresh the Python view of the native loop's state."""
        if self._nc is None:
            return
        from .. import _native as N
        lib = self.engine.lib
        st = N.GangStats()
        lib.gpbs_gang_coord_stats(self._nc, C.byref(st))
        self._nstats = st
        self._epoch, self.timeouts, self._degraded = st.epochs, st.timeouts, bool(st.degraded)
        self.reforms, self.metric_syncs, self.gang_switches = st.reforms, st.metric_syncs, st.gang_switches
        self.atc_global_us = st.atc_global_us
        self.members = [r for r in range(self.world) if (st.members >> r) & 1]
        o = (C.c_int64 * 3)()
        for i, t in enumerate(self.tenants):
            lib.gpbs_gang_coord_tenant(self._nc, i, o)
            self.state[t], self.gang_on[t], self.wait_ewma_us[t] = int(o[0]), bool(o[1]), int(o[2])
        last, tot = (C.c_int64 * 4)(), (C.c_int64 * 4)()
        nm, nt_ = {}, {}
        for i, t in enumerate(self.metric_tenants):
            lib.gpbs_gang_coord_metrics(self._nc, i, last, tot)
            for dst, src in ((nm, last), (nt_, tot)):
                inst, cyc, ref, miss = (int(x) for x in src)
                dst[t] = {"inst": inst, "cycles": cyc, "l2_refs": ref, "l2_misses": miss,
                          "miss_rate": miss * 100000 // inst if inst else 0}
        if st.metric_syncs:
            self._node_metrics, self._node_totals = nm, nt_
        nt = len(self.tenants)
        cap = 8192
        eps = (C.c_int64 * cap)()
        sts = (C.c_int32 * max(1, cap * nt))()
        n = lib.gpbs_gang_coord_history(self._nc, eps, sts, cap)
        self._history = [(int(eps[j]), {t: int(sts[j * nt + i]) for i, t in enumerate(self.tenants)})
                         for j in range(max(0, n))]

    # live views of the native loop's state (plain attributes for the Python loop)
    @property
    def degraded(self) -> bool:
        self._pull()
        return self._degraded

    @degraded.setter
    def degraded(self, v: bool):
        self._degraded = v

    @property
    def epoch(self) -> int:
        self._pull()
        return self._epoch

    @epoch.setter
    def epoch(self, v: int):
        self._epoch = v

    @property
    def history(self) -> List[tuple]:
        self._pull()
        return self._history

    @property
    def node_metrics(self) -> Dict[int, Dict[str, int]]:
        self._pull()
        return self._node_metrics

    @property
    def node_totals(self) -> Dict[int, Dict[str, int]]:
        self._pull()
        return self._node_totals

    def start(self):
        if self.native:
            self._start_native()
            return self
        self._th = threading.Thread(target=self._loop, daemon=True, name="gpbs-gang")
        self._th.start()
        return self

    def stop(self, timeout: float = 30.0):
        """Collective: returns once every rank has left the epoch loop (a
        degraded rank has already left it)."""
        self._want_stop = True
        if self._nc is not None:
            rc = self.engine.lib.gpbs_gang_coord_stop(self._nc, int(timeout * 1e9))
            self._pull()
            if rc == 0:
                err = self._nstats.error
                self.engine.lib.gpbs_gang_coord_destroy(self._nc)
                self._nc = None
                if not self.degraded:
                    self._ntr.close()
                if err:
                    raise RuntimeError(f"gang shm exchange failed ({err})")
            return
        if self._th is not None:
            self._th.join(timeout)
        if self.error:
            raise self.error

    def stats(self) -> Dict[str, float]:
        if self.native:
            self._pull()
            st = getattr(self, "_nstats", None)
            if st is not None:
                return {"epochs": self.epoch, "transport": self.transport, "native": True,
                        "sync_p50_us": st.sync_p50_ns / 1e3, "sync_p99_us": st.sync_p99_ns / 1e3,
                        "sync_max_us": st.sync_max_ns / 1e3, "skew_p50_us": st.skew_p50_ns / 1e3,
                        "skew_max_us": st.skew_max_ns / 1e3, "timeouts": self.timeouts,
                        "degraded": self.degraded, "reforms": self.reforms, "members": list(self.members),
                        "atc_global_us": self.atc_global_us, "metric_syncs": self.metric_syncs,
                        "wait_driven": self.wait_driven, "gang_on": {str(t): v for t, v in self.gang_on.items()},
                        "wait_ewma_us": {str(t): v for t, v in self.wait_ewma_us.items()},
                        "gang_switches": self.gang_switches}
        lat = sorted(self.lat_ns) or [0]
        skew = sorted(self.skew_ns) or [0]
        return {"epochs": self.epoch, "transport": self.transport, "sync_p50_us": lat[len(lat) // 2] / 1e3,
                "sync_p99_us": lat[min(len(lat) - 1, int(0.99 * len(lat)))] / 1e3, "sync_max_us": lat[-1] / 1e3,
                "skew_p50_us": skew[len(skew) // 2] / 1e3, "skew_max_us": skew[-1] / 1e3,
                "timeouts": self.timeouts, "degraded": self.degraded, "reforms": self.reforms,
                "members": list(self.members),
                "atc_global_us": self.atc_global_us, "metric_syncs": self.metric_syncs,
                "wait_driven": self.wait_driven, "gang_on": {str(t): v for t, v in self.gang_on.items()},
                "wait_ewma_us": {str(t): v for t, v in self.wait_ewma_us.items()},
                "gang_switches": self.gang_switches}
