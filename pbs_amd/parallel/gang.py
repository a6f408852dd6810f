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
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

FAVOUR, EXCLUDE, NONE = 1, 2, 0
NO_ATC = 1 << 30  # MIN-neutral stand-in for "no ATC pool on this rank"


class GangCoordinator:
    def __init__(self, engine, group, tenants: List[int], epoch_ms: float = 4.0, share: float = 0.5,
                 device: Optional[str] = None, demand: Optional[Callable[[int], bool]] = None,
                 slack_ms: float = 1.0, atc_pool: Optional[int] = None,
                 metric_tenants: Optional[List[int]] = None, metric_every: int = 5):
        self.engine = engine
        self.group = group
        self.tenants = list(tenants)
        self.epoch_ns = int(epoch_ms * 1e6)
        self.share = float(share)
        self.device = device
        self.demand = demand or self._engine_demand
        self.slack_ns = int(slack_ms * 1e6)
        self.epoch = 0
        self.state: Dict[int, int] = {t: NONE for t in self.tenants}
        self.history: List[tuple] = []  # (epoch, {tenant: state}) -- bounded
        self.lat_ns: List[int] = []
        self._want_stop = False
        self._th: Optional[threading.Thread] = None
        self.error: Optional[BaseException] = None
        self.atc_pool = atc_pool
        self.atc_global_us = 0
        self.metric_tenants = list(metric_tenants or [])
        self.metric_every = max(1, int(metric_every))
        self.node_metrics: Dict[int, Dict[str, int]] = {}
        self.metric_syncs = 0

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
    def decide(self, epoch: int, demand_all: List[int]) -> Dict[int, int]:
        """Pure function of (epoch, all-rank demand): identical on every rank."""
        eligible = [t for t, d in zip(self.tenants, demand_all) if d]
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
    def _loop(self):
        dev = torch.device(self.device) if self.device else torch.device("cpu")
        try:
            while True:
                t0 = time.monotonic_ns()
                vec = [1 if self.demand(t) else 0 for t in self.tenants]
                vec += [self._atc_local(), 0 if self._want_stop else 1]
                buf = torch.tensor(vec, dtype=torch.int32, device=dev)
                dist.all_reduce(buf, op=dist.ReduceOp.MIN, group=self.group)
                red = buf.tolist()
                t1 = time.monotonic_ns()
                self.lat_ns.append(t1 - t0)
                if len(self.lat_ns) > 4096:
                    del self.lat_ns[:2048]
                if not red[-1]:
                    break
                if self.atc_pool is not None and 0 < red[-2] < NO_ATC:
                    self.atc_global_us = red[-2]
                    self.engine.atc_sync(self.atc_pool, red[-2])
                if self.metric_tenants and self.epoch % self.metric_every == 0:
                    self._sync_metrics(dev)
                dec = self.decide(self.epoch, red[:-2])
                until = self.engine.now() + self.epoch_ns + self.slack_ns
                for t, st in dec.items():
                    self.engine.gang_set(t, st, until)
                self.state = dec
                self.history.append((self.epoch, dict(dec)))
                if len(self.history) > 8192:
                    del self.history[:4096]
                self.epoch += 1
                rest = self.epoch_ns - (time.monotonic_ns() - t1)
                if rest > 0:
                    time.sleep(rest / 1e9)
        except BaseException as e:  # pragma: no cover - surfaced via .error
            self.error = e
        finally:
            for t in self.tenants:
                try:
                    self.engine.gang_set(t, NONE, 0)
                except Exception:
                    pass

    def _atc_local(self) -> int:
        if self.atc_pool is None:
            return NO_ATC
        try:
            v = self.engine.atc_sync(self.atc_pool, 0)
        except Exception:
            return NO_ATC
        return v if v > 0 else NO_ATC

    def _sync_metrics(self, dev):
        """SUM-reduce the metric tenants' last-period counter deltas."""
        vals = []
        for t in self.metric_tenants:
            try:
                vals += [int(x) for x in self.engine.tenant_info(t).pmc]
            except Exception:
                vals += [0, 0, 0, 0]
        buf = torch.tensor(vals, dtype=torch.int64, device=dev)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
        red = buf.tolist()
        out = {}
        for i, t in enumerate(self.metric_tenants):
            inst, cyc, ref, miss = red[4 * i:4 * i + 4]
            out[t] = {"inst": inst, "cycles": cyc, "l2_refs": ref, "l2_misses": miss,
                      "miss_rate": miss * 100000 // inst if inst else 0}
        self.node_metrics = out
        self.metric_syncs += 1

    def start(self):
        self._th = threading.Thread(target=self._loop, daemon=True, name="gpbs-gang")
        self._th.start()
        return self

    def stop(self, timeout: float = 30.0):
        """Collective: returns once every rank has left the epoch loop."""
        self._want_stop = True
        if self._th is not None:
            self._th.join(timeout)
        if self.error:
            raise self.error

    def stats(self) -> Dict[str, float]:
        lat = sorted(self.lat_ns) or [0]
        return {"epochs": self.epoch, "sync_p50_us": lat[len(lat) // 2] / 1e3, "sync_max_us": lat[-1] / 1e3,
                "atc_global_us": self.atc_global_us, "metric_syncs": self.metric_syncs}
