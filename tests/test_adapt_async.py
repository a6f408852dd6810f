"""Asynchronous device adaptation in the engine (credit.cpp adapt_async).

The GPU backend runs period k's PBS update (k_adapt) while the dispatcher
goes on and the engine applies it at tick k+1 (csrc/hip/runtime.cpp
ctr_adapt_launch / ctr_adapt_harvest); a period whose launch is still
running at the next tick is recomputed on the host.  Here a Python backend
stands in for the device (it computes with the C host adapt_update), on a
simulated clock: the sequence of quanta must be exactly the host engine's,
one metric period late -- also when launches come back late at random and
when the backend refuses to launch.
"""
import ctypes as C
import random

from pbs_amd import _native as N
from pbs_amd.core.config import MI355X_PROFILE
from pbs_amd.core.engine import Engine

PERIOD_US = 1000


def _script(nticks, ntenants, seed):
    """Per tick, per tenant: (inst, miss) -- phases that move the quanta."""
    rng = random.Random(seed)
    out = []
    for k in range(nticks):
        row = []
        for t in range(ntenants):
            phase = ((k // (7 + 3 * t)) + t) % 3
            inst = 0 if rng.random() < 0.05 else 1_000_000 + rng.randrange(20_000)
            miss = inst * (5 if phase == 0 else (40 if phase == 1 else 300)) // 1000
            row.append((inst, miss))
        out.append(row)
    return out


class Backend:
    def __init__(self, engine, script, tids, async_mode=False, late_p=0.0, refuse_p=0.0, seed=0):
        self.e, self.script, self.tids = engine, script, tids
        self.tick = 0
        self.lib = N.load_core()
        self.rng = random.Random(seed)
        self.late_p, self.refuse_p = late_p, refuse_p
        self.pending = {}
        self.stats = {"launch": 0, "late": 0, "refused": 0, "miss": 0}
        self.ops = N.CounterOps()
        self.ops.tenant_deltas = N.COUNTER_TENANT_DELTAS(self._deltas)
        if async_mode:
            self.ops.adapt_launch = N.COUNTER_ADAPT_LAUNCH(self._launch)
            self.ops.adapt_harvest = N.COUNTER_ADAPT_HARVEST(self._harvest)
        engine.set_counter_ops(self.ops)

    def _deltas(self, user, n, ids, out):
        # one script row per metric period, however many pools tick in it
        k = self.e.now() // (PERIOD_US * 1000)
        row = self.script[min(k, len(self.script) - 1)]
        self.tick += 1
        for k in range(n):
            t = ids[k]
            inst, miss = row[self.tids.index(t)] if t in self.tids else (0, 0)
            out[4 * k + 0], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3] = inst, 2 * inst, miss * 4, miss
        return 0

    def _launch(self, user, n, ids, deltas, ssum, scnt, states, params):
        if self.rng.random() < self.refuse_p:
            self.stats["refused"] += 1
            return -11
        res = []
        for k in range(n):
            s = N.AdaptState()
            C.memmove(C.byref(s), C.byref(states[k]), C.sizeof(s))
            p = N.AdaptParams()
            C.memmove(C.byref(p), params, C.sizeof(p))
            self.lib.gpbs_adapt_update(C.byref(s), C.byref(p), deltas[4 * k], deltas[4 * k + 3], ssum[k], scnt[k])
            res.append((ids[k], s))
        self.pending[tuple(ids[k] for k in range(n))] = res  # keyed like the runtime: by the launch's tenants
        self.stats["launch"] += 1
        return 0

    def _harvest(self, user, mx, ids_out, states_out):
        key = tuple(ids_out[k] for k in range(mx))  # in: the caller's launched tenants
        res = self.pending.pop(key, None)
        if res is None:
            self.stats["miss"] += 1
            return -22
        if self.rng.random() < self.late_p:
            self.stats["late"] += 1
            return -11
        for i, (t, s) in enumerate(res[:mx]):
            ids_out[i] = t
            C.memmove(C.byref(states_out[i]), C.byref(s), C.sizeof(s))
        return min(len(res), mx)


def _run(script, async_mode, **kw):
    # the detector alone (grow_pct 0): the class-change seed is an engine
    # event on its own clock, outside the one-period-late relation
    prof = dict(MI355X_PROFILE, quantum_align_us=0, idle_skip=1, metric_period_us=PERIOD_US,
                adapt=dict(MI355X_PROFILE["adapt"], grow_pct=0))
    e = Engine(sim_clock=True, partitions=[(0, x) for x in range(4)], **prof)
    e.tenant_create("Domain-0", nslots=1)
    tids = [e.tenant_create(f"t{i}", nslots=2) for i in range(3)]
    for t in tids:
        e.wake(t)
    be = Backend(e, script, tids, async_mode=async_mode, **kw)
    # align to the first metric tick, then one period per step
    seq = []
    for _ in range(len(script)):
        e.advance(e.now() + PERIOD_US * 1000)
        seq.append(tuple(e.tenant_info(t).tslice_us for t in tids))
    pc = e.perfc()
    return seq, pc, be.stats


def test_async_device_adapt_is_the_host_sequence_one_period_late():
    script = _script(300, 3, seed=5)
    host, pch, _ = _run(script, False)
    dev, pcd, st = _run(script, True)
    assert st["launch"] > 200
    assert len(set(host)) > 3  # the script moves the quanta
    assert dev[1:] == host[:-1]
    assert pcd["adapt_device"] == st["launch"]
    assert pcd["adapt_rearm"] > 0


def test_async_device_adapt_late_and_refused_periods_stay_exact():
    script = _script(300, 3, seed=9)
    host, _, _ = _run(script, False)
    dev, pcd, st = _run(script, True, late_p=0.2, refuse_p=0.1, seed=3)
    assert st["late"] > 10 and st["refused"] > 5
    assert pcd["adapt_late"] == st["late"]
    # a refused launch adapts on the host at once (no lag for that period):
    # compare the state sequence where both paths have caught up
    assert dev[-1] == host[-1] or dev[-1] == host[-2]
    # every lagged tick equals the host one period earlier or the same tick
    ok = sum(1 for k in range(1, len(dev)) if dev[k] in (host[k - 1], host[k]))
    assert ok == len(dev) - 1


def _run_two_pools(script, async_mode):
    """Two credit pools on one counter backend (one GpuContext serving both):
    each pool's metric tick launches and harvests its own tenants only."""
    prof = dict(MI355X_PROFILE, quantum_align_us=0, idle_skip=1, metric_period_us=PERIOD_US,
                adapt=dict(MI355X_PROFILE["adapt"], grow_pct=0))  # the detector alone, as _run
    e = Engine(sim_clock=True, partitions=[(0, x) for x in range(8)], **prof)
    e.tenant_create("Domain-0", nslots=1)
    p1 = e.pool_create("pool1", "credit")
    for part in range(4, 8):
        e.pool_unassign(0, part)
        e.pool_assign(p1, part)
    a = [e.tenant_create(f"a{i}", nslots=2) for i in range(2)]
    b = [e.tenant_create(f"b{i}", nslots=2, pool=p1) for i in range(2)]
    tids = a + b
    for t in tids:
        e.wake(t)
    be = Backend(e, script, tids, async_mode=async_mode)
    seq = []
    for _ in range(len(script)):
        e.advance(e.now() + PERIOD_US * 1000)
        seq.append(tuple(e.tenant_info(t).tslice_us for t in tids))
    return seq, e.perfc(), be.stats


def test_async_adapt_two_pools_never_cross_results():
    """with two PBS pools on one device_adapt context, pool A must
    never apply pool B's launch.  Each pool's quanta are the host engine's
    quanta (an unsynchronised tick interleaving may shift a pool by one
    period, never mix tenants)."""
    script = _script(240, 4, seed=11)
    host, _, _ = _run_two_pools(script, False)
    dev, pcd, st = _run_two_pools(script, True)
    assert st["launch"] > 200
    assert pcd["adapt_device"] == st["launch"]
    assert len(set(host)) > 3
    for k in range(2, len(dev)):
        for j in range(4):
            assert dev[k][j] in (host[k - 1][j], host[k - 2][j], host[k][j]), (k, j)
