"""Credit scheduler semantics on the native engine (simulated clock).

Mirrors the xm-test sched-credit / cpupool / vcpu-pin / pause suites
(X:tools/xm-test/tests/sched-credit/01_sched_credit_weight_cap_pos.py,
tests/cpupool/*, tests/vcpu-pin/*, tests/pause/*) plus the credit mechanics
of X:xen/common/sched_credit.c (acct, boost, park, steal).
"""
import pytest

from pbs_amd.core import oracle as O
from pbs_amd.core.engine import Engine
from pbs_amd.core.errors import GpbsError

MS = 1_000_000


def mk(nparts=4, **kw):
    e = Engine(sim_clock=True, partitions=[(0, x) for x in range(nparts)], **kw)
    e.tenant_create("Domain-0", nslots=1)
    return e


def share(e, ts, dur_ms=200, step_us=50):
    base = {t: e.tenant_info(t).run_ns for t in ts}
    t0 = e.now()
    end = t0 + dur_ms * MS
    while e.now() < end:
        e.advance(e.now() + step_us * 1000)
    return {t: (e.tenant_info(t).run_ns - base[t]) / (end - t0) for t in ts}


def test_defaults_weight_256_cap_0():
    e = mk()
    t = e.tenant_create("a", nslots=2)
    assert e.sched_credit_get(t) == (256, 0)
    e.sched_credit_set(t, weight=512, cap=100)
    assert e.sched_credit_get(t) == (512, 100)


@pytest.mark.parametrize("bad", [dict(weight=0), dict(weight=65536), dict(cap=-5), dict(cap=301)])
def test_weight_cap_validation(bad):
    e = mk()
    t = e.tenant_create("a", nslots=3)
    with pytest.raises(GpbsError):
        e.sched_credit_set(t, **{**dict(weight=-1, cap=-1), **bad})


def test_tslice_ratelimit_validation_and_recompute():
    e = mk()
    assert e.sched_params_get(0) == (100, 100)  # boot default; ratelimit clamped to tslice
    e.sched_params_set(0, 5000, 1000)
    assert e.sched_params_get(0) == (5000, 1000)
    for ts, rl in [(99, 100), (1000001, 1000), (5000, 99), (5000, 500001), (1000, 2000)]:
        with pytest.raises(GpbsError):
            e.sched_params_set(0, ts, rl)
    assert "tslice             = 5000us" in e.debug_keys("r")


def test_proportional_share_by_weight():
    e = mk(nparts=2)
    a = e.tenant_create("a", nslots=2)
    b = e.tenant_create("b", nslots=2, weight=768)
    e.wake(a)
    e.wake(b)
    s = share(e, [a, b], dur_ms=400)
    # 2 partitions, weights 1:3 -> shares 0.5 : 1.5 partitions
    assert abs(s[a] - 0.5) < 0.12 and abs(s[b] - 1.5) < 0.12, s
    assert e.check() == ""


def test_cap_parks_tenant():
    e = mk(nparts=2)
    a = e.tenant_create("capped", nslots=2, cap=50)
    b = e.tenant_create("b", nslots=2)
    e.wake(a)
    e.wake(b)
    s = share(e, [a, b], dur_ms=400)
    assert s[a] < 0.75, s  # at most ~half a partition
    assert e.perfc()["vcpu_park"] > 0 and e.perfc()["vcpu_unpark"] > 0
    assert any(r.event == "PARK" for r in e.trace(from_start=True))


def test_work_conserving_single_tenant_uses_all_partitions():
    e = mk(nparts=4)
    a = e.tenant_create("a", nslots=4)
    e.wake(a)
    s = share(e, [a], dur_ms=50)
    assert s[a] > 3.8


def test_wake_boost_preempts_over_tenant():
    e = mk(nparts=1)
    hog = e.tenant_create("hog", nslots=1)
    lat = e.tenant_create("lat", nslots=1)
    e.wake(hog)
    e.advance(e.now() + 20 * MS)
    lat_delays = []
    for _ in range(20):
        e.advance(e.now() + 3 * MS)
        t0 = e.now()
        e.wake(lat)  # BOOST on wake, tickles the partition
        si = e.slot_info(e.slot_id(lat, 0))
        lat_delays.append(0 if si["is_running"] else 1)
        e.advance(e.now() + 50_000)
        e.block(lat)
    assert sum(lat_delays) <= 4, lat_delays  # boosted wakeups run immediately
    assert e.perfc()["tickle_local_under"] + e.perfc()["tickle_local_over"] > 0


def test_idle_partition_steals_work():
    e = mk(nparts=4)
    a = e.tenant_create("a", nslots=4)
    # home every (blocked) slot on partition 0, then allow all partitions
    for i in range(4):
        e.pin(a, i, [0])
    for i in range(4):
        e.pin(a, i, [0, 1, 2, 3])
    assert all(e.slot_info(e.slot_id(a, i))["processor"] == 0 for i in range(4))
    # wakes queue on the busy partition 0 and tickle idlers, which steal
    for i in range(4):
        e.wake(a, i)
    s = share(e, [a], dur_ms=50)
    assert s[a] > 3.0, s
    assert e.perfc()["migrate_queued"] + e.perfc()["migrate_running"] > 0


def test_pause_unpause_and_destroy():
    e = mk(nparts=2)
    a = e.tenant_create("a", nslots=2)
    b = e.tenant_create("b", nslots=2)
    e.wake(a)
    e.wake(b)
    e.pause(a)
    s = share(e, [a, b], dur_ms=40)
    assert s[a] == 0 and s[b] > 1.9
    e.unpause(a)
    s = share(e, [a, b], dur_ms=200)
    assert s[a] > 0.7
    e.tenant_destroy(b)
    s = share(e, [a], dur_ms=40)
    assert s[a] > 1.9
    assert e.check() == ""
    with pytest.raises(GpbsError):
        e.tenant_info(b) if False else e.sched_credit_get(b)


def test_pools_partition_cpus_and_migrate_tenant():
    e = mk(nparts=4)
    p1 = e.pool_create("Pool-gpu", "credit")
    e.pool_unassign(0, 3)
    e.pool_unassign(0, 2)
    e.pool_assign(p1, 2)
    e.pool_assign(p1, 3)
    assert e.pool_info(0)["cpus"] == [0, 1] and e.pool_info(p1)["cpus"] == [2, 3]
    a = e.tenant_create("a", nslots=2)
    b = e.tenant_create("b", nslots=2, pool=p1)
    e.wake(a)
    e.wake(b)
    e.advance(e.now() + 10 * MS)
    for x in range(4):
        inf = e.partition_info(x)
        assert inf["curr_tenant"] == (a if x < 2 else b)
    e.tenant_move(a, p1)
    e.advance(e.now() + 20 * MS)
    assert e.tenant_info(a).pool == p1
    for x in range(2):
        assert e.partition_info(x)["idle"] == 1
    with pytest.raises(GpbsError):
        e.pool_destroy(p1)  # has tenants
    e.pool_rename(p1, "renamed")
    assert e.pool_find("renamed") == p1
    assert e.check() == ""


def test_unassign_last_cpu_of_busy_pool_rejected():
    e = mk(nparts=2)
    with pytest.raises(GpbsError):
        e.pool_unassign(0, 0) or e.pool_unassign(0, 1)


def test_slot_set_offlines_slots():
    e = mk(nparts=4)
    a = e.tenant_create("a", nslots=4)
    e.wake(a)
    e.set_nslots(a, 2)
    s = share(e, [a], dur_ms=20)
    assert 1.8 < s[a] < 2.2
    e.set_nslots(a, 6)
    e.wake(a)
    s = share(e, [a], dur_ms=20)
    assert s[a] > 3.8


def test_pin_restricts_processor():
    e = mk(nparts=4)
    a = e.tenant_create("a", nslots=2)
    e.pin(a, 0, [3])
    e.pin(a, 1, [3])
    e.wake(a)
    e.advance(e.now() + 20 * MS)
    for i in range(2):
        assert e.slot_info(e.slot_id(a, i))["processor"] == 3


def test_acct_matches_oracle_fair_share():
    """csched_acct fair-share over active domains == oracle (Appendix C)."""
    doms = [O.ODom(id=1, weight=256, slots=[O.OSlot(), O.OSlot()]),
            O.ODom(id=2, weight=512, cap=50, slots=[O.OSlot()]),
            O.ODom(id=3, weight=100, slots=[O.OSlot(credit=-250)])]
    bal, order, parks = O.credit_acct(doms, ncpus=4, cpt=100, balance=0)
    # total credit 400 split by weight*active: 512, 512, 100
    # dom1: fair = ceil(400*256*2/1124) = 183 < peak 200 -> 92 per slot
    assert [s.credit for s in doms[0].slots] == [92, 92]
    # dom2: capped at ceil(50*100/100) = 50; its unused share is redistributed
    assert doms[1].slots[0].credit == 50
    # dom3: -250 + 100 -> -150, floored at -cpt
    assert doms[2].slots[0].credit == -100 and doms[2].slots[0].pri == O.PRI_OVER
    assert bal == 92 + 92 + 50 - 100
    # after a domain leaves credit unused (xtra), capped-out domains are moved to the head
    assert order == [3, 2, 1]


def test_dump_keys_and_dmesg():
    e = mk(nparts=2)
    a = e.tenant_create("a", nslots=1)
    e.wake(a)
    e.advance(e.now() + 5 * MS)
    z = e.debug_keys("z")
    assert "pmuinfo: INST_RETIRED=" in z and "sched_count:" in z and "cpus: 0-1" in z
    q = e.debug_keys("q")
    assert "pmuinfo: pmc[0]=" in q and "VCPU0: CPU" in q
    r = e.debug_keys("r")
    assert "Scheduler: SMP Credit Scheduler (PBS) (credit)" in r and "CPU[00]" in r
    assert "pmuinfo" in e.dmesg()
    assert "sched_ctx" in e.debug_keys("p")


def test_heartbeat_reaps_dead_tenant():
    e = Engine(sim_clock=True, partitions=[(0, x) for x in range(2)], heartbeat_timeout_us=5000)
    e.tenant_create("Domain-0", nslots=1)
    a = e.tenant_create("a", nslots=2)
    b = e.tenant_create("b", nslots=2)
    e.wake(a)
    e.wake(b)
    for _ in range(20):
        e.advance(e.now() + 1 * MS)
        e.heartbeat(b)
    assert e.tenant_info(a).paused == 1 and e.tenant_info(b).paused == 0
    assert e.perfc()["tenant_dead"] == 1
    assert "missed heartbeats" in e.dmesg()


def test_burn_credits_rounding():
    assert O.burn_credits(499) == 0 and O.burn_credits(500) == 1 and O.burn_credits(1_000_000) == 1000


def test_static_scheduler_splits_by_weight():
    e = Engine(sched="static", sim_clock=True, partitions=[(0, x) for x in range(8)])
    a = e.tenant_create("a", nslots=8)
    b = e.tenant_create("b", nslots=8, weight=768)
    e.wake(a)
    e.wake(b)
    s = share(e, [a, b], dur_ms=20)
    assert abs(s[a] - 2.0) < 0.2 and abs(s[b] - 6.0) < 0.2, s
    assert "partitions:" in e.debug_keys("z")


def _running_tenants(e, tenants, nparts):
    on = {}
    for t in tenants:
        for k in range(e.tenant_info(t).nslots):
            si = e.slot_info(e.slot_id(t, k))
            if si["is_running"]:
                on[si["processor"]] = t
    return [on.get(p, -1) for p in range(nparts)]


@pytest.mark.parametrize("cosched", [0, 3])
def test_gang_alignment_of_memory_context(cosched):
    """coschedule=3: the partitions of one (gpu, ctx) class follow the leader's
    tenant, so two bandwidth tenants alternate whole-GPU quanta instead of
    splitting the XCDs; credit shares stay fair either way."""
    n = 8
    e = mk(nparts=n, coschedule=cosched, quantum_align_us=0)
    e.sched_params_set(0, 1000, 0)
    a = e.tenant_create("a", nslots=n)
    b = e.tenant_create("b", nslots=n)
    for k in range(n):  # one slot of each tenant per partition
        e.pin(a, k, [k])
        e.pin(b, k, [k])
    for k in range(n):  # start maximally misaligned
        e.wake(a if k % 2 else b, k)
    e.advance(e.now() + 200_000)
    for k in range(n):
        e.wake(b if k % 2 else a, k)
    aligned = samples = 0
    base = {t: e.tenant_info(t).run_ns for t in (a, b)}
    t0 = e.now()
    while e.now() < t0 + 300 * MS:
        e.advance(e.now() + 100_000)
        cur = _running_tenants(e, [a, b], n)
        samples += 1
        aligned += len(set(cur)) == 1
    frac = aligned / samples
    print("aligned", cosched, frac)
    sh = {t: (e.tenant_info(t).run_ns - base[t]) / (e.now() - t0) for t in (a, b)}
    assert abs(sh[a] - sh[b]) < 0.15 * n, sh
    if cosched >= 3:
        assert frac > 0.9, frac
        assert e.check() == ""
    else:
        assert frac < 0.9, frac  # plain credit leaves the XCDs split


@pytest.mark.parametrize("strict", [0, 1])
def test_ratelimit_hold_does_not_inherit_adaptive_quantum(strict):
    """Q13: sched_credit.c:1732 holds a just-switched-in slot for ratelimit,
    then :1795-1797 (`out:`) overwrite the hold with the tenant's adaptive
    slice, so a BOOSTed waker that tickled it waits a whole PBS quantum.
    gpbs holds for the remaining ratelimit only; strict_ref=1 reproduces."""
    q = 11000
    e = Engine(sim_clock=True, partitions=[(0, 0)], quantum_align_us=0,
               adapt=dict(min_us=q, max_us=q, strict_ref=strict))
    e.tenant_create("Domain-0", nslots=1)
    e.sched_params_set(0, q, 250)
    hog = e.tenant_create("hog", nslots=1)
    lat = e.tenant_create("lat", nslots=1)
    s = e.adapt_state(hog)
    s.tslice_us = q
    e.set_adapt_state(hog, s)
    e.wake(hog)
    e.advance(e.now() + 30 * MS)
    waits = []
    for _ in range(5):
        e.wake(lat)                      # boost-preempts the hog
        e.advance(e.now() + 100_000)
        e.block(lat)                     # hog switches back in ...
        e.advance(e.now() + 20_000)      # ... and 20 us later lat wakes again
        e.wake(lat)
        t0 = e.now()
        while not e.slot_info(e.slot_id(lat, 0))["is_running"] and e.now() - t0 < 20 * MS:
            e.advance(e.now() + 10_000)
        waits.append(e.now() - t0)
        e.block(lat)
        e.advance(e.now() + 3 * MS)
    if strict:
        assert max(waits) > 5 * MS and min(waits) > 1 * MS, waits  # the reference quirk
    else:
        assert max(waits) <= 300_000, waits  # within the ratelimit


def _feed(e, rates, dt_us):
    """Advance the sim clock, charging modeled counters to running slots:
    rates[tenant] = (inst, miss) per us of run time."""
    for t, (ins, miss) in rates.items():
        for k in range(e.tenant_info(t).nslots):
            sid = e.slot_id(t, k)
            si = e.slot_info(sid)
            if si["is_running"]:
                p = list(si["pmc"])
                p[0] += ins * dt_us
                p[1] += dt_us * 2000
                p[2] += miss * dt_us * 4
                p[3] += miss * dt_us
                e.set_pmc(sid, p)
    e.advance(e.now() + dt_us * 1000)


def _procs(e, t):
    return [e.slot_info(e.slot_id(t, k))["processor"] for k in range(e.tenant_info(t).nslots)]


def test_contention_classes_are_soft_affinity_and_work_conserving():
    """coschedule=2: counter rates classify tenants (compute -> context 0,
    memory -> context 1), slots spread one per partition of their class; the
    class is soft: an idle compute context steals waiting memory slots, and
    they go home once the compute tenant is back."""
    parts = [(0, x, c) for x in range(4) for c in range(2)]
    e = Engine(sim_clock=True, partitions=parts, coschedule=2, class_period_us=2000, quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    comp = e.tenant_create("gemm", nslots=4)
    mem = e.tenant_create("hbm", nslots=8)
    rates = {comp: (1000, 1), mem: (100, 100)}
    e.wake(comp)
    e.wake(mem)
    for _ in range(300):  # 30 ms
        _feed(e, rates, 100)
    ctx = {p: c for p, (_, _, c) in enumerate(parts)}
    assert all(ctx[p] == 0 for p in _procs(e, comp)), _procs(e, comp)
    home = _procs(e, mem)
    assert sorted(home) == sorted([p for p in ctx if ctx[p] == 1] * 2), home  # two per memory partition
    # compute tenant goes idle: its partitions steal waiting memory slots
    e.block(comp)
    base = e.tenant_info(mem).run_ns
    t0 = e.now()
    for _ in range(100):
        _feed(e, rates, 100)
    share = (e.tenant_info(mem).run_ns - base) / (e.now() - t0)
    assert share > 6.0, share
    # compute tenant returns: it gets its context back, strays go home
    e.wake(comp)
    for _ in range(100):
        _feed(e, rates, 100)
    base_c, t0 = e.tenant_info(comp).run_ns, e.now()
    for _ in range(100):
        _feed(e, rates, 100)
    assert (e.tenant_info(comp).run_ns - base_c) / (e.now() - t0) > 3.5
    for k in range(8):
        si = e.slot_info(e.slot_id(mem, k))
        if not si["is_running"]:
            assert ctx[si["processor"]] == 1, (k, si["processor"])
    assert e.check() == ""


def test_atc_places_slots_least_loaded_and_apart():
    """sched_credit_atc.c:634-651 + :545-570: new slots go to the least-loaded
    partition not used by a sibling; siblings are pinned away from each other."""
    e = mk(nparts=4, sched="atc")
    busy = e.tenant_create("busy", nslots=4)
    for k in range(4):
        e.pin(busy, k, [0] if k < 3 else [1])   # queue load on partitions 0 and 1
    e.wake(busy)
    t = e.tenant_create("t", nslots=2)
    procs = [e.slot_info(e.slot_id(t, k))["processor"] for k in range(2)]
    assert len(set(procs)) == 2 and set(procs) <= {2, 3}, procs
    for k in range(2):
        sid = e.slot_id(t, k)
        aff = __import__("pbs_amd.utils.snapshot", fromlist=["slot_affinity"]).slot_affinity(e, sid)
        other = procs[1 - k]
        assert other not in aff and procs[k] in aff, (k, aff)
    assert e.check() == ""


def test_class_placement_is_not_undone_by_cross_class_steals():
    """Regression: sending a running slot to its class home briefly idles the
    partition it left, which used to steal it straight back (a cascade that
    left both tenants spread over both halves of every XCD)."""
    parts = [(0, x, c) for x in range(8) for c in range(2)]
    e = Engine(sim_clock=True, partitions=parts, coschedule=3, class_period_us=2000, quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    mem = e.tenant_create("infer", nslots=8)
    comp = e.tenant_create("train", nslots=8)
    e.wake(mem)
    e.wake(comp)
    for _ in range(300):
        _feed(e, {mem: (100, 100), comp: (1000, 1)}, 100)
    assert sorted(_procs(e, mem)) == list(range(1, 16, 2)), _procs(e, mem)
    assert sorted(_procs(e, comp)) == list(range(0, 16, 2)), _procs(e, comp)
    assert e.check() == ""


def test_four_contexts_memory_tenants_coreside_on_distinct_contexts():
    """nctx=4: the compute class keeps context 0, the memory class spans
    contexts 1-3 and its tenants start on different contexts, so three memory
    tenants and a compute tenant all co-reside on every XCD instead of
    time-sharing one memory context.  Regression: an in-class steal used to
    leave a tenant stacked on one XCD for good in a fully busy pool."""
    parts = [(0, x, c) for x in range(8) for c in range(4)]
    e = Engine(sim_clock=True, partitions=parts, coschedule=3, class_period_us=2000, quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    comp = e.tenant_create("gemm", nslots=8)
    mems = [e.tenant_create(n, nslots=8) for n in ("hbm", "coll", "kv")]
    rates = {comp: (1000, 1), **{m: (100, 100) for m in mems}}
    for t in (comp, *mems):
        e.wake(t)
    for _ in range(400):
        _feed(e, rates, 100)
    ctx = {p: c for p, (_, _, c) in enumerate(parts)}
    xcd = {p: x for p, (_, x, _) in enumerate(parts)}
    assert sorted(ctx[p] for p in _procs(e, comp)) == [0] * 8
    for m in mems:
        procs = _procs(e, m)
        assert sorted(xcd[p] for p in procs) == list(range(8)), (m, procs)  # one slot per XCD
        assert all(ctx[p] >= 1 for p in procs), (m, procs)
    # every throughput tenant keeps running: no time-sharing of contexts
    base = {t: e.tenant_info(t).run_ns for t in (comp, *mems)}
    t0 = e.now()
    for _ in range(100):
        _feed(e, rates, 100)
    for t in (comp, *mems):
        assert (e.tenant_info(t).run_ns - base[t]) / (e.now() - t0) > 7.5, t
    assert e.check() == ""


def _boost_run(exclusive):
    parts = [(0, x, c) for x in range(2) for c in range(4)]
    e = Engine(sim_clock=True, partitions=parts, coschedule=3, class_period_us=2000, quantum_align_us=0,
               boost_exclusive=exclusive)
    e.tenant_create("Domain-0", nslots=1)
    comp = e.tenant_create("gemm", nslots=2)
    mems = [e.tenant_create(n, nslots=2) for n in ("hbm", "coll")]
    lat = e.tenant_create("lat", nslots=2)
    rates = {comp: (1000, 1), **{m: (100, 100) for m in mems}, lat: (100, 100)}
    for t in (comp, *mems):
        e.wake(t)
    for _ in range(200):  # classify and settle
        _feed(e, rates, 100)
    base = {t: e.tenant_info(t).run_ns for t in (comp, *mems)}
    e.perfc_reset()
    overlap = 0  # 100-us steps in which the request and a memory tenant both ran on one XCD
    for _ in range(20):  # requests: 300 us of work, 1.7 ms think time
        e.wake(lat)
        for _ in range(3):
            _feed(e, rates, 100)
            on = {(parts[p][1]) for p in _procs(e, lat) if e.slot_info(e.slot_id(lat, _procs(e, lat).index(p)))["is_running"]}
            for m in mems:
                for k in range(2):
                    si = e.slot_info(e.slot_id(m, k))
                    if si["is_running"] and parts[si["processor"]][1] in on:
                        overlap += 1
        e.block(lat)
        for _ in range(17):
            _feed(e, rates, 100)
    run = {t: e.tenant_info(t).run_ns - base[t] for t in (comp, *mems)}
    return e, overlap, run, comp, mems


def test_boost_exclusive_parks_memory_siblings_during_a_request():
    """boost_exclusive=1: while the latency tenant's BOOSTed request runs on
    an XCD, memory-class tenants on the sibling contexts park (and resume
    when it blocks); the compute tenant keeps running.  Off: they co-run."""
    e0, ov0, run0, comp, mems = _boost_run(0)
    e1, ov1, run1, _, _ = _boost_run(1)
    assert ov0 > 0 and e0.perfc().get("boost_park", 0) == 0
    assert ov1 == 0, ov1
    assert e1.perfc()["boost_park"] > 0
    # compute tenant unaffected, memory tenants lose at most the request time (~15 %)
    assert run1[comp] >= 0.97 * run0[comp], (run0, run1)
    for m in mems:
        assert run1[m] >= 0.8 * run0[m], (m, run0, run1)
    assert e1.check() == ""


def _two_class_engine(sched):
    from pbs_amd.core.config import MI355X_PROFILE
    prof = dict(MI355X_PROFILE)
    prof["sched"] = sched
    e = Engine(sim_clock=True, partitions=[(0, 0), (0, 1)], **prof)
    e.tenant_create("Domain-0", nslots=1)
    a = e.tenant_create("mem", nslots=1)
    b = e.tenant_create("cmp", nslots=1)
    e.wake(a)
    e.wake(b)
    return e, a, b


def _feed_classes(e, a, b, periods, k0=1):
    for k in range(k0, k0 + periods):  # mem: 5e4 misses / 1e5 inst; cmp: 10 / 1e5
        e.set_pmc(e.slot_id(a, 0), [k * 1_000_000, k * 1_000_000, k * 1000, k * 500_000])
        e.set_pmc(e.slot_id(b, 0), [k * 1_000_000, k * 1_000_000, k * 1000, k * 100])
        e.advance(e.now() + 1_000_000)


def test_credit_classq_maps_class_to_bound_without_detector():
    """credit-classq (VERDICT r4 item 3 ablation): the memory-class tenant runs
    with max_us and the compute-class one with min_us as soon as classified,
    with no PBS detector activity (no adapt inc / dec / re-arm)."""
    e, a, b = _two_class_engine("credit-classq")
    _feed_classes(e, a, b, 60)
    assert e.lib.gpbs_tenant_class(e.h, a) == 1 and e.lib.gpbs_tenant_class(e.h, b) == 0
    assert e.tenant_info(a).tslice_us == 11000 and e.tenant_info(b).tslice_us == 1000
    pc = e.perfc()
    assert pc["adapt_inc"] == 0 and pc["adapt_dec"] == 0 and pc["adapt_rearm"] == 0
    ba, bb = e.bound_stats(a), e.bound_stats(b)
    assert ba["periods"] == 60 and bb["at_min"] == 60
    assert ba["at_max"] >= 50  # at max from its classification on


def test_bound_stats_count_pbs_quantum_at_the_bounds_and_reset():
    """PBS mode: a steady memory-bound tenant's quantum climbs to max_us and
    stays; bound_stats counts the measured periods at each bound and resets."""
    e, a, b = _two_class_engine("credit")
    _feed_classes(e, a, b, 40)
    assert e.tenant_info(a).tslice_us == 11000 and e.tenant_info(b).tslice_us == 1000
    st = e.bound_stats(a, reset=True)
    assert st["periods"] == 40 and 0 < st["at_max"] < 40 and st["at_min"] <= 5  # from the initial quantum
    _feed_classes(e, a, b, 10, k0=41)
    assert e.bound_stats(a) == {"periods": 10, "at_min": 0, "at_max": 10}


def test_runtime_section_of_gpbs_toml(tmp_path):
    """gpbs.toml [runtime] carries the GPU runtime's sampler parameters
    (the round-4 GPBS_HWC_* environment knobs); unknown keys are refused."""
    from pbs_amd.core import config as cfgmod
    p = tmp_path / "gpbs.toml"
    p.write_text("[boot]\ntslice_us = 2000\n[runtime]\nbudget_pct = 8\nguard_us = 200\nalign = 1\n")
    cfg = cfgmod.load(str(p), cfgmod.MI355X_PROFILE)
    assert cfg["boot"]["tslice_us"] == 2000
    assert cfg["runtime"] == {"budget_pct": 8, "guard_us": 200, "align": 1}
    assert set(cfg["runtime"]) <= set(cfgmod.RUNTIME_KEYS)
    p.write_text("[runtime]\nowner_burst = 1\n")
    with pytest.raises(ValueError):
        cfgmod.load(str(p))
    assert cfgmod.load(None)["runtime"] == {}


def test_measurement_tenure_extends_one_tenure_once():
    """The counter sampler's measurement tenure (gpbs_tenant_measure): the
    next tenure of the tenant that starts after the request runs at least the
    requested length -- once -- and later tenures return to its quantum."""
    from pbs_amd.core.config import MI355X_PROFILE
    prof = dict(MI355X_PROFILE)
    prof["sched"] = "credit"
    e = Engine(sim_clock=True, partitions=[(0, 0)], **prof)
    a = e.tenant_create("mem", nslots=1)
    b = e.tenant_create("cmp", nslots=1)
    e.wake(a)
    e.wake(b)
    _feed_classes(e, a, b, 30)
    assert e.tenant_info(b).tslice_us == 1000
    e.trace(from_start=True)  # move the cursor past the history
    assert e.measure(b) == 0
    assert e.measure(b, 4500) == 0
    _feed_classes(e, a, b, 40, k0=31)
    sw = [r for r in e.trace() if r.event == "SWITCH" and r.a[1] == b]
    assert sw, "no tenure of the tenant"
    assert sw[0].a[2] >= 4500  # the first tenure after the request
    assert all(r.a[2] < 4500 for r in sw[1:])
    assert e.measure(b) == 1


def test_class_change_seeds_the_detector_at_the_class_bound():
    """PBS with grow_pct (MI355X profile): a confirmed class change restarts
    the detector from the new class's bound -- a tenant turning memory-bound
    runs max_us at once instead of climbing from min_us -- while the
    reference detector (grow_pct 0) climbs step by step."""
    from pbs_amd.core.config import MI355X_PROFILE
    out = {}
    for g in (100, 0):
        prof = dict(MI355X_PROFILE)
        prof["sched"] = "credit"
        prof["adapt"] = dict(MI355X_PROFILE["adapt"], grow_pct=g)
        e = Engine(sim_clock=True, partitions=[(0, 0), (0, 1)], **prof)
        e.tenant_create("Domain-0", nslots=1)
        a = e.tenant_create("phase", nslots=1)
        b = e.tenant_create("cmp", nslots=1)
        e.wake(a)
        e.wake(b)
        for k in range(1, 41):  # both compute-bound: a settles at min_us
            e.set_pmc(e.slot_id(a, 0), [k * 1_000_000, k * 1_000_000, k * 1000, k * 100])
            e.set_pmc(e.slot_id(b, 0), [k * 1_000_000, k * 1_000_000, k * 1000, k * 100])
            e.advance(e.now() + 1_000_000)
        assert e.lib.gpbs_tenant_class(e.h, a) == 0 and e.tenant_info(a).tslice_us == 1000
        seen = []
        m0 = 40 * 100
        for k in range(41, 61):  # a turns memory-bound (5e4 misses / 1e5 inst)
            e.set_pmc(e.slot_id(a, 0), [k * 1_000_000, k * 1_000_000, k * 1000, m0 + (k - 40) * 500_000])
            e.set_pmc(e.slot_id(b, 0), [k * 1_000_000, k * 1_000_000, k * 1000, k * 100])
            e.advance(e.now() + 1_000_000)
            seen.append((e.lib.gpbs_tenant_class(e.h, a), e.tenant_info(a).tslice_us))
        out[g] = seen
    first = next(i for i, (c, _) in enumerate(out[100]) if c == 1)
    assert out[100][first][1] == 11000  # seeded at the class change
    assert all(q == 11000 for _, q in out[100][first:])
    assert out[0][first][1] < 11000  # the reference detector is still climbing
