"""Demand-driven SE budgets (class_budget, simulated clock).

Every PRESENT classified tenant gets a set of shader engines of every XCD,
sized from the classes present (csrc/core/engine.cpp budget_layout); surplus
slots go offline.  The layout follows phase changes (a tenant whose counters
turn memory-bound) and tenants that stop and start, which a hand-picked
static SE split cannot (bench.py --mix phase measures that on MI355X).
"""
from collections import Counter

import pytest

from pbs_amd.core.config import MI355X_PROFILE
from pbs_amd.core.engine import Engine

from test_engine_credit import _feed

COMPUTE, MEMORY = (1000, 1), (100, 100)  # (inst, miss) per us: rate 100 vs 1e5 per 100k inst


def _engine(**over):
    parts = [(0, x, c) for x in range(8) for c in range(4)]
    prof = dict(MI355X_PROFILE)
    # mem_split 0: these tests pin the time-shared memory region (round 5's
    # layout, still the compute region's); test_crowded_memory_region_* below
    # covers the split
    prof.update(class_split=2, idle_skip=1, quantum_align_us=0, class_budget=1, present_us=5000, mem_split=0)
    prof.update(over)
    e = Engine(sim_clock=True, partitions=parts, **prof)
    e.tenant_create("Domain-0", nslots=1)
    return e, parts


def _ctx_owners(e, parts):
    """ctx -> Counter(tenant running there) over the 8 XCDs."""
    out = {c: Counter() for c in range(4)}
    for p, (_, _, c) in enumerate(parts):
        out[c][e.partition_info(p)["curr_tenant"]] += 1
    return out


def _online(e, t):
    return e.tenant_info(t).online_slots


def _settle(e, rates, steps=400):
    for _ in range(steps):
        _feed(e, rates, 100)


def test_budget_4mix_one_memory_se_each():
    e, parts = _engine()
    g, h, r = (e.tenant_create(n, nslots=32) for n in ("gemm", "hbm", "coll"))
    rates = {g: COMPUTE, h: MEMORY, r: MEMORY}
    for t in rates:
        e.wake(t)
    _settle(e, rates)
    own = _ctx_owners(e, parts)
    assert own[0][g] == 8 and own[1][g] == 8, own
    assert own[2][h] == 8 and own[3][r] == 8, own
    assert (_online(e, g), _online(e, h), _online(e, r)) == (16, 8, 8)
    assert e.perfc()["relayout"] >= 1
    assert e.check() == ""


def test_budget_follows_phase_change_and_a_stopped_tenant():
    e, parts = _engine()
    g, p, s = (e.tenant_create(n, nslots=32) for n in ("gemm", "phase", "hbm"))
    rates = {g: COMPUTE, p: COMPUTE, s: MEMORY}
    for t in rates:
        e.wake(t)
    _settle(e, rates)
    own = _ctx_owners(e, parts)
    # two compute tenants share the compute half one SE each; the lone memory
    # tenant takes both memory SEs
    assert own[0][g] == 8 and own[1][p] == 8 and own[2][s] == 8 and own[3][s] == 8, own
    # the phase tenant turns memory-bound: it moves to a memory SE, the GEMM
    # gets the whole compute half
    rates[p] = MEMORY
    rearm0 = e.perfc()["adapt_rearm"]
    _settle(e, rates)
    own = _ctx_owners(e, parts)
    assert own[0][g] == 8 and own[1][g] == 8, own
    assert {own[2].most_common(1)[0][0], own[3].most_common(1)[0][0]} == {p, s}, own
    assert e.perfc()["adapt_rearm"] > rearm0  # the PBS window re-armed on the phase change
    # the stream tenant stops: after present_us the phase tenant holds both memory SEs
    e.block(s)
    rates.pop(s)
    _settle(e, rates)
    own = _ctx_owners(e, parts)
    assert own[2][p] == 8 and own[3][p] == 8, own
    # ... and with the phase tenant compute-bound again and the stream still
    # gone, the two GEMMs split the GPU two SEs each
    rates[p] = COMPUTE
    _settle(e, rates, 600)
    own = _ctx_owners(e, parts)
    assert sorted([own[0][g] + own[1][g], own[2][p] + own[3][p]]) == [16, 16] or \
        sorted([own[0][p] + own[1][p], own[2][g] + own[3][g]]) == [16, 16], own
    # the stream comes back: it is re-placed on the memory half
    e.wake(s)
    rates[s] = MEMORY
    _settle(e, rates)
    own = _ctx_owners(e, parts)
    assert own[2][s] == 8 and own[3][s] == 8, own
    assert e.check() == ""


def test_budget_time_shares_a_crowded_class_region():
    e, parts = _engine(shared_q_us=0)  # PBS region quanta: shares even out within the 200 ms window
    g = e.tenant_create("gemm", nslots=32)
    mem = [e.tenant_create(f"m{i}", nslots=32) for i in range(3)]
    rates = {g: COMPUTE, **{m: MEMORY for m in mem}}
    for t in rates:
        e.wake(t)
    _settle(e, rates)
    assert [_online(e, m) for m in mem] == [16, 16, 16]
    assert _online(e, g) == 16
    base = {t: e.tenant_info(t).run_ns for t in rates}
    t0 = e.now()
    _settle(e, rates, 1500)
    dt = e.now() - t0
    share = {t: (e.tenant_info(t).run_ns - base[t]) / dt for t in rates}
    assert share[g] > 15.5, share
    ms = [share[m] for m in mem]
    assert sum(ms) > 15.0 and max(ms) - min(ms) < 2.5, share
    assert e.check() == ""


def test_probe_layout_gives_unclassified_tenants_exclusive_partitions():
    """Seven busy tenants, none classified yet: each gets whole XCDs of its
    own (a time-shared tenant would never see a clean counter window, and an
    XCD shared with a stream would charge it the stream's L2 misses); once
    every tenant has a class the class layout takes over (crowded regions
    time-share)."""
    e, parts = _engine()
    names = ["g0", "g1", "g2", "m0", "m1", "m2", "m3"]
    ts = [e.tenant_create(n, nslots=32) for n in names]
    rates = {t: (COMPUTE if n.startswith("g") else MEMORY) for t, n in zip(ts, names)}
    for t in ts:
        e.wake(t)
    for _ in range(60):  # the first class ticks: probe layout
        _feed(e, {}, 100)
    owners = [e.partition_info(p)["curr_tenant"] for p in range(len(parts))]
    per = Counter(o for o in owners if o in ts)
    assert sorted(per.values()) == [4, 4, 4, 4, 4, 4, 8], per  # 8 XCDs dealt to 7 tenants, all 4 SEs each
    for t in ts:
        xs = {parts[p][1] for p in range(len(parts)) if owners[p] == t}
        assert all(owners[x * 4 + c] == t for x in xs for c in range(4)), (t, xs)
    assert sum(_online(e, t) for t in ts) == 32
    assert e.perfc()["probe_layout"] >= 1
    _settle(e, rates, 600)
    classes = {n: e.lib.gpbs_tenant_class(e.h, t) for n, t in zip(names, ts)}
    assert all(c == (0 if n.startswith("g") else 1) for n, c in classes.items()), classes
    own = _ctx_owners(e, parts)
    comp = {t for t, n in zip(ts, names) if n.startswith("g")}
    assert all(t in comp for c in (0, 1) for t in own[c] if t >= 0), own
    assert all(t not in comp for c in (2, 3) for t in own[c] if t >= 0), own
    assert e.check() == ""


def test_crowded_regions_split_by_xcd_blocks_with_class_budget_2():
    """class_budget = 2: a class region with more tenants than SEs is split
    by blocks of whole XCDs (3 GEMMs on SEs {0,1}: 3+3+2 XCDs; 4 streams on
    SEs {2,3}: 2 XCDs each) -- nothing is time-shared."""
    e, parts = _engine(class_budget=2)
    gs = [e.tenant_create(f"g{i}", nslots=32) for i in range(3)]
    ms = [e.tenant_create(f"m{i}", nslots=32) for i in range(4)]
    rates = {**{t: COMPUTE for t in gs}, **{t: MEMORY for t in ms}}
    for t in rates:
        e.wake(t)
    _settle(e, rates, 800)
    owners = {p: e.partition_info(p)["curr_tenant"] for p in range(len(parts))}
    for p, (_, x, c) in enumerate(parts):
        assert owners[p] in (gs if c < 2 else ms), (p, owners[p])
    xcds = {t: sorted({parts[p][1] for p in owners if owners[p] == t}) for t in rates}
    assert sorted(len(xcds[t]) for t in gs) == [2, 3, 3], xcds
    assert all(len(xcds[t]) == 2 for t in ms), xcds
    assert sorted(_online(e, t) for t in gs) == [4, 6, 6]
    # every tenant runs all the time on its own partitions
    base = {t: e.tenant_info(t).run_ns for t in rates}
    t0 = e.now()
    _settle(e, rates, 300)
    dt = e.now() - t0
    for t in rates:
        share = (e.tenant_info(t).run_ns - base[t]) / dt
        assert abs(share - _online(e, t)) < 0.2, (t, share, _online(e, t))
    assert e.check() == ""


def test_time_shared_region_runs_per_tenant_quanta_fairly():
    """A time-shared class region (class_budget 1) dispatches every co-sharer
    with its OWN quantum (no region-wide override), and the
    region's virtual time keeps the shares equal whatever the quanta: a
    co-sharer whose counters stop (no clean window on the hardware -- the PBS
    idle-sample rule skips its periods and its quantum stays at the 1 ms
    floor) runs 1 ms turns next to partners at 11 ms, and still gets its
    quarter of the region, in more, shorter turns (csrc/core/credit.cpp
    quantum_us / region_pick; the 8mix shape: 3 GEMMs + 4 memory tenants of 8
    slots each)."""
    e, parts = _engine(present_us=10000)
    gs = [e.tenant_create(f"g{i}", nslots=8) for i in range(3)]
    ms = [e.tenant_create(f"m{i}", nslots=8) for i in range(4)]
    rates = {**{t: COMPUTE for t in gs}, **{t: MEMORY for t in ms}}
    for t in rates:
        e.wake(t)
    _settle(e, rates, 800)
    assert all(e.tenant_info(m).tslice_us > 5000 for m in ms)
    st = e.adapt_state(ms[3])
    st.tslice_us, st.tick_period_us = 1000, 333
    e.set_adapt_state(ms[3], st)
    rates[ms[3]] = (0, 0)  # its counters stop
    base = {t: e.tenant_info(t).run_ns for t in rates}
    t0 = e.now()
    e.trace(from_start=True)
    _settle(e, rates, 3200)
    dt = e.now() - t0
    share = {t: (e.tenant_info(t).run_ns - base[t]) / dt for t in rates}
    info = {m: e.tenant_info(m) for m in ms}
    assert info[ms[3]].tslice_us == 1000 and info[ms[3]].target_tslice_us == 1000  # its own quantum
    assert all(info[m].tslice_us > 5000 for m in ms[:3])  # ... next to its partners' 11 ms
    recs = e.trace()
    q = {m: [r.a[2] for r in recs if r.event == "SWITCH" and r.a[1] == m] for m in ms}
    assert q[ms[3]] and max(q[ms[3]]) == 1000 and min(min(q[m]) for m in ms[:3]) > 5000, q
    assert len(q[ms[3]]) > 2 * len(q[ms[0]]), {m: len(v) for m, v in q.items()}  # more, shorter turns
    mem = [share[m] for m in ms]
    assert min(mem) > 3.5 and max(mem) - min(mem) < 0.7, share
    assert e.check() == ""


def test_time_shared_region_steals_no_stacking_siblings():
    """8mix shape (3 compute + 4 memory tenants, 16 slots each online): every
    tenant of a time-shared class region has a home slot on every partition
    of it, so an in-class steal onto a partition that already holds the
    tenant's sibling only stacks it (and the class tick undoes it: sleep +
    migrate + wake, a runner revocation each).  Round-4 MI355X traces of the
    slow 8mix mode showed ~1900 such steals per GEMM tenant per 1.6 s run.
    The default skips them (perfc steal_sibling_skip) without changing the
    shares; sibling_steal=1 restores the Xen behaviour."""
    out = {}
    for ss in (1, 0):
        # the reference's additive quantum steps: the steal pattern this
        # guards against was traced with them (round 4)
        # (region_vt 0: credit orders the region, the setting the guard was made for)
        e, parts = _engine(sibling_steal=ss, adapt=dict(MI355X_PROFILE["adapt"], grow_pct=0), shared_q_us=0,
                           region_vt=0, region_q=1)
        ws = (512, 256, 256, 256, 256, 256, 256)  # a heavier tenant keeps UNDER slots queued on busy peers
        ts = [e.tenant_create(f"t{i}", nslots=32, weight=w) for i, w in enumerate(ws)]
        rates = {t: (COMPUTE if i < 3 else MEMORY) for i, t in enumerate(ts)}
        for t in ts:
            e.wake(t)
        _settle(e, rates, 300)
        e.perfc_reset()
        r0 = {t: e.tenant_info(t).run_ns for t in ts}
        _settle(e, rates, 2000)
        pc = e.perfc()
        share = [(e.tenant_info(t).run_ns - r0[t]) / 200e6 for t in ts]
        out[ss] = (pc["migrate_queued"], pc["steal_sibling_skip"], pc["vcpu_sleep"], share)
        assert e.check() == ""
    assert out[1][0] > 20 and out[1][1] == 0, out  # Xen semantics: stacking steals happen
    assert out[0][0] == 0 and out[0][1] > 0 and out[0][2] == 0, out  # guarded: none, no send-home churn
    for a, b in zip(out[0][3][:3], out[1][3][:3]):  # the compute region's shares unchanged (partitions' worth);
        assert abs(a - b) < 0.3, out                # the memory tenants' 11 ms quanta are too coarse for 200 ms
    assert out[0][3][0] > max(out[0][3][1:3]) + 1.0, out  # the weight still counts


def test_class_steal_off_keeps_a_short_gap_in_its_class():
    """boot class_steal=0: while the compute tenant pauses for 3 ms (less than
    present_us, so the layout stays), slots waiting in the time-shared memory
    region do not steal the idle compute partitions (on a GPU every such
    steal moves a runner onto an unmasked queue next to the returning owner --
    config #5's decode p99).  class_steal=1 keeps Xen's cross-class work
    conservation (load_balance's second step)."""
    out = {}
    for cs in (1, 0):
        e, parts = _engine(class_steal=cs)
        # three memory tenants time-share the two memory SEs: slots wait there
        g, h, r, h2 = (e.tenant_create(n, nslots=32) for n in ("gemm", "hbm", "coll", "hbm_b"))
        rates = {g: COMPUTE, h: MEMORY, r: MEMORY, h2: MEMORY}
        for t in rates:
            e.wake(t)
        _settle(e, rates)
        mig0 = e.perfc()["migrate_queued"]
        e.block(g)
        on_compute = 0
        for i in range(30):  # 3 ms; the all-reduce's runner drains and refills every ms (wakes tickle idlers)
            if i % 10 == 5:
                e.block(r)
            elif i % 10 == 6:
                e.wake(r)
            _feed(e, {h: MEMORY, r: MEMORY, h2: MEMORY}, 100)
            own = _ctx_owners(e, parts)
            on_compute = max(on_compute, sum(own[c][t] for c in (0, 1) for t in (h, r, h2)))
        e.wake(g)
        _settle(e, rates, 100)
        out[cs] = (on_compute, e.perfc()["migrate_queued"] - mig0, _online(e, g))
        assert e.check() == ""
    assert out[1][0] > 0 and out[1][1] > 0, out  # Xen semantics: the idle compute SEs run memory slots
    assert out[0][0] == 0 and out[0][2] == 16, out  # guarded: the gap stays a gap, the layout unchanged


def test_two_tenant_probe_gives_class_halves():
    """A newcomer next to one classified tenant (config #5: the trainer
    arriving next to the decode server): while it is probed, the incumbent
    keeps its class's half of every XCD and the newcomer takes the other
    half -- clean halves, so shim tenants launch on masked queues instead of
    running unmasked over each other until the newcomer is classified."""
    e, parts = _engine()
    h = e.tenant_create("decode", nslots=32)
    e.wake(h)
    _settle(e, {h: MEMORY}, 200)
    assert e.lib.gpbs_tenant_class(e.h, h) == 1
    g = e.tenant_create("trainer", nslots=32)
    e.wake(g)
    for _ in range(50):  # 5 ms of relayout ticks; the newcomer reports no counters yet: unclassified
        _feed(e, {h: MEMORY}, 100)
    assert e.lib.gpbs_tenant_class(e.h, g) < 0
    own = _ctx_owners(e, parts)
    assert own[0][g] == 8 and own[1][g] == 8, own  # newcomer: the compute half
    assert own[2][h] == 8 and own[3][h] == 8, own  # incumbent memory tenant: its half
    assert e.perfc()["probe_layout"] >= 1
    _settle(e, {h: MEMORY, g: COMPUTE}, 300)  # classified: the class layout is the same split
    own = _ctx_owners(e, parts)
    assert own[0][g] == 8 and own[1][g] == 8 and own[2][h] == 8 and own[3][h] == 8, own
    assert e.check() == ""


def test_class_fall_reclassifies_an_ended_memory_phase_sooner():
    """boot class_fall=1: the classifier's smoothed miss rate follows a drop
    at alpha 1/2, so a phase tenant whose memory-bound phase ends is back in
    the compute class in fewer metric periods (a rise already crosses the
    threshold in one sample either way)."""
    took = {}
    for cf in (0, 1):
        e, parts = _engine(class_fall=cf)
        g, p, s = (e.tenant_create(n, nslots=32) for n in ("gemm", "phase", "hbm"))
        rates = {g: COMPUTE, p: MEMORY, s: MEMORY}
        for t in rates:
            e.wake(t)
        _settle(e, rates)
        assert e.lib.gpbs_tenant_class(e.h, p) == 1
        rates[p] = COMPUTE
        n = 0
        while e.lib.gpbs_tenant_class(e.h, p) != 0 and n < 2000:
            _feed(e, rates, 100)
            n += 1
        took[cf] = n
        assert e.check() == ""
    assert took[1] < 2000 and took[1] < took[0], took


def test_flapping_tenant_is_laid_out_in_the_memory_region():
    """class_pin_us: a tenant whose last three class changes fall within the
    window is laid out as memory class when the memory region is already
    time-shared (two or more other memory tenants: phase-ts) -- it joins
    that region instead of taking compute SEs from the GEMM tenant on every
    compute phase (s23/s24: the move halved the GEMM's SEs for no gain to
    the phase tenant).  Its first changes still move it (the live
    phase-change test needs that); next to a single memory tenant (the phase
    mix) it keeps moving, and without the pin it always does."""
    def run(pin_us, n_mem):
        # (the round-5 region dispatch the pin was measured with: one region
        # quantum, credit order)
        e, parts = _engine(class_pin_us=pin_us, region_q=1, region_vt=0)
        g, p = (e.tenant_create(n, nslots=32) for n in ("gemm", "phase"))
        ms = [e.tenant_create(f"m{i}", nslots=32) for i in range(n_mem)]
        rates = {g: COMPUTE, p: COMPUTE}
        rates.update({m: MEMORY for m in ms})
        for t in rates:
            e.wake(t)
        _settle(e, rates, 600)
        seen = []
        for k in range(8):  # 8 phases of 60 ms: memory, compute, memory, ...
            rates[p] = MEMORY if k % 2 == 0 else COMPUTE
            _settle(e, rates, 600)
            seen.append((e.lib.gpbs_tenant_class(e.h, p), e.tenant_info(p).budget_ctx & 0xF,
                         e.tenant_info(g).budget_ctx & 0xF))
        assert e.check() == ""
        return seen
    free = run(0, 3)
    pinned = run(2_000_000, 3)
    single = run(2_000_000, 1)
    # without the pin, every compute phase takes a compute SE from the GEMM
    assert all(c == 0 and (ctx & 0x3) and gctx != 0x3 for c, ctx, gctx in free[1::2]), free
    # with it, the first change-back still moves it; after the third change it stays
    assert pinned[1][0] == 0 and pinned[1][1] & 0x3, pinned
    assert all(ctx & 0x3 == 0 and gctx == 0x3 for c, ctx, gctx in pinned[3:]), pinned
    # a single memory tenant: no pin, the compute phases still move it
    assert all(c == 0 and (ctx & 0x3) for c, ctx, gctx in single[1::2]), single


def test_atc_keeps_the_class_budget_layout():
    """sched=atc on a class_budget layout: the budget places every slot (one
    per partition of its tenant's SEs); ATC's hard-affinity spreading of a
    tenant's slots (X:xen/common/sched_credit_atc.c:634-651) is skipped there
    -- on top of the layout it pinned slots away from their class homes and
    left half the partitions idle (4mix under atc: 0.58, s29)."""
    e, parts = _engine(sched="atc")
    ts = [e.tenant_create(n, nslots=32) for n in ("gemm", "hbm", "coll")]
    rates = {t: (COMPUTE if i == 0 else MEMORY) for i, t in enumerate(ts)}
    for t in ts:
        e.wake(t)
    _settle(e, rates, 3000)
    busy = foreign = n = 0
    for _ in range(100):
        _settle(e, rates, 5)
        for p, (_, x, c) in enumerate(parts):
            cur = e.partition_info(p)["curr_tenant"]
            n += 1
            if cur in ts:
                busy += 1
                foreign += (ts.index(cur) == 0) != (c < 2)
    assert busy == n and foreign == 0, (busy, n, foreign)
    assert [e.tenant_info(t).budget_ctx & 0xF for t in ts] == [0x3, 0x4, 0x8]
    assert e.check() == ""


def test_shared_region_quantum_floor():
    """region_q=1 + shared_q_us (the round-5 MI355X profile, now the gpbs-sq30
    ablation): a time-shared class region rotates
    at least that long -- three GEMM tenants sharing the compute region
    switch every 30 ms, not at their 1 ms PBS floor; 0 keeps the PBS
    region quantum (the largest adaptive quantum of the co-sharers)."""
    out = {}
    for sq in (0, 30000):
        e, parts = _engine(shared_q_us=sq, region_q=1)
        ts = [e.tenant_create(f"g{i}", nslots=32) for i in range(3)] + [e.tenant_create("hbm", nslots=32)]
        rates = {t: (COMPUTE if i < 3 else MEMORY) for i, t in enumerate(ts)}
        for t in ts:
            e.wake(t)
        _settle(e, rates, 600)
        e.trace(from_start=True)
        _settle(e, rates, 1000)
        q = [r.a[2] for r in e.trace() if r.event == "SWITCH" and r.a[1] in ts[:3]]
        out[sq] = sorted(q)[len(q) // 2] if q else 0
        assert e.check() == ""
    assert out[0] <= 2000 and out[30000] >= 30000, out


def test_reported_quanta_are_the_switch_to_switch_run_lengths():
    """the quantum the engine reports for a tenant of a
    time-shared region (tenant_info.tslice_us, the bound statistics, the
    bench's per-tenant quanta) is the s_timer quantum it is dispatched with:
    on a simulated time-shared region, every tenure that ended at its quantum
    (no wake / block in between) lasted exactly the SWITCH record's quantum,
    and that is the tenant's reported quantum -- per tenant: the 1 ms
    co-sharer and its 11 ms partners differ, and a tenant with a measured
    switch cost gets its floor (switch_floor_x x cost), not its adaptive
    target."""
    e, parts = _engine(present_us=10000)
    gs = [e.tenant_create(f"g{i}", nslots=8) for i in range(3)]
    ms = [e.tenant_create(f"m{i}", nslots=8) for i in range(4)]
    rates = {**{t: COMPUTE for t in gs}, **{t: MEMORY for t in ms}}
    for t in rates:
        e.wake(t)
    _settle(e, rates, 800)
    st = e.adapt_state(ms[3])
    st.tslice_us, st.tick_period_us = 1000, 333
    e.set_adapt_state(ms[3], st)
    rates[ms[3]] = (0, 0)  # counters stop: its adaptive quantum stays at 1 ms
    x = MI355X_PROFILE["switch_floor_x"]
    e.switch_cost(ms[2], 75_000)  # a measured 75 us switch: floor x * 75 us
    _settle(e, rates, 200)
    e.trace(from_start=True)
    _settle(e, rates, 2000)
    recs = [r for r in e.trace() if r.event == "SWITCH"]
    info = {m: e.tenant_info(m) for m in ms}
    assert info[ms[3]].tslice_us == 1000
    assert info[ms[2]].target_tslice_us == 11000 and info[ms[2]].tslice_us == max(11000, min(x * 75, 60000))
    assert info[ms[2]].switch_cost_us == 75
    # per partition, a tenure = from its SWITCH to the partition's next SWITCH.
    # The s_timer fires every dispatched quantum; a tenant re-picked at the
    # expiry (still the least-served co-sharer: region virtual time)
    # continues without a switch, so a tenure that ended at an expiry lasted
    # a whole number of its quanta.
    by_part = {}
    for r in recs:
        by_part.setdefault(r.cpu, []).append(r)
    checked = {m: 0 for m in ms}
    for p, rs in by_part.items():
        for a, b in zip(rs, rs[1:]):
            nxt, q = a.a[1], a.a[2]
            if nxt not in ms:
                continue
            assert q == info[nxt].tslice_us, (p, nxt, q, info[nxt].tslice_us)  # dispatched == reported
            run_us = (b.t_ns - a.t_ns) / 1000
            k = round(run_us / q)
            if k >= 1 and abs(run_us - k * q) <= 1:  # ended at an expiry of its own s_timer
                checked[nxt] += 1
    assert all(checked[m] > 0 for m in ms), checked
    assert e.check() == ""


def test_short_request_tenant_stays_present_and_leaves_the_probe_layout():
    """An in-region latency tenant (round-6 slo mix): 100 us requests every
    2 ms, so it is blocked at almost every class tick, and its tenures are too
    short for a clean counter window (here: no counters at all).  Its wakes
    count as work (presence), so the region is not re-laid every ~10 ms; and
    after probe_max_us of presence without a class it is laid out as memory
    class -- the GEMM keeps the compute half instead of an XCD-block probe
    share."""
    e, parts = _engine(present_us=10000, probe_max_us=50000)
    g = e.tenant_create("gemm", nslots=32)
    ms = [e.tenant_create(f"m{i}", nslots=32) for i in range(3)]
    lat = e.tenant_create("lat", nslots=32)
    rates = {g: COMPUTE, **{m: MEMORY for m in ms}}
    for t in rates:
        e.wake(t)
    _settle(e, rates, 300)
    relayouts = []
    for k in range(200):  # 400 ms of 2 ms request cycles
        e.wake(lat)
        _feed(e, rates, 100)
        e.block(lat)
        for _ in range(19):
            _feed(e, rates, 100)
        if k == 99:
            relayouts.append(e.perfc()["relayout"])
    relayouts.append(e.perfc()["relayout"])
    assert e.lib.gpbs_tenant_class(e.h, lat) < 0  # never classified ...
    info = e.tenant_info(lat)
    assert info.budget_ctx & 0xF == 0xC and info.budget_shared, info  # ... but laid out in the memory region
    assert e.tenant_info(g).budget_ctx & 0xF == 0x3  # the GEMM keeps the compute half
    assert relayouts[1] - relayouts[0] <= 1, relayouts  # the last 200 ms: a settled layout
    assert e.perfc()["probe_expired"] > 0
    assert e.check() == ""


@pytest.mark.parametrize("mode", [1, 2])
def test_crowded_memory_region_is_split_by_partitions(mode):
    """boot mem_split (the MI355X profile's default): a crowded memory region
    is split by partitions in context-major order -- an equal block per
    backlogged tenant, a small one (an eighth of the region) for a light
    tenant (a latency tenant busy at few class ticks) -- while a crowded
    compute region stays time-shared.  mem_split 2: the light tenant's block
    overlaps the last backlogged tenant's instead of idling."""
    e, parts = _engine(present_us=10000, probe_max_us=50000, mem_split=mode)
    gs = [e.tenant_create(f"g{i}", nslots=32) for i in range(3)]
    ms = [e.tenant_create(f"m{i}", nslots=32) for i in range(3)]
    lat = e.tenant_create("lat", nslots=32)
    rates = {**{g: COMPUTE for g in gs}, **{m: MEMORY for m in ms}}
    for t in rates:
        e.wake(t)
    _settle(e, rates, 300)
    for _ in range(200):  # 400 ms of 2 ms request cycles
        e.wake(lat)
        _feed(e, rates, 100)
        e.block(lat)
        for _ in range(19):
            _feed(e, rates, 100)
    info = {t: e.tenant_info(t) for t in gs + ms + [lat]}
    # compute region: time-shared, every GEMM on both compute SEs
    assert all(info[g].budget_shared and info[g].budget_ctx & 0xF == 0x3 for g in gs), info
    # memory region: 16 partitions -> 6 / 5 / 5 / ... minus the light tenant's 2
    sizes = [info[m].online_slots for m in ms]
    assert sorted(sizes) == ([4, 5, 5] if mode == 1 else [5, 5, 6]) and info[lat].online_slots == 2, (sizes, info[lat])
    assert not any(info[m].budget_shared for m in ms + [lat])
    owned = Counter()
    for p, (_, _, c) in enumerate(parts):
        if c >= 2:
            owned[e.partition_info(p)["curr_tenant"]] += 1
    # each memory tenant runs on its whole block (the light tenant's idle
    # block may lend itself to a waiting slot: class_steal work conservation)
    assert all(owned[m] == info[m].online_slots for m in ms), owned
    if mode == 2:  # the light block lies inside the largest backlogged block (SE2 of XCDs 0-5)
        assert info[lat].budget_ctx & 0xF == 0x4, hex(info[lat].budget_ctx)
        big = max(ms, key=lambda m: info[m].online_slots)
        lat_parts = {p for p in range(len(parts)) if parts[p][2] == 2 and parts[p][1] in (4, 5)}
        assert info[big].online_slots == 6 and lat_parts, info[big]
    assert e.perfc()["mem_split"] >= 1
    assert e.check() == ""


def test_swapped_classes_mirror_the_halves_instead_of_moving_tenants():
    """Equal class halves are the same hardware: when two tenants swap
    classes (config #5's trainer out-missing the decode tenant over some
    windows) the layout keeps both where they are and mirrors which half is
    the compute one -- no CU-mask change, no revocation.  A single tenant
    changing class still moves (it joins the other class's half)."""
    e, parts = _engine()
    a, b = e.tenant_create("a", nslots=32), e.tenant_create("b", nslots=32)
    rates = {a: COMPUTE, b: MEMORY}
    for t in rates:
        e.wake(t)
    _settle(e, rates)
    before = {t: e.tenant_info(t).budget_ctx & 0xF for t in (a, b)}
    assert before == {a: 0x3, b: 0xC}, before
    rel = e.perfc()["relayout"]
    _settle(e, {a: MEMORY, b: COMPUTE})
    assert e.lib.gpbs_tenant_class(e.h, a) == 1 and e.lib.gpbs_tenant_class(e.h, b) == 0
    after = {t: e.tenant_info(t).budget_ctx & 0xF for t in (a, b)}
    assert after == before, after  # nobody moved
    assert e.perfc()["mirror"] >= 1 and e.perfc()["relayout"] > rel
    own = _ctx_owners(e, parts)
    assert own[0][a] == 8 and own[1][a] == 8 and own[2][b] == 8 and own[3][b] == 8, own
    # a third tenant of the compute class joins b's (compute) half
    c = e.tenant_create("c", nslots=32)
    e.wake(c)
    _settle(e, {a: MEMORY, b: COMPUTE, c: COMPUTE})
    assert e.tenant_info(c).budget_ctx & 0xF in (0x4, 0x8), hex(e.tenant_info(c).budget_ctx)
    assert e.tenant_info(a).budget_ctx & 0xF == 0x3
    assert e.check() == ""


def test_split_blocks_stay_put_when_a_tenant_joins_the_region():
    """A memory tenant joining a split region (a phase tenant turning
    memory-bound) shrinks its neighbours' blocks in place: every incumbent
    keeps most of the partitions it held (each moved partition is a
    revocation), whatever the tenant ids."""
    e, parts = _engine(mem_split=1)
    g = e.tenant_create("gemm", nslots=32)
    late = e.tenant_create("late", nslots=32)  # lowest id of the memory tenants
    ms = [e.tenant_create(f"m{i}", nslots=32) for i in range(3)]
    rates = {g: COMPUTE, late: COMPUTE, **{m: MEMORY for m in ms}}
    for t in rates:
        e.wake(t)
    _settle(e, rates, 300)

    def homes(t):
        return {p for p, (_, _, c) in enumerate(parts) if c >= 2 and e.partition_info(p)["curr_tenant"] == t}

    before = {m: homes(m) for m in ms}
    assert all(len(v) >= 5 for v in before.values()), before
    _settle(e, {**rates, late: MEMORY}, 300)  # its phase turns memory-bound
    assert e.lib.gpbs_tenant_class(e.h, late) == 1
    after = {m: homes(m) for m in ms}
    assert len(homes(late)) == 4 and all(len(v) == 4 for v in after.values()), (after, homes(late))
    for m in ms:
        assert len(before[m] & after[m]) >= 3, (m, before[m], after[m])
    assert e.check() == ""


def test_two_tenant_probe_keeps_halves_when_one_is_classified():
    """Two present tenants, both probing, hold a class half each.  When the
    one on the upper half is classified compute first (config #5: the
    trainer, while the decode tenant has no clean window yet), neither
    moves: the pool's orientation is mirrored instead of swapping the two
    tenants' CU masks."""
    e, parts = _engine()
    a, b = e.tenant_create("a", nslots=32), e.tenant_create("b", nslots=32)
    e.wake(a)
    e.wake(b)
    _settle(e, {}, 50)  # no counters yet: the two-tenant probe (class halves)
    assert e.tenant_info(a).budget_ctx & 0xF == 0x3 and e.tenant_info(b).budget_ctx & 0xF == 0xC
    _settle(e, {b: COMPUTE}, 300)  # b classified compute; a still without counters
    assert e.lib.gpbs_tenant_class(e.h, b) == 0 and e.lib.gpbs_tenant_class(e.h, a) < 0
    assert e.tenant_info(a).budget_ctx & 0xF == 0x3 and e.tenant_info(b).budget_ctx & 0xF == 0xC
    assert e.perfc()["mirror"] >= 1
    _settle(e, {a: MEMORY, b: COMPUTE}, 300)  # a classified memory: the class layout, mirrored
    assert e.lib.gpbs_tenant_class(e.h, a) == 1
    assert e.tenant_info(a).budget_ctx & 0xF == 0x3 and e.tenant_info(b).budget_ctx & 0xF == 0xC
    assert e.check() == ""
