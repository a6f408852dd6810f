"""SE-exclusive partition mode and the PBS idle-sample rule (simulated clock).

* class_split = 2 of 4 partitions per XCD: the compute class owns shader
  engines {0,1} of every XCD and the memory class SEs {2,3}; each class group
  is one gang (all its SEs switch tenant together), so two memory tenants
  alternate on the memory SEs instead of splitting them SE by SE.
* Q14 idle-sample rule: a tenant that retired no instructions in a metric
  period is not fed to the phase detector (the reference's curr = 0 branch
  would shrink a memory-bound tenant's quantum whenever it pauses).
"""
from pbs_amd.core.config import MI355X_PROFILE
from pbs_amd.core.engine import Engine

from test_engine_credit import _feed, _procs

MS = 1_000_000


def _se_engine(**over):
    parts = [(0, x, c) for x in range(8) for c in range(4)]
    prof = dict(MI355X_PROFILE)
    prof.update(class_split=2, idle_skip=1, quantum_align_us=0)
    prof.update(over)
    e = Engine(sim_clock=True, partitions=parts, **prof)
    e.tenant_create("Domain-0", nslots=1)
    return e, parts


def test_se_mode_class_groups_and_whole_group_gangs():
    e, parts = _se_engine()
    comp = e.tenant_create("gemm", nslots=16)
    hbm = e.tenant_create("hbm", nslots=16)
    coll = e.tenant_create("coll", nslots=16)
    rates = {comp: (1000, 1), hbm: (100, 100), coll: (100, 100)}
    for t in (comp, hbm, coll):
        e.wake(t)
    for _ in range(600):  # classify, place, settle
        _feed(e, rates, 100)
    ctx = {p: c for p, (_, _, c) in enumerate(parts)}
    assert sorted(ctx[p] for p in _procs(e, comp)) == [0] * 8 + [1] * 8
    for m in (hbm, coll):
        assert all(ctx[p] >= 2 for p in _procs(e, m)), (m, _procs(e, m))
    mem_parts = [p for p in range(len(parts)) if ctx[p] >= 2]
    aligned = samples = 0
    base = {t: e.tenant_info(t).run_ns for t in (comp, hbm, coll)}
    t0 = e.now()
    for _ in range(1000):
        _feed(e, rates, 100)
        running = {e.partition_info(p)["curr_tenant"] for p in mem_parts}
        running.discard(-1)
        samples += 1
        aligned += len(running) <= 1
    dt = e.now() - t0
    share = {t: (e.tenant_info(t).run_ns - base[t]) / dt for t in (comp, hbm, coll)}
    # the compute tenant holds all 16 compute SEs; the two memory tenants
    # alternate on the 16 memory SEs with equal credit shares
    assert share[comp] > 15.5, share
    assert abs(share[hbm] - share[coll]) < 2.0 and share[hbm] + share[coll] > 15.0, share
    assert aligned / samples > 0.9, (aligned, samples)
    assert e.check() == ""


def test_se_mode_work_conserving_when_compute_idles():
    e, parts = _se_engine()
    comp = e.tenant_create("gemm", nslots=16)
    hbm = e.tenant_create("hbm", nslots=32)
    rates = {comp: (1000, 1), hbm: (100, 100)}
    e.wake(comp)
    e.wake(hbm)
    for _ in range(300):
        _feed(e, rates, 100)
    e.block(comp)
    base = e.tenant_info(hbm).run_ns
    t0 = e.now()
    for _ in range(200):
        _feed(e, rates, 100)
    # the memory tenant spreads onto the idle compute SEs
    assert (e.tenant_info(hbm).run_ns - base) / (e.now() - t0) > 24, e.tenant_info(hbm)
    assert e.check() == ""


def _bursty_quantum(idle_skip):
    e = Engine(sim_clock=True, partitions=[(0, 0)], **dict(MI355X_PROFILE, idle_skip=idle_skip))
    e.tenant_create("Domain-0", nslots=1)
    m = e.tenant_create("hbm", nslots=1)
    rates = {m: (100, 100)}  # 1e5 misses per 100k instructions: cache-sensitive
    for _ in range(40):  # 3 ms of work, 3 ms paused between quotas
        e.wake(m)
        for _ in range(30):
            _feed(e, rates, 100)
        e.block(m)
        for _ in range(30):
            _feed(e, rates, 100)
    return e, m


def test_idle_sample_rule_keeps_memory_bound_quantum():
    e1, m1 = _bursty_quantum(1)
    e0, m0 = _bursty_quantum(0)
    q1, q0 = e1.tenant_info(m1).tslice_us, e0.tenant_info(m0).tslice_us
    assert e1.perfc()["adapt_idle_skip"] > 0
    assert e0.perfc().get("adapt_idle_skip", 0) == 0
    # skipping the paused periods lets PBS grow the quantum to its maximum;
    # feeding them (reference semantics) keeps knocking it down
    assert q1 == MI355X_PROFILE["adapt"]["max_us"], q1
    assert q0 < q1, (q0, q1)


def test_se_mode_two_compute_tenants_take_aligned_halves():
    """Config #2 (two GEMM tenants, one class alone in the pool): each tenant
    ends on one class half -- SEs {0,1} or {2,3} of every XCD -- so its
    runner's CU-masked stream covers exactly what it owns.  Before the
    wrong-SE rule the credit dynamics settled at {0,3} / {1,2} (the XCD
    counts were right, so nothing moved them), and both runners launched
    unmasked full-GPU grids that queued behind the other's SEs (0.73 vs 1.26
    solo-equivalents under plain sharing on MI355X)."""
    e, parts = _se_engine()
    a = e.tenant_create("gemm", nslots=16)
    b = e.tenant_create("gemm_b", nslots=16)
    rates = {a: (1000, 1), b: (1000, 1)}
    e.wake(a)
    e.wake(b)
    for _ in range(300):
        _feed(e, rates, 100)
    ctx = {p: c for p, (_, _, c) in enumerate(parts)}
    halves = [{ctx[p] // 2 for p in _procs(e, t)} for t in (a, b)]
    assert all(len(h) == 1 for h in halves) and halves[0] != halves[1], halves
    for t in (a, b):  # one slot per (XCD, SE) of the half
        assert len(set(_procs(e, t))) == 16
    assert e.check() == ""
