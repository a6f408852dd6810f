"""S4: the other pluggable schedulers -- credit2 (X:xen/common/sched_credit2.c)
and sedf (X:xen/common/sched_sedf.c) -- on the engine's simulated clock,
plus pools running different schedulers side by side (cpupool semantics)."""
import pytest

from pbs_amd.core.engine import Engine
from pbs_amd.core.errors import GpbsError

MS = 1_000_000


def share(e, ts, dur_ms=400, step_us=50):
    base = {t: e.tenant_info(t).run_ns for t in ts}
    t0 = e.now()
    end = t0 + dur_ms * MS
    while e.now() < end:
        e.advance(e.now() + step_us * 1000)
    return {t: (e.tenant_info(t).run_ns - base[t]) / (end - t0) for t in ts}


def mk(sched, parts):
    e = Engine(sched=sched, sim_clock=True, partitions=parts)
    e.tenant_create("Domain-0", nslots=1)
    return e


# ------------------------------------------------------------------ credit2 --

def test_credit2_weights_shape_the_share_on_one_partition():
    """t2c: credit burns at max_weight/weight, so 256:512 -> 1:2."""
    e = mk("credit2", [(0, 0)])
    a = e.tenant_create("a", nslots=1, weight=256)
    b = e.tenant_create("b", nslots=1, weight=512)
    e.wake(a)
    e.wake(b)
    s = share(e, [a, b], dur_ms=600)
    assert abs(s[a] + s[b] - 1.0) < 0.02, s
    assert 1.8 < s[b] / s[a] < 2.2, s
    assert e.sched_ext_get(b)["weight"] == 512
    assert e.check() == ""


def test_credit2_shared_runqueue_per_gpu_is_work_conserving():
    """One runqueue per GPU: three single-slot tenants on a GPU with two XCD
    partitions keep both partitions busy and share them evenly; a second GPU
    gets its own runqueue and load is balanced onto it."""
    e = mk("credit2", [(g, x) for g in range(2) for x in range(2)])
    ts = [e.tenant_create(f"t{i}", nslots=1) for i in range(6)]
    for t in ts:
        e.wake(t)
    s = share(e, ts, dur_ms=600)
    assert abs(sum(s.values()) - 4.0) < 0.05, s  # all four partitions busy
    for t in ts:
        assert 0.55 < s[t] < 0.78, s  # 4/6 each, within the 2 ms granularity
    dump = e.debug_keys("r")
    assert dump.count("Runqueue") >= 2, dump
    assert "max_weight" in dump
    assert e.check() == ""


def test_credit2_reset_and_no_cap():
    e = mk("credit2", [(0, 0)])
    a = e.tenant_create("a", nslots=1)
    e.wake(a)
    share(e, [a], dur_ms=50)
    w, c = e.sched_credit_get(a)
    assert (w, c) == (256, 0)
    e.sched_credit_set(a, cap=50)  # credit2 (Xen 4.2) has no caps: accepted, ignored
    assert e.sched_credit_get(a)[1] == 0
    info = e.sched_ext_get(a)
    assert info["credit"] != 0
    with pytest.raises(GpbsError):
        e.sched_params_set(0, 2000, 500)  # no global parameters in credit2
    assert "credits(us)" in e.debug_keys("z")


def test_credit2_waker_preempts_lower_credit_runner():
    """runq_tickle: a waking slot with more credit than the current one
    tickles its partition -- a mostly idle tenant gets on quickly."""
    e = mk("credit2", [(0, 0)])
    hog = e.tenant_create("hog", nslots=1)
    lat = e.tenant_create("lat", nslots=1)
    e.wake(hog)
    share(e, [hog], dur_ms=30)  # hog burns credit below the waker's
    e.wake(lat)
    e.advance(e.now() + 50_000)
    assert e.slot_info(e.slot_id(lat, 0))["is_running"]


# --------------------------------------------------------------------- sedf --

def test_sedf_time_driven_reservations_without_extra_time():
    """EDF: (10 ms, 3 ms) and (10 ms, 5 ms) reservations get 30 % and 50 %;
    without extratime the rest of the partition idles."""
    e = mk("sedf", [(0, 0)])
    a = e.tenant_create("a", nslots=1)
    b = e.tenant_create("b", nslots=1)
    e.sched_ext_set(a, period_us=10_000, slice_us=3_000, extratime=0)
    e.sched_ext_set(b, period_us=10_000, slice_us=5_000, extratime=0)
    e.wake(a)
    e.wake(b)
    s = share(e, [a, b], dur_ms=500, step_us=100)
    assert abs(s[a] - 0.30) < 0.02, s
    assert abs(s[b] - 0.50) < 0.02, s
    x = e.sched_ext_get(a)
    assert (x["period_us"], x["slice_us"], x["extratime"]) == (10_000, 3_000, 0)
    assert e.check() == ""


def test_sedf_extra_time_goes_to_best_effort_tenants():
    """A best-effort (extratime-aware, no reservation) tenant soaks up what
    the reservations leave; the reserved tenant keeps its 30 %."""
    e = mk("sedf", [(0, 0)])
    rt = e.tenant_create("rt", nslots=1)
    be = e.tenant_create("be", nslots=1)
    e.sched_ext_set(rt, period_us=10_000, slice_us=3_000, extratime=0)
    e.wake(rt)
    e.wake(be)
    s = share(e, [rt, be], dur_ms=500, step_us=100)
    assert abs(s[rt] - 0.30) < 0.02, s
    assert s[be] > 0.65, s
    assert "EXTRAQ" in e.debug_keys("r")


def test_sedf_weight_driven_reservations():
    """sedf_adjust_weights: weight-driven slots split WEIGHT_PERIOD minus
    WEIGHT_SAFETY (95 ms of every 100 ms) by weight."""
    e = mk("sedf", [(0, 0)])
    a = e.tenant_create("a", nslots=1)
    b = e.tenant_create("b", nslots=1)
    e.sched_ext_set(a, weight=1, extratime=0, period_us=100_000)
    e.sched_ext_set(b, weight=3, extratime=0, period_us=100_000)
    assert e.sched_ext_get(a)["slice_us"] == 23_750
    assert e.sched_ext_get(b)["slice_us"] == 71_250
    e.wake(a)
    e.wake(b)
    # The first wake counts as a short block (initial deadline = now + slice,
    # sched_sedf.c:1106-1110 then :1125-1136): that period is forfeited.
    share(e, [a, b], dur_ms=200, step_us=200)
    s = share(e, [a, b], dur_ms=1000, step_us=200)
    assert abs(s[a] - 0.2375) < 0.02 and abs(s[b] - 0.7125) < 0.02, s


def test_sedf_parameter_validation():
    """sedf_adjust sanity checks (:1425-1433): period in [10 us, 10 s],
    slice in [5 us, period], and period or weight required."""
    e = mk("sedf", [(0, 0)])
    a = e.tenant_create("a", nslots=1)
    for bad in (dict(period_us=10_000, slice_us=20_000), dict(period_us=5, slice_us=5),
                dict(period_us=10_000, slice_us=1), dict()):
        with pytest.raises(GpbsError):
            e.sched_ext_set(a, **bad)


def _io_wake_delay(latency_us):
    e = mk("sedf", [(0, 0)])
    hog = e.tenant_create("hog", nslots=1)
    io = e.tenant_create("io", nslots=1)
    e.sched_ext_set(hog, period_us=20_000, slice_us=15_000, extratime=0)
    e.sched_ext_set(io, period_us=100_000, slice_us=20_000, latency_us=latency_us, extratime=0)
    e.wake(hog)
    e.wake(io)
    share(e, [hog, io], dur_ms=300, step_us=100)
    e.block(io)
    share(e, [hog], dur_ms=305, step_us=100)  # long block: several of io's periods
    e.wake(io)
    t0 = e.now()
    while e.now() < t0 + 30 * MS:
        e.advance(e.now() + 50_000)
        if e.slot_info(e.slot_id(io, 0))["is_running"]:
            return e.now() - t0, e
    return None, e


def test_sedf_latency_hint_shortens_the_first_period_after_a_long_block():
    """Improved-Atropos wake (2c): a tenant waking after a long block gets a
    period of `latency` with a scaled slice, so its deadline beats the
    running reservation's and it preempts at once; without the hint its
    deadline is a whole period away and it waits for the competitor's slice."""
    with_hint, e = _io_wake_delay(2_000)
    without, _ = _io_wake_delay(0)
    assert with_hint is not None and with_hint <= 100_000, with_hint
    assert without is not None and without > 1_000_000, without
    assert "lb=" in e.debug_keys("r")
    assert e.check() == ""


# ----------------------------------------------------------- mixed pools ----

def test_pools_with_different_schedulers_side_by_side():
    """cpupools: one engine, a credit pool and a credit2 and a sedf pool, each
    with its own scheduler instance; a tenant moved between pools keeps
    running under the new policy."""
    e = Engine(sim_clock=True, partitions=[(0, x) for x in range(4)])
    e.tenant_create("Domain-0", nslots=1)
    for name, sched, part in (("c2", "credit2", 2), ("edf", "sedf", 3)):
        p = e.pool_create(name, sched)
        e.pool_unassign(0, part)
        e.pool_assign(p, part)
    pools = {i["name"]: i for i in (e.pool_info(p) for p in e.pools())}
    assert pools["c2"]["sched"] == "credit2" and pools["edf"]["sched"] == "sedf"
    t = e.tenant_create("mover", nslots=1, pool=pools["c2"]["id"])
    e.wake(t)
    assert share(e, [t], dur_ms=50)[t] > 0.95
    e.tenant_move(t, pools["edf"]["id"])
    assert share(e, [t], dur_ms=50)[t] > 0.9  # best effort: all the extra time
    e.tenant_move(t, 0)
    assert share(e, [t], dur_ms=50)[t] > 0.95
    assert e.check() == ""


@pytest.mark.parametrize("sched", ["credit", "credit2", "sedf"])
def test_initial_placement_spreads_slots_for_every_scheduler(sched):
    """Every slot starts on the least-populated partition, preferring XCDs the
    tenant does not occupy yet (default_vcpu0_location applied per slot):
    three 8-slot tenants on 8 XCDs x 4 contexts land one slot per XCD each and
    never share a partition -- a scheduler without load balancing (sedf)
    would otherwise keep a stacked partition busy next to an idle one.
    Regression: sedf ran such a mix at 3.5 of 8 partitions per tenant."""
    e = Engine(sched=sched, sim_clock=True, partitions=[(0, x, c) for x in range(8) for c in range(4)])
    e.tenant_create("Domain-0", nslots=1)
    ts = [e.tenant_create(n, nslots=8) for n in ("gemm", "hbm", "coll")]
    procs = {t: [e.slot_info(e.slot_id(t, k))["processor"] for k in range(8)] for t in ts}
    flat = [p for t in ts for p in procs[t]]
    assert len(set(flat)) == len(flat), procs
    for t in ts:
        assert sorted(p // 4 for p in procs[t]) == list(range(8)), procs  # one per XCD
    for t in ts:
        e.wake(t)
    s = share(e, ts, dur_ms=100)
    assert all(v > 7.9 for v in s.values()), s
