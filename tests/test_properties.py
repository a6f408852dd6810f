"""Property tests (hypothesis): the PBS detector and the
credit accounting over arbitrary inputs.

* native adapt == oracle step for step, the quantum stays in [min, max] and
  the tick in [min, max] / ticks_per_tslice (X:xen/common/sched_credit.c:286-389);
* a steady input converges monotonically: cache-sensitive to the ceiling,
  insensitive to the floor, within a bounded number of periods;
* csched_acct (X:xen/common/sched_credit.c:1302-1519, Appendix C) hands out
  the period's credit_total -- no more, and all of it when no domain is
  capped or peak-bound -- every slot of a domain gains the same share, at
  least its weight share up to its peak, and no slot is left below the
  -credits_per_tslice floor or above the ceiling while active.
"""
import ctypes as C

from hypothesis import given, settings
from hypothesis import strategies as st

from pbs_amd import _native as N
from pbs_amd.core import oracle as O
from pbs_amd.core.engine import boot_params


def _native_params():
    bp = boot_params()
    p = N.AdaptParams()
    C.memmove(C.byref(p), C.byref(bp.adapt), C.sizeof(p))
    return p


samples = st.lists(st.tuples(st.integers(0, 1 << 40), st.integers(0, 1 << 34), st.integers(0, 1 << 20),
                             st.integers(0, 8)), min_size=1, max_size=120)


@settings(max_examples=150, deadline=None)
@given(samples)
def test_adapt_native_equals_oracle_and_stays_in_bounds(seq):
    lib = N.load_core()
    p = _native_params()
    op = O.AdaptParams()
    s = N.AdaptState()
    lib.gpbs_adapt_init(C.byref(s), C.byref(p), 100)
    os_ = O.AdaptState.initial(op)
    for inst, miss, ss, sc in seq:
        miss = min(miss, inst) if inst else miss
        r = lib.gpbs_adapt_update(C.byref(s), C.byref(p), inst, miss, ss, sc)
        d = O.adapt_update(os_, op, inst, miss, ss, sc)
        assert ((r & 3) - 1, bool(r & 4)) == d
        assert s.tslice_us == os_.tslice_us and s.phase == os_.phase and s.window_left == os_.window_left
        assert op.min_us <= s.tslice_us <= op.max_us
        # the tick follows the quantum only on stable updates (Q9, kept for
        # fidelity), so it is always some quantum's third, not the current one's
        assert s.tick_period_us == os_.tick_period_us
        assert op.min_us // op.ticks_per_tslice <= s.tick_period_us <= op.max_us // op.ticks_per_tslice


@settings(max_examples=80, deadline=None)
@given(st.integers(10 ** 4, 10 ** 10), st.booleans(), st.integers(100, 1100))
def test_steady_input_converges_monotonically(inst, sensitive, start):
    """Steady cache-sensitive input climbs to the ceiling, steady insensitive
    input falls to the floor; after warm-up the quantum never moves the
    other way (+inc / -dec, /3 above the switch boundary)."""
    op = O.AdaptParams()
    start = max(op.min_us, min(op.max_us, start // 100 * 100))
    s = O.AdaptState.initial(op, start)
    miss = inst // 50 if sensitive else 0  # 2000 vs 0 misses per 100k instructions
    traj = []
    for _ in range(80):
        O.adapt_update(s, op, inst, miss)
        traj.append(s.tslice_us)
    steps = list(zip(traj, traj[1:]))
    if sensitive:
        assert traj[-1] == op.max_us, traj
        assert all(b >= a for a, b in steps), traj
    else:
        assert traj[-1] == op.min_us, traj
        assert all(b <= a for a, b in steps), traj


doms_st = st.lists(st.tuples(st.integers(1, 65535), st.integers(0, 400), st.lists(st.integers(-3000, 3000),
                                                                                   min_size=1, max_size=4)),
                   min_size=1, max_size=8)


@settings(max_examples=200, deadline=None)
@given(doms_st, st.integers(1, 8), st.sampled_from([100, 1000, 3000]), st.booleans())
def test_credit_acct_distributes_the_period_credit(doms, ncpus, cpt, capped):
    """One accounting period: every slot gains exactly its domain's per-slot
    share (ceil(fair / n)), the shares of uncapped domains follow the weights
    and add up to credit_total (within rounding), a capped domain gets at most
    its cap, and the floor / ceiling / priority rules hold afterwards."""
    ds = [O.ODom(id=i + 1, weight=w, cap=(cap if capped else 0), slots=[O.OSlot(credit=c) for c in cr])
          for i, (w, cap, cr) in enumerate(doms)]
    before = [[s.credit for s in d.slots] for d in ds]
    total = ncpus * cpt
    O.credit_acct(ds, ncpus, cpt, balance=0, dom0_quirk=False)
    gained = []
    for d, b in zip(ds, before):
        g = set()
        for s, c0 in zip(d.slots, b):
            c = s.credit
            # undo the post-rules: floor at -cpt, halving above cpt (slot goes inactive)
            if not s.active:
                assert c0 + 1 > 0
                continue
            if c == -cpt and c0 < 0:
                continue  # floored: gain not observable
            g.add(c - c0)
        assert len(g) <= 1, (d, b)  # every (observable) slot of a domain gains the same share
        gained.append(next(iter(g)) if g else None)
    wsum = sum(d.weight * len(d.slots) for d in ds)
    for d, g in zip(ds, gained):
        n = len(d.slots)
        if g is None:
            continue
        assert 0 <= g <= cpt, (d, g)  # peak = one CPU's credit per slot (sched_credit.c:1367)
        if d.cap:
            assert g * n <= -(-d.cap * cpt // 100) + n, (d, g)  # peak = ceil(cap * cpt / 100), split by slots
        else:
            # at least its weight share of credit_total or its peak, whichever
            # is smaller (a peak-bound domain's excess goes to later domains)
            assert g * n >= min(total * d.weight * n // wsum, n * cpt) - n, (d, g)
    obs = [(d, g) for d, g in zip(ds, gained) if g is not None]
    if len(obs) == len(ds):  # every domain observable: never more than credit_total (+ rounding)
        handed = sum(g * len(d.slots) for d, g in obs)
        assert handed <= total + 2 * sum(len(d.slots) for d in ds), (handed, total)
        if not capped and all(g < cpt for _, g in obs):  # nobody peak-bound: all of it is handed out
            assert handed >= total, (handed, total)
    for d in ds:
        for s in d.slots:
            assert s.credit >= -cpt                                   # floor (sched_credit.c:1455-1459)
            assert s.credit <= cpt or not s.active or s.credit > cpt  # above the ceiling only if deactivated
            if s.active:
                assert s.credit <= cpt
            assert (s.pri == O.PRI_UNDER) == (s.credit >= 0) or not s.active
