"""Pure-Python oracle of the reference's scheduling semantics.

An independent transcription (not a binding) of:

* the built PBS phase detector / adaptive quantum
  (X:xen/common/sched_credit.c:261-389),
* the unbuilt ATC policy (X:xen/common/sched_credit_atc.c:210-543, Appendix B),
* the credit fair-share accounting with the PBS ceiling change
  (X:xen/common/sched_credit.c:1302-1519, Appendix C).

The native engine (csrc/core) and the HIP batched kernel (csrc/hip/adapt.hip)
are tested bit-for-bit against these functions.  Python ints model C
``unsigned long long`` arithmetic exactly when values stay below 2**63; the
``strict_ref`` flag reproduces the reference's u16/u32/int truncations.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import List, Optional

WINDOW = 5
PHASE_LOW = 1   # cache-sensitive (SPIN_LOW_PHASE)
PHASE_HIGH = 2


@dataclass
class AdaptParams:
    threshold: int = 100
    band_lo: int = 70
    band_hi: int = 130
    min_us: int = 100
    max_us: int = 1100
    inc_us: int = 100
    dec_us: int = 200
    switch_boundary: int = 900
    ticks_per_tslice: int = 3
    spin_floor: int = 10000
    scale: int = 100000
    strict_ref: int = 0


@dataclass
class AdaptState:
    tslice_us: int = 100
    tick_period_us: int = 33
    window_left: int = WINDOW
    stable_count: int = 0
    phase: int = PHASE_LOW
    last_err: int = 0
    last_curr: int = 0
    last_win: int = 0
    filter: List[List[int]] = field(default_factory=lambda: [[0, 0, 0] for _ in range(WINDOW)])

    @classmethod
    def initial(cls, p: AdaptParams, tslice_us: int = 100) -> "AdaptState":
        return cls(tslice_us=tslice_us, tick_period_us=tslice_us // p.ticks_per_tslice)


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def _cdiv(a: int, b: int) -> int:
    """C truncating division for possibly-negative ints."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def dec(t: int, p: AdaptParams) -> int:
    if t >= p.switch_boundary * 3:
        return t // (3 * p.inc_us) * p.inc_us
    return t - p.dec_us if t >= p.min_us + p.dec_us else p.min_us


def inc(t: int, p: AdaptParams) -> int:
    return p.max_us if t + p.inc_us >= p.max_us else t + p.inc_us


def _entry(p: AdaptParams, spin: int, inst: int, miss: int):
    if p.strict_ref:
        return [spin & 0xFFFF, inst & 0xFFFFFFFF, miss & 0xFFFFFFFF]
    return [spin, inst, miss]


def adapt_update(s: AdaptState, p: AdaptParams, inst: int, miss: int, spin_sum: int = 0, spin_count: int = 0):
    """One 1-ms metric update of one tenant.  Returns (direction, rearmed)."""
    before = s.tslice_us
    rearm = False
    thr = p.threshold
    curr = (miss * p.scale // inst) if inst else 0
    if p.strict_ref:
        curr = _i32(curr)
    avg_spin = spin_sum // spin_count if spin_count else 0
    s.last_curr = curr
    if s.window_left > 0:
        s.filter[WINDOW - s.window_left] = _entry(p, avg_spin, inst, miss)
        s.window_left -= 1
        if 0 < curr < thr:
            s.tslice_us = dec(s.tslice_us, p)
        s.last_win = -1
        s.last_err = -1
    else:
        inst_mean = sum(e[1] for e in s.filter) // WINDOW
        miss_mean = sum(e[2] for e in s.filter) // WINDOW
        win = (miss_mean * p.scale // inst_mean) if inst_mean else 0
        if p.strict_ref:
            win = _i32(win)
        if win > 0:
            err = _cdiv(curr * 100, win)
            if p.strict_ref:
                err = _i32(err)
        else:
            err = 100 if curr == 0 else 0
        s.last_win = win
        s.last_err = _i32(err)
        stable = (p.band_lo <= err <= p.band_hi) or (err > p.band_hi and win >= thr) or (curr < thr and win < thr)
        if stable:
            s.stable_count += 1
            s.filter = s.filter[1:] + [_entry(p, avg_spin, inst, miss)]
            if win >= thr:
                s.phase = PHASE_LOW
                s.tslice_us = inc(s.tslice_us, p)
            else:
                s.phase = PHASE_HIGH
                s.tslice_us = dec(s.tslice_us, p)
            s.tick_period_us = s.tslice_us // p.ticks_per_tslice
        else:
            s.stable_count = 0
            s.filter = [[0, 0, 0] for _ in range(WINDOW)]
            s.filter[0] = _entry(p, avg_spin, inst, miss)
            s.window_left = WINDOW - 1
            if curr < thr:
                s.tslice_us = dec(s.tslice_us, p)
            rearm = True
    d = 1 if s.tslice_us > before else (-1 if s.tslice_us < before else 0)
    return d, rearm


# ----------------------------------------------------------------- ATC -----

@dataclass
class AtcParams:
    default_us: int = 30000
    min_us: int = 300
    max_us: int = 30000
    zero_step_us: int = 500
    climb_step_us: int = 1000
    climb_floor_us: int = 1300
    base_us: int = 49980
    slope_us: int = 3300
    alpha: int = 4
    warmup: int = 3
    apply_period_us: int = 21000
    wait_unit_ns: int = 0  # gpbs: ns per reference spin iteration (0/1 = raw)


@dataclass
class AtcState:
    spin: int = 0
    spin_count: int = 0
    prev_spin_count: int = 0
    count: int = 3
    zero_count: int = 0
    tslice_us: int = 30000
    hist: List[List[int]] = field(default_factory=lambda: [[0, 0] for _ in range(4)])  # [bucket, tslice]

    @classmethod
    def initial(cls, p: AtcParams) -> "AtcState":
        s = cls(count=p.warmup, tslice_us=p.default_us)
        s.hist[0][1] = p.default_us
        return s


EDGES = [1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 32768]


def atc_bucket(x: int) -> int:
    if x < 1024:
        return 1
    i = 0
    while i < 10 and not x < EDGES[i]:
        i += 1
    return i + 6


def atc_report(s: AtcState, p: AtcParams, wait: int):
    if p.wait_unit_ns > 1:
        wait //= p.wait_unit_ns
    s.spin = s.spin // p.alpha + wait // p.alpha * (p.alpha - 1)
    s.spin_count += 1


def _climb_down(prev: int, p: AtcParams) -> int:
    return prev - p.climb_step_us if prev >= p.climb_floor_us else p.min_us


def atc_update(s: AtcState, p: AtcParams):
    b = atc_bucket(s.spin)
    if s.spin_count <= 1 and b == 1:
        s.zero_count += 1
        s.prev_spin_count = s.spin_count
        s.spin_count = 0
        s.spin = 0
        s.tslice_us = s.tslice_us + p.zero_step_us if s.tslice_us < p.max_us - p.zero_step_us else p.max_us
        if s.count == 0:
            s.hist = s.hist[1:] + [[b, s.tslice_us]]  # Q10 fix: push the current slice
        return
    if s.count > 0:
        if b == 1:
            t = p.max_us
        elif b <= 15:
            t = p.base_us - p.slope_us * b
        else:
            t = p.min_us
        s.hist[p.warmup - s.count] = [b, t]
        s.count -= 1
    else:
        h = s.hist
        if h[2][0] < b:
            nh = h[1:]
            t = _climb_down(nh[2][1], p)
        elif h[2][0] == b:
            nh = h[1:]
            t = nh[2][1]
        else:
            falling = h[0][0] >= h[1][0] and h[1][1] >= h[2][1]
            nh = h[1:]
            t = _climb_down(nh[2][1], p) if falling else nh[2][1]
        s.hist = [list(x) for x in nh] + [[b, t]]
    s.prev_spin_count = s.spin_count
    s.spin_count = 0
    s.tslice_us = t


def atc_apply(states: List[AtcState], p: AtcParams) -> int:
    """csched_update_acct: update every active tenant, then the global min."""
    mn = 30000 * 10
    for s in states:
        atc_update(s, p)
        mn = min(mn, s.tslice_us)
    for s in states:
        s.tslice_us = mn
        s.hist[3][1] = mn
    return mn


# ------------------------------------------------------- credit accounting --

@dataclass
class OSlot:
    credit: int = 0
    pri: int = -1
    parked: bool = False
    active: bool = True


@dataclass
class ODom:
    id: int
    weight: int = 256
    cap: int = 0
    slots: List[OSlot] = field(default_factory=list)

    @property
    def active_count(self):
        return sum(1 for s in self.slots if s.active)


PRI_BOOST, PRI_UNDER, PRI_OVER, PRI_IDLE = 0, -1, -2, -64


def credit_acct(doms: List[ODom], ncpus: int, cpt: int, balance: int, dom0_quirk: bool = True):
    """One csched_acct pass over the active domains (in list order).

    Returns (new_balance, new_order, parks) where parks lists (dom, slot,
    parked) transitions.  Mutates slot credits/priorities/activity.
    """
    active = [d for d in doms if d.active_count > 0]
    weight_total = sum(d.weight * d.active_count for d in active)
    credit_total = ncpus * cpt
    if balance < 0:
        credit_total += -balance
    if weight_total == 0:
        return 0, [d.id for d in active], []
    weight_left = weight_total
    credit_balance = 0
    xtra = False
    order = [d.id for d in active]
    parks = []
    for d in list(active):
        n = d.active_count
        w = d.weight
        weight_left -= w * n
        peak = n * cpt
        if balance < 0:
            peak += (-balance * w * n + weight_total - 1) // weight_total
        capc = 0
        if d.cap:
            capc = (d.cap * cpt + 99) // 100
            peak = min(peak, capc)
            capc = (capc + n - 1) // n
        fair = (credit_total * w * n + weight_total - 1) // weight_total
        if fair < peak:
            xtra = True
        else:
            if weight_left:
                credit_total += ((fair - peak) * weight_total + weight_left - 1) // weight_left
            if xtra:
                order.remove(d.id)
                order.insert(0, d.id)
            fair = peak
        fair = (fair + n - 1) // n
        for s in [s for s in d.slots if s.active]:
            s.credit += fair
            c = s.credit
            if c < 0:
                s.pri = PRI_OVER
                if d.cap and c < -capc and not s.parked:
                    s.parked = True
                    parks.append((d.id, d.slots.index(s), 1))
                if c < -cpt:
                    c = -cpt
                    s.credit = c
            else:
                s.pri = PRI_UNDER
                if s.parked:
                    s.parked = False
                    parks.append((d.id, d.slots.index(s), 0))
                if dom0_quirk:
                    if _cdiv(c, 100) > cpt // 100 and d.id == 0:
                        if n >= 2:
                            s.active = False
                    elif _cdiv(c, 100) > cpt // 100 and d.id != 0:
                        c = _cdiv(c, 2)
                        s.credit = c
                elif c > cpt:
                    s.active = False
                    c = _cdiv(c, 2)
                    s.credit = c
            credit_balance += c
    return credit_balance, order, parks


def burn_credits(delta_ns: int) -> int:
    """credits burned for delta_ns of running (1 credit per us, rounded)."""
    if delta_ns <= 0:
        return 0
    return (delta_ns * 1000 + 500000) // 1000000


def clone(x):
    return copy.deepcopy(x)
