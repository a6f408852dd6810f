"""Fault injection (S13; the mce-test analog, X:tools/tests/mce-test): the
scheduler keeps its invariants and fairness while counters go stale or reset,
heartbeats get lost, actuation lags and timers fire late."""
import os
import subprocess
import sys

from pbs_amd.core.engine import Engine

MS = 1_000_000


def _feed(e, rates, dt_us):
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


def _mk(spec, **kw):
    parts = [(0, x, c) for x in range(4) for c in range(2)]
    e = Engine(sim_clock=True, partitions=parts, quantum_align_us=0, **kw)
    e.tenant_create("Domain-0", nslots=1)
    assert e.fault_set(spec) >= 1
    return e


def test_counter_faults_keep_adaptation_and_classes_sane():
    e = _mk("counter_reset=20000,counter_drop=100000,seed=7", coschedule=2, class_period_us=2000)
    comp = e.tenant_create("gemm", nslots=4)
    mem = e.tenant_create("hbm", nslots=4)
    e.wake(comp)
    e.wake(mem)
    for _ in range(400):
        _feed(e, {comp: (1000, 1), mem: (100, 100)}, 100)
    hits = e.fault_hits()
    assert hits["counter_reset"] > 0 and hits["counter_drop"] > 0
    assert e.perfc()["counter_reset"] > 0          # Q5 skip path exercised
    for t in (comp, mem):
        ts = e.tenant_info(t).tslice_us
        assert 100 <= ts <= 1100, ts                 # adaptation stays in bounds
    assert e.check() == ""


def test_timer_jitter_and_actuation_delay_preserve_fair_share():
    e = _mk("timer_jitter=300000:400,actuate_delay=200000,seed=3")
    e.sched_params_set(0, 1000, 100)
    a = e.tenant_create("a", nslots=8)
    b = e.tenant_create("b", nslots=8, weight=512)
    e.wake(a)
    e.wake(b)
    base = {t: e.tenant_info(t).run_ns for t in (a, b)}
    t0 = e.now()
    while e.now() < t0 + 400 * MS:
        e.advance(e.now() + 50_000)
    sh = {t: (e.tenant_info(t).run_ns - base[t]) / (e.now() - t0) for t in (a, b)}
    hits = e.fault_hits()
    assert hits["timer_jitter"] > 0 and hits["actuate_delay"] > 0
    assert abs(sh[a] - 8 / 3) < 0.6 and abs(sh[b] - 16 / 3) < 0.6, sh  # 1:2 over 8 partitions
    assert e.check() == ""


def test_heartbeat_loss_pauses_the_tenant():
    e = _mk("heartbeat_drop=1000000", heartbeat_timeout_us=5000)
    t = e.tenant_create("silent", nslots=2)
    e.wake(t)
    for _ in range(40):
        e.heartbeat(t)              # every one of them is dropped
        e.advance(e.now() + 500_000)
    assert e.tenant_info(t).paused >= 1
    assert any(r.event == "DEAD" for r in e.trace(from_start=True))
    assert e.fault_hits()["heartbeat_drop"] >= 40


def test_env_var_arms_faults_at_engine_creation():
    code = ("from pbs_amd.core.engine import Engine\n"
            "e = Engine(sim_clock=True, partitions=[(0, 0), (0, 1)])\n"
            "e.tenant_create('Domain-0', nslots=1)\n"
            "t = e.tenant_create('a', nslots=2); e.wake(t)\n"
            "e.advance(e.now() + 50_000_000)\n"
            "print(e.fault_hits()['timer_jitter'], 'armed' in e.dmesg())\n")
    env = dict(os.environ, GPBS_FAULT="timer_jitter=500000:50,seed=11")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    hits, armed = out.stdout.split()
    assert int(hits) > 0 and armed == "True", out.stderr


def test_torn_page_fault_is_caught_by_the_seqlock():
    """torn_page: every control-page publish pauses half-written; a reader
    polling the page concurrently retries (odd sequence / changed sequence)
    and never returns a torn assignment (gate set iff the mask is non-empty)."""
    import ctypes as C
    import tempfile
    import threading

    from pbs_amd import _native as N
    from pbs_amd.runtime.daemon import Daemon
    d = Daemon(os.path.join(tempfile.mkdtemp(), "gpbsd.sock"), gpus=[0], nctx=2, sim=True, profile="mi355x")
    d.start(reaper_s=0)
    try:
        regs = [d.register(name=n, slots=16, pid=os.getpid()) for n in ("a", "b")]
        assert d.engine.fault_set("torn_page=1000000:300") == 1
        lib = N.load_core()
        h = lib.gpbs_ctl_open(regs[0]["ctl"].encode())
        page = regs[0]["page"]
        stop = threading.Event()
        seen = {"reads": 0, "retries": 0, "bad": 0}

        def reader():
            g, q, ep = C.c_uint32(), C.c_uint32(), C.c_uint32()
            m = (C.c_uint64 * 2)()
            pr, tid = C.c_int32(), C.c_int32()
            while not stop.is_set():
                r = lib.gpbs_ctl_read(C.c_void_p(h), page, C.byref(g), m, C.byref(q), C.byref(pr), C.byref(tid),
                                      C.byref(ep))
                if r < 0:
                    continue
                seen["reads"] += 1
                seen["retries"] += r
                if bool(g.value) != bool(m[0] | m[1]):
                    seen["bad"] += 1

        th = threading.Thread(target=reader)
        th.start()
        for t in (r["tenant"] for r in regs):
            d.engine.wake(t)
        import time
        deadline = time.monotonic() + 10.0
        k = 0
        # at least 300 steps; then until the reader has met a torn page (the
        # torn window is wall-clock: the bridge completes it later)
        while k < 300 or (seen["retries"] == 0 and time.monotonic() < deadline):
            d.advance_us(250)
            k += 1
            if k >= 300 and seen["retries"] == 0:
                time.sleep(0.001)
        stop.set()
        th.join()
        assert d.engine.fault_hits()["torn_page"] > 0
        assert seen["reads"] > 0 and seen["retries"] > 0, seen
        assert seen["bad"] == 0, seen
        # a publish that meets a pending torn one completes it
        # first, so once the last torn publish lands the page holds exactly
        # the engine's assignment (no stale mask word, no lost quantum)
        d.engine.fault_set("")
        d.advance_us(250)
        time.sleep(0.05)  # the bridge completes the last deferred half
        g, q, ep = C.c_uint32(), C.c_uint32(), C.c_uint32()
        m = (C.c_uint64 * 2)()
        pr, tid = C.c_int32(), C.c_int32()
        assert lib.gpbs_ctl_read(C.c_void_p(h), page, C.byref(g), m, C.byref(q), C.byref(pr), C.byref(tid),
                                 C.byref(ep)) >= 0
        want = 0
        for p in range(d.engine.num_partitions):
            if d.engine.partition_info(p)["curr_tenant"] == regs[0]["tenant"]:
                want |= 1 << p
        assert (m[0] | (m[1] << 64)) == want, (hex(m[0]), hex(m[1]), hex(want))
        assert bool(g.value) == bool(want)
        lib.gpbs_ctl_close(C.c_void_p(h), 0)
    finally:
        d.stop()
