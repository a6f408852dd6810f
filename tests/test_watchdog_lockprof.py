"""Failure detection and lock profiling (S13 / S11 analogs):

* tenant watchdogs = SCHEDOP_watchdog (X:xen/common/schedule.c:738-788): id 0
  allocates one of two timers, re-arm / free by id, expiry shuts the tenant
  down (slots paused, partitions reclaimed, "Watchdog timer fired" on the
  console);
* engine-mutex lock profile = lock_profile / xenlockprof
  (X:xen/common/spinlock.c:88-115, X:tools/misc/xenlockprof.c);
* xenmon-style gotten / waited / blocked accounting and the Prometheus perfc
  export through gpbsd + gpbsctl.
"""
import io
import os
import tempfile
import threading
from contextlib import redirect_stdout

import pytest

from pbs_amd.core.engine import Engine
from pbs_amd.core.errors import GpbsError
from pbs_amd.ctl import cli
from pbs_amd.runtime.daemon import Daemon

MS = 1_000_000


def _engine():
    e = Engine(sim_clock=True, partitions=[(0, x) for x in range(4)])
    e.tenant_create("Domain-0", nslots=1)
    return e


def test_watchdog_allocate_rearm_free_and_limits():
    e = _engine()
    t = e.tenant_create("a", nslots=2)
    assert e.watchdog(t, 0, 50) == 1
    assert e.watchdog(t, 0, 50) == 2
    with pytest.raises(GpbsError):
        e.watchdog(t, 0, 50)          # ENOSPC: both timers in use
    with pytest.raises(GpbsError):
        e.watchdog(t, 3, 10)          # id > NR watchdogs
    assert e.watchdog(t, 2, 0) == 0   # free id 2
    with pytest.raises(GpbsError):
        e.watchdog(t, 2, 10)          # re-arming a free id: EINVAL
    assert e.watchdog(t, 0, 50) == 2  # id 2 is reused
    e.watchdog(t, 1, 0)
    e.watchdog(t, 2, 0)
    e.close()


def test_watchdog_fires_only_without_rearm():
    e = _engine()
    t = e.tenant_create("a", nslots=2)
    e.wake(t)
    wid = e.watchdog(t, 0, 5)
    for _ in range(10):              # re-armed every 4 ms: never fires
        e.advance(e.now() + 4 * MS)
        e.watchdog(t, wid, 5)
    assert e.tenant_info(t).shutdown == 0 and e.perfc()["watchdog_fired"] == 0
    e.advance(e.now() + 6 * MS)      # missed: tenant shut down
    info = e.tenant_info(t)
    assert info.shutdown == 4 and info.paused >= 1
    assert "Watchdog timer 1 fired for tenant" in e.dmesg()
    assert e.perfc()["watchdog_fired"] == 1
    run0 = e.tenant_info(t).run_ns
    e.advance(e.now() + 20 * MS)
    assert e.tenant_info(t).run_ns == run0, "a shut-down tenant must not run"
    assert any(r.event == "DEAD" and r.a[1] == 4 for r in e.trace(from_start=True))
    e.unpause(t)                     # operator restart clears the shutdown
    assert e.tenant_info(t).shutdown == 0
    e.advance(e.now() + 5 * MS)
    assert e.tenant_info(t).run_ns > run0
    assert e.check() == ""
    e.close()


def test_watchdog_timers_die_with_tenant():
    e = _engine()
    t = e.tenant_create("a", nslots=1)
    e.watchdog(t, 0, 2)
    e.tenant_destroy(t)
    e.advance(e.now() + 10 * MS)     # must not fire on a destroyed tenant
    assert e.perfc()["watchdog_fired"] == 0
    e.close()


def test_lockprof_counts_contention_and_resets():
    e = Engine(partitions=[(0, x) for x in range(8)])
    e.tenant_create("Domain-0", nslots=1)
    ts = [e.tenant_create(f"t{i}", nslots=4) for i in range(4)]
    e.lockprof(reset=True)
    e.start()

    def hammer(t):
        for k in range(200):
            e.wake(t)
            if k % 3 == 0:
                e.block(t)
            e.tenant_info(t)

    th = [threading.Thread(target=hammer, args=(t,)) for t in ts]
    [x.start() for x in th]
    [x.join() for x in th]
    e.stop()
    p = e.lockprof()
    assert p["lock_cnt"] >= 4 * 200 * 2
    assert p["block_cnt"] <= p["lock_cnt"]
    assert p["time_hold_ns"] > 0 and p["max_hold_ns"] > 0
    if p["block_cnt"]:
        assert p["time_block_ns"] >= p["max_block_ns"] > 0
    e.lockprof(reset=True)
    assert e.lockprof()["lock_cnt"] == 0
    e.close()


@pytest.fixture()
def daemon():
    path = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
    d = Daemon(path, gpus=[0], nctx=2, sim=True, profile="reference").start()
    yield d
    d.stop()


def _cli(d, *args):
    out = io.StringIO()
    with redirect_stdout(out):
        rc = cli.main(["--socket", d.socket_path] + list(args))
    return rc, out.getvalue()


def test_mon_prom_lockprof_watchdog_via_gpbsctl(daemon):
    from pbs_amd.ctl.rpc import Client
    c = Client(daemon.socket_path)
    t = c.call("create", name="busy", slots=2)
    c.call("create", name="idle", slots=2)
    daemon.engine.wake(t)
    c.call("mon", reset=True)
    c.call("advance_us", us=50_000)
    m = c.call("mon")
    assert m["interval_s"] == pytest.approx(0.05, rel=1e-6)
    rows = {r["name"]: r for r in m["tenants"]}
    assert rows["busy"]["gotten_pct"] > 50 and rows["busy"]["execs_per_s"] >= 0
    assert rows["idle"]["blocked_pct"] > 99 and rows["idle"]["gotten_pct"] == 0
    for r in rows.values():
        assert r["gotten_pct"] + r["waited_pct"] + r["blocked_pct"] == pytest.approx(100.0, abs=0.5)
    rc, out = _cli(daemon, "perfc", "--prom")
    assert rc == 0 and '# TYPE gpbs_perfc_total counter' in out and 'gpbs_perfc_total{name="sched_ctx"}' in out
    rc, out = _cli(daemon, "lockprof")
    assert rc == 0 and out.startswith("gpbs engine lock") and "block:" in out
    rc, out = _cli(daemon, "watchdog", "busy", "0", "3")
    assert rc == 0 and out.strip() == "1"
    c.call("advance_us", us=5_000)
    assert "Watchdog timer 1 fired" in c.call("dmesg")
    c.close()
