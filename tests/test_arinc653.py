"""ARINC 653 time partitions (S4; X:xen/common/sched_arinc653.c): a cyclic
major frame of windows, the owner alone runs in its window, idle otherwise
(never work-conserving), tables validated and effective at once
(arinc653_sched_set :222-289, a653sched_do_schedule :516-597), every
partition of the pool switching on the same window boundaries."""
import io
import os
import tempfile
from contextlib import redirect_stderr, redirect_stdout

import pytest

from pbs_amd.core.engine import Engine
from pbs_amd.core.errors import GpbsError
from pbs_amd.ctl import cli
from pbs_amd.runtime.daemon import Daemon

MS = 1_000_000


def mk(nparts=4):
    e = Engine(sched="arinc653", sim_clock=True, partitions=[(0, x) for x in range(nparts)])
    e.tenant_create("Domain-0", nslots=1)
    return e


def run_frames(e, frames, frame_ms):
    now = e.now()
    for _ in range(frames):
        now += frame_ms * MS
        e.advance(now)


def test_windows_give_exact_time_and_idle_the_rest():
    e = mk()
    a = e.tenant_create("a", nslots=4)
    b = e.tenant_create("b", nslots=4)
    e.wake(a)
    e.wake(b)
    e.arinc653_set(0, 10000, [(a, -1, 3000), (b, -1, 5000)])
    run_frames(e, 20, 10)
    ra, rb = e.tenant_info(a).run_ns, e.tenant_info(b).run_ns
    assert ra == 20 * 3 * MS * 4 and rb == 20 * 5 * MS * 4, (ra, rb)  # 4 slots, one per partition
    assert e.tenant_info(a).tslice_us == 3000 and e.tenant_info(b).tslice_us == 5000
    assert e.check() == ""


def test_not_work_conserving_blocked_owner_idles_its_window():
    e = mk()
    a = e.tenant_create("a", nslots=4)
    b = e.tenant_create("b", nslots=4)
    e.wake(b)  # a never wakes
    e.arinc653_set(0, 8000, [(a, -1, 4000), (b, -1, 4000)])
    run_frames(e, 10, 8)
    assert e.tenant_info(a).run_ns == 0
    assert e.tenant_info(b).run_ns == 10 * 4 * MS * 4  # only its own windows


def test_slot_entry_runs_only_that_slot():
    e = mk()
    a = e.tenant_create("a", nslots=4)
    e.wake(a)
    e.arinc653_set(0, 5000, [(a, 2, 5000)])
    run_frames(e, 4, 5)
    runs = [e.slot_info(e.slot_id(a, k))["run_ns"] for k in range(4)]
    assert runs[2] == 4 * 5 * MS and runs[0] == runs[1] == runs[3] == 0, runs


def test_partitions_switch_together_on_window_boundaries():
    e = mk(nparts=8)
    a = e.tenant_create("a", nslots=8)
    b = e.tenant_create("b", nslots=8)
    e.wake(a)
    e.wake(b)
    t0 = e.now()
    e.arinc653_set(0, 6000, [(a, -1, 2000), (b, -1, 4000)])
    run_frames(e, 5, 6)
    sw = [r for r in e.trace(from_start=True) if r.event == "SWITCH" and r.t_ns >= t0]
    times = {}
    for r in sw:
        times.setdefault(r.t_ns, set()).add(r.cpu)
    # every switch instant moves all 8 partitions at once, at a window edge
    for t, cpus in times.items():
        assert len(cpus) == 8, (t, cpus)
        assert (t - t0) % (2 * MS) == 0, t - t0


@pytest.mark.parametrize("major,entries", [
    (0, [(1, -1, 100)]),           # major frame must be positive
    (1000, []),                    # at least one entry
    (1000, [(1, -1, 0)]),          # runtime must be positive
    (1000, [(1, -1, 600), (1, -1, 500)]),  # windows exceed the frame
    (1000, [(1, -2, 100)]),        # bad slot
])
def test_invalid_tables_are_rejected(major, entries):
    e = mk()
    e.tenant_create("a", nslots=1)
    with pytest.raises(GpbsError):
        e.arinc653_set(0, major, entries)
    assert e.arinc653_get(0)["explicit"] is False  # the old (automatic) table stays


def test_non_arinc_pool_rejects_tables():
    e = Engine(sched="credit", sim_clock=True, partitions=[(0, 0)])
    with pytest.raises(GpbsError):
        e.arinc653_set(0, 1000, [(0, -1, 100)])


def test_automatic_table_until_one_is_installed():
    e = mk()
    a = e.tenant_create("a", nslots=4)
    b = e.tenant_create("b", nslots=4)
    e.wake(a)
    e.wake(b)
    s = e.arinc653_get(0)
    assert not s["explicit"] and [x[0] for x in s["entries"]] == [a, b]
    assert s["major_frame_us"] == 20000
    run_frames(e, 10, 20)
    ra, rb = e.tenant_info(a).run_ns, e.tenant_info(b).run_ns
    assert ra == rb == 10 * 10 * MS * 4


def test_new_table_takes_effect_at_once():
    e = mk()
    a = e.tenant_create("a", nslots=4)
    b = e.tenant_create("b", nslots=4)
    e.wake(a)
    e.wake(b)
    e.arinc653_set(0, 100000, [(a, -1, 100000)])  # a owns a 100 ms frame
    e.advance(e.now() + 10 * MS)
    e.arinc653_set(0, 10000, [(b, -1, 10000)])  # mid-frame: b from now on
    b0 = e.tenant_info(b).run_ns
    run_frames(e, 3, 10)
    assert e.tenant_info(b).run_ns - b0 == 3 * 10 * MS * 4


def _cli(d, *args):
    out, err = io.StringIO(), io.StringIO()
    with redirect_stdout(out), redirect_stderr(err):
        rc = cli.main(["--socket", d.socket_path] + list(args))
    return rc, out.getvalue(), err.getvalue()


def test_gpbsctl_sched_arinc653():
    path = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
    d = Daemon(path, gpus=[0], nctx=1, sim=True, profile="reference").start()
    try:
        assert _cli(d, "pool-gpu-remove", "Pool-0", "0-3")[0] == 0
        assert _cli(d, "pool-create", "rt", "--sched", "arinc653", "--cpus", "0-3")[0] == 0
        assert _cli(d, "create", "ctl", "--slots", "4", "--pool", "rt")[0] == 0
        assert _cli(d, "create", "nav", "--slots", "4", "--pool", "rt")[0] == 0
        rc, out, _ = _cli(d, "sched-arinc653", "-p", "rt")
        assert rc == 0 and "(automatic)" in out
        rc, out, _ = _cli(d, "sched-arinc653", "-p", "rt", "-f", "20000", "ctl=5000", "nav:1=10000")
        assert rc == 0, out
        lines = out.splitlines()
        assert lines[0] == "Cpupool rt: major_frame=20000us"
        assert lines[2].split() == ["ctl", lines[2].split()[1], "all", "5000"]
        assert lines[3].split()[2:] == ["1", "10000"]
        rc, _, err = _cli(d, "sched-arinc653", "-p", "rt", "-f", "1000", "ctl=5000")
        assert rc != 0 and "exceeds the major frame" in err
        rc, _, err = _cli(d, "sched-arinc653", "ctl=5000")
        assert rc == 1 and "Must specify the major frame" in err
        rc, _, err = _cli(d, "sched-arinc653", "-p", "Pool-0")
        assert rc != 0 and "arinc653" in err
    finally:
        d.stop()


def test_snapshot_restores_the_table():
    from pbs_amd.utils import snapshot
    e = mk()
    a = e.tenant_create("a", nslots=4)
    b = e.tenant_create("b", nslots=4)
    e.arinc653_set(0, 9000, [(b, -1, 2000), (a, 1, 3000)])
    doc = snapshot.capture(e)
    e2 = mk()
    snapshot.restore(e2, doc)
    s = e2.arinc653_get(0)
    names = {e2.tenant_info(t).name: t for t in e2.tenants()}
    assert s["explicit"] and s["major_frame_us"] == 9000
    assert s["entries"] == [(names["b"], -1, 2000.0), (names["a"], 1, 3000.0)]
