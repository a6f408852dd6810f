"""gpbsctl <-> gpbsd integration (the xm-test analog: tools/xm-test/tests/
sched-credit/01_sched_credit_weight_cap_pos.py, tests/cpupool/*, pause/*,
vcpu-pin/*; positive and negative cases, exact xl output formats and error
strings from X:tools/libxl/xl_cmdimpl.c:4637-4930)."""
import io
import os
import tempfile
from contextlib import redirect_stderr, redirect_stdout

import pytest

from pbs_amd.ctl import cli
from pbs_amd.runtime.daemon import Daemon


@pytest.fixture()
def daemon():
    path = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
    d = Daemon(path, gpus=[0, 1], nctx=2, sim=True, profile="reference").start()
    yield d
    d.stop()


def run(d, *args):
    out, err = io.StringIO(), io.StringIO()
    with redirect_stdout(out), redirect_stderr(err):
        rc = cli.main(["--socket", d.socket_path] + list(args))
    return rc, out.getvalue(), err.getvalue()


def test_sched_credit_weight_cap_pos(daemon):
    rc, out, _ = run(daemon, "create", "dom1", "--slots", "4")
    assert rc == 0
    rc, out, _ = run(daemon, "sched-credit", "-d", "dom1")
    assert rc == 0
    lines = out.splitlines()
    assert lines[0] == "%-33s %4s %6s %4s" % ("Name", "ID", "Weight", "Cap")
    assert lines[1] == "%-33s %4d %6d %4d" % ("dom1", 1, 256, 0)
    assert run(daemon, "sched-credit", "-d", "dom1", "-w", "512", "-c", "100")[0] == 0
    rc, out, _ = run(daemon, "sched-credit", "-d", "dom1")
    assert out.splitlines()[1].split()[-2:] == ["512", "100"]


@pytest.mark.parametrize("args,msg", [
    (["-d", "dom1", "-s"], "Specifying a cpupool or schedparam is not allowed with domain options."),
    (["-p", "Pool-0", "-w", "3"], "Specifying a cpupool or schedparam is not allowed with domain options."),
    (["-w", "300"], "Must specify a domain."),
    (["-t", "5000"], "Must specify schedparam to set schedule parameter values."),
])
def test_sched_credit_option_errors(daemon, args, msg):
    run(daemon, "create", "dom1")
    rc, _, err = run(daemon, "sched-credit", *args)
    assert rc == 1 and msg in err


@pytest.mark.parametrize("w,c", [("0", None), ("65536", None), (None, "-5"), (None, "900")])
def test_sched_credit_weight_cap_neg(daemon, w, c):
    run(daemon, "create", "dom1", "--slots", "2")
    args = ["sched-credit", "-d", "dom1"]
    if w:
        args += ["-w", w]
    if c:
        args += ["-c", c]
    rc, _, err = run(daemon, *args)
    assert rc != 0 and "failed" in err


def test_schedparam_get_set_and_ranges(daemon):
    rc, out, _ = run(daemon, "sched-credit", "-s")
    assert out.strip() == "Cpupool Pool-0: tslice=100us ratelimit=100us"
    assert run(daemon, "sched-credit", "-s", "-t", "5000", "-r", "1000")[0] == 0
    rc, out, _ = run(daemon, "sched-credit", "-s", "-p", "Pool-0")
    assert out.strip() == "Cpupool Pool-0: tslice=5000us ratelimit=1000us"
    rc, _, err = run(daemon, "sched-credit", "-s", "-t", "2000000")
    assert rc != 0 and "Time slice out of range" in err
    rc, _, err = run(daemon, "sched-credit", "-s", "-r", "50")
    assert rc != 0 and "Ratelimit out of range" in err
    rc, _, err = run(daemon, "sched-credit", "-s", "-t", "1000", "-r", "2000")
    assert rc != 0 and "Ratelimit cannot be greater than timeslice" in err
    rc, _, err = run(daemon, "sched-credit", "-s", "-p", "nope")
    assert rc != 0 and "unknown cpupool 'nope'" in err


def test_list_all_pools(daemon):
    run(daemon, "create", "a")
    run(daemon, "create", "b")
    rc, out, _ = run(daemon, "sched-credit")
    lines = out.splitlines()
    assert lines[0].startswith("Cpupool Pool-0: tslice=")
    assert [l.split()[0] for l in lines[2:]] == ["Domain-0", "a", "b"]


def test_pools_lifecycle(daemon):
    assert run(daemon, "pool-create", "p1", "--sched", "credit")[0] == 0
    assert run(daemon, "pool-gpu-remove", "Pool-0", "node:1")[0] == 0
    assert run(daemon, "pool-gpu-add", "p1", "node:1")[0] == 0
    rc, out, _ = run(daemon, "pool-list", "-c")
    assert "p1" in out
    run(daemon, "create", "t1")
    assert run(daemon, "pool-migrate", "t1", "p1")[0] == 0
    rc, out, _ = run(daemon, "sched-credit", "-p", "p1")
    assert "t1" in out and "Cpupool p1:" in out
    rc, _, err = run(daemon, "pool-destroy", "p1")
    assert rc != 0  # has a tenant
    assert run(daemon, "pool-migrate", "t1", "Pool-0")[0] == 0
    assert run(daemon, "pool-rename", "p1", "p2")[0] == 0
    assert run(daemon, "pool-destroy", "p2")[0] == 0


def test_xgmi_split(daemon):
    assert run(daemon, "pool-xgmi-split")[0] == 0
    rc, out, _ = run(daemon, "pool-list")
    assert "Pool-gpu0" in out and "Pool-gpu1" in out


def test_pause_unpause_pin_slotset_debugkeys(daemon):
    run(daemon, "create", "t", "--slots", "4")
    assert run(daemon, "pause", "t")[0] == 0
    rc, out, _ = run(daemon, "list")
    assert any(l.split()[0] == "t" and l.split()[3] == "p" for l in out.splitlines()[1:])
    assert run(daemon, "unpause", "t")[0] == 0
    assert run(daemon, "slot-pin", "t", "all", "0-3")[0] == 0
    assert run(daemon, "slot-set", "t", "2")[0] == 0
    rc, out, _ = run(daemon, "slot-list", "t")
    assert len(out.splitlines()) == 5
    rc, out, _ = run(daemon, "debug-keys", "z")
    assert "pmuinfo: INST_RETIRED=" in out and "sched_count:" in out
    rc, out, _ = run(daemon, "dmesg")
    assert "pmuinfo" in out
    rc, _, err = run(daemon, "pause", "nosuch")
    assert rc != 0 and "does not exist" in err


def test_snapshot_restore_roundtrip(daemon, tmp_path):
    run(daemon, "create", "keep", "--slots", "3", "--weight", "700", "--cap", "150")
    run(daemon, "pool-create", "px")
    run(daemon, "pool-gpu-remove", "Pool-0", "node:1")
    run(daemon, "pool-gpu-add", "px", "node:1")
    run(daemon, "pool-migrate", "keep", "px")
    snap = str(tmp_path / "s.json")
    assert run(daemon, "snapshot", snap)[0] == 0
    # a fresh daemon restores pools, tenants, weights and caps
    path = os.path.join(tempfile.mkdtemp(), "g2.sock")
    d2 = Daemon(path, gpus=[0, 1], nctx=2, sim=True, profile="reference", state_path=snap).start()
    try:
        rc, out, _ = run(d2, "sched-credit", "-p", "px")
        assert "keep" in out and " 700  150" in out
    finally:
        d2.stop()


def test_sched_credit2_and_sedf_verbs(daemon):
    """xl sched-credit2 / sched-sedf (xl_cmdimpl.c:4675-4726, 4932-5110):
    pools running those schedulers, list / show / set, formats and errors."""
    assert run(daemon, "pool-gpu-remove", "Pool-0", "node:1")[0] == 0
    assert run(daemon, "pool-create", "c2", "--sched", "credit2")[0] == 0
    assert run(daemon, "pool-gpu-add", "c2", "node:1")[0] == 0
    run(daemon, "create", "a", "--pool", "c2")
    rc, out, _ = run(daemon, "sched-credit2")
    assert rc == 0 and "Cpupool c2:" in out
    assert "%-33s %4s %6s" % ("Name", "ID", "Weight") in out
    assert run(daemon, "sched-credit2", "-d", "a", "-w", "768")[0] == 0
    rc, out, _ = run(daemon, "sched-credit2", "-d", "a")
    assert out.splitlines()[1].split()[-1] == "768"
    rc, _, err = run(daemon, "sched-credit2", "-p", "c2", "-w", "3")
    assert rc == 1 and "Specifying a cpupool is not allowed with other options." in err
    rc, _, err = run(daemon, "sched-credit2", "-w", "3")
    assert rc == 1 and "Must specify a domain." in err
    # sedf pool on a split of Pool-0
    assert run(daemon, "pool-create", "edf", "--sched", "sedf")[0] == 0
    assert run(daemon, "pool-gpu-remove", "Pool-0", "3")[0] == 0
    assert run(daemon, "pool-gpu-add", "edf", "3")[0] == 0
    run(daemon, "create", "rt", "--pool", "edf")
    assert run(daemon, "sched-sedf", "-d", "rt", "-p", "20", "-s", "5", "-e", "0")[0] == 0
    rc, out, _ = run(daemon, "sched-sedf", "-d", "rt")
    hdr = "%-33s %4s %6s %-6s %7s %5s %6s" % ("Name", "ID", "Period", "Slice", "Latency", "Extra", "Weight")
    assert out.splitlines()[0] == hdr
    assert out.splitlines()[1].split()[2:] == ["20", "5", "0", "0", "0"]
    rc, _, err = run(daemon, "sched-sedf", "-d", "rt", "-p", "20", "-s", "30")
    assert rc != 0 and "failed" in err  # slice > period
    rc, out, _ = run(daemon, "sched-sedf", "-c", "edf")
    assert "Cpupool edf:" in out and "rt" in out
    rc, _, err = run(daemon, "sched-sedf", "-c", "edf", "-p", "3")
    assert rc == 1 and "Specifying a cpupool is not allowed with other options." in err
    # the credit verbs do not apply to a credit2 / sedf tenant's pool
    rc, out, _ = run(daemon, "sched-credit")
    assert "Cpupool c2:" not in out and "Cpupool edf:" not in out
