"""Config #1: synthetic CPU-loop tenants under the PBS credit scheduler on the
host CPU -- perf_event counters (hardware events, or the software stand-ins a
PMU-less VM offers) and SIGSTOP/SIGCONT + sched_setaffinity actuation."""
import os
import sys
import time

import pytest

from pbs_amd import _native as N
from pbs_amd.runtime.cpu import CpuHost, perf_mode

LOOP = [sys.executable, "-c", "while True: pass"]


def test_perf_counters_count_this_process():
    lib = N.load_core()
    if perf_mode() == "none":
        pytest.skip("perf_event_open unavailable")
    import ctypes as C
    h = lib.gpbs_perf_open(0, -1)
    assert h
    a = (C.c_uint64 * 4)()
    b = (C.c_uint64 * 4)()
    lib.gpbs_perf_read(h, a)
    x = 0
    for i in range(300000):
        x += i
    lib.gpbs_perf_read(h, b)
    lib.gpbs_perf_close(h)
    assert b[0] > a[0] and b[1] > a[1]


def _cpu():
    cpus = sorted(os.sched_getaffinity(0))
    return cpus[-1]


def test_two_cpu_loop_tenants_share_one_cpu_by_weight():
    host = CpuHost([_cpu()], tslice_us=10000, ratelimit_us=1000)
    try:
        a = host.spawn("loop-a", LOOP, weight=256)
        b = host.spawn("loop-b", LOOP, weight=512)
        time.sleep(0.3)  # interpreter start-up while stopped/gated
        host.start()
        time.sleep(0.5)
        c0 = host.cpu_seconds()
        r0 = {t: host.engine.tenant_info(t).run_ns for t in (a, b)}
        time.sleep(2.0)
        c1 = host.cpu_seconds()
        r1 = {t: host.engine.tenant_info(t).run_ns for t in (a, b)}
        used = {t: c1[t] - c0[t] for t in (a, b)}
        sched = {t: (r1[t] - r0[t]) / 1e9 for t in (a, b)}
        # the engine's accounting: 1:2 by weight on one partition
        assert 1.5 < sched[b] / max(sched[a], 1e-9) < 2.7, sched
        # what the processes actually got from the kernel follows it
        assert used[a] > 0.2 and used[b] > 0.2, used
        assert 1.4 < used[b] / used[a] < 2.8, used
        # never both at once on the single CPU (gated by SIGSTOP)
        assert used[a] + used[b] < 2.0 * 1.15, used
        st = host.gate_stats()
        assert st["signals"] > 20 and st["pins"] > 0
        if perf_mode() != "none":
            assert host.engine.slot_info(host.engine.slot_id(a, 0))["pmc"][1] > 0
    finally:
        host.close()
