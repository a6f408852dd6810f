"""gpbsd lifecycle and multi-GPU actuation (CPU, simulated clock).

* Two daemons started and stopped in one process, with a tenant that
  registered and then exited (its pid stays in the reaper's table), must not
  crash: the reaper is joined before the engine is torn down, and a closed
  engine raises instead of handing NULL to C (round-1 config #5 core dump).
* A daemon spanning two GPUs drives the partition tables of BOTH GPUs: one
  backend per GPU on the engine's backend mux, switch events routed by
  partition range, counter deltas summed node-wide.
"""
import ctypes as C
import os
import subprocess
import sys
import tempfile
import time

import pytest

from pbs_amd import _native as N
from pbs_amd.core.errors import GpbsError
from pbs_amd.runtime.daemon import Daemon


def _sock():
    return os.path.join(tempfile.mkdtemp(), "gpbsd.sock")


def test_two_daemons_in_one_process_with_exited_tenant():
    for round_ in range(2):
        d = Daemon(_sock(), gpus=[0], nctx=2, sim=False).start(reaper_s=0.01)
        child = subprocess.Popen([sys.executable, "-c", "pass"])
        child.wait()
        # registered, then "unregistered" without destroy: register() tracks
        # its pid (a tenant_find here would race the 10 ms reaper)
        r = d.register(name=f"llm{round_}", slots=4, pid=child.pid)
        assert r["tenant"] >= 0
        time.sleep(0.05)  # the reaper runs concurrently with the stop below
        d.stop()
        assert d.engine.closed
        with pytest.raises(GpbsError):
            d.engine.tenant_info(0)


class FakeGpu:
    """A per-GPU backend: records the partitions it is told to switch and
    reports fixed per-tick counter deltas (INST = base, MISS = base/10)."""

    def __init__(self, engine, part_lo, nparts, base):
        self.lo, self.hi, self.base = part_lo, part_lo + nparts, base
        self.switched = []
        self.flushes = 0
        self.act = N.ActuatorOps()
        self.act.on_switch = N.ACT_ON_SWITCH(self._sw)
        self.act.on_flush = N.ACT_ON_FLUSH(self._fl)
        self.ctr = N.CounterOps()
        self.ctr.tenant_deltas = N.COUNTER_TENANT_DELTAS(self._deltas)
        engine.mux_add(self.lo, self.hi, self.act, self.ctr)

    def _sw(self, user, part, prev, nxt, slot, q, now):
        self.switched.append(part)

    def _fl(self, user, now):
        self.flushes += 1

    def _deltas(self, user, n, ids, out):
        for k in range(n):
            out[4 * k + 0] = self.base
            out[4 * k + 1] = self.base * 2
            out[4 * k + 2] = self.base // 5
            out[4 * k + 3] = self.base // 10
        return 0


def test_daemon_drives_the_partition_tables_of_every_gpu():
    d = Daemon(_sock(), gpus=[0, 1], nctx=2, sim=True)
    per_gpu = 8 * 2
    fakes = {}

    def factory(gpu, part_lo):
        fakes[gpu] = FakeGpu(d.engine, part_lo, per_gpu, 1000 * (gpu + 1))
        return fakes[gpu]

    d.attach_backends(factory)
    d.start()
    assert d.engine.mux_count() == 2
    t = d.create(name="wide", slots=32)
    d.engine.wake(t)
    for _ in range(50):
        d.advance_us(200)
    f0, f1 = fakes[0], fakes[1]
    assert f0.switched and f1.switched
    assert all(f0.lo <= p < f0.hi for p in f0.switched)
    assert all(f1.lo <= p < f1.hi for p in f1.switched)
    assert {p for p in f0.switched} | {p for p in f1.switched} == set(range(2 * per_gpu))
    assert f0.flushes > 0 and f1.flushes > 0
    # node-wide counters: the metric tick sums both GPUs' deltas
    pmc = d.engine.tenant_info(t).pmc
    assert pmc[0] == 1000 + 2000 and pmc[3] == 100 + 200, pmc
    # overlapping ranges are refused
    with pytest.raises(GpbsError):
        FakeGpu(d.engine, 4, 8, 1)
    d.stop()
    assert d.engine.closed
