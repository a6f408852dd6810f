"""Host-CPU tenants under the gpbs engine (config #1: "2 synthetic CPU-loop
tenants under the reference credit scheduler on host CPU").

The closest thing to the reference's own setting: partitions are host CPUs,
tenants are Linux processes, the PBS counter source is perf_event (the four
Perfctr-xen events, or software stand-ins where the host exposes no PMU) and
a partition switch is SIGSTOP/SIGCONT plus sched_setaffinity
(csrc/counters/perf_event.cpp, csrc/actuate/cpu_gate.cpp).

    host = CpuHost(host_cpus=[2], tslice_us=10000)
    a = host.spawn("a", [sys.executable, "-c", "while True: pass"], weight=256)
    b = host.spawn("b", [...], weight=512)
    host.start(); time.sleep(2); host.stop()
"""
from __future__ import annotations

import ctypes as C
import os
import signal
import subprocess
from typing import Dict, List, Optional

from .. import _native as N
from ..core.engine import Engine

PERF_MODES = {0: "none", 1: "hw", 2: "sw"}


def perf_mode() -> str:
    return PERF_MODES.get(N.load_core().gpbs_perf_available(), "none")


def proc_cpu_seconds(pid: int) -> float:
    """utime + stime of a process (and its reaped children) from /proc."""
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    tck = os.sysconf("SC_CLK_TCK")
    return (int(fields[11]) + int(fields[12])) / tck


class CpuHost:
    def __init__(self, host_cpus: List[int], sched: str = "credit", tslice_us: int = 10000,
                 ratelimit_us: int = 1000, **engine_kw):
        self.lib = N.load_core()
        engine_kw.setdefault("quantum_align_us", 0)
        self.engine = Engine(sched=sched, **engine_kw)
        self.host_cpus = list(host_cpus)
        self.parts = []
        for i, _ in enumerate(self.host_cpus):
            p = self.engine.partition_add(0, i)
            self.engine.pool_assign(0, p)
            self.parts.append(p)
        self.engine.tenant_create("Domain-0", nslots=1)
        self.engine.sched_params_set(0, tslice_us, ratelimit_us)
        self.gate = self.lib.gpbs_gate_create(b"signal")
        if not self.gate:
            raise RuntimeError("cannot create CPU gate")
        self.gate = C.c_void_p(self.gate)
        h = self.lib.gpbs_cpu_backend_create(self.engine.h, self.gate)
        if not h:
            raise RuntimeError("cannot attach CPU backend")
        self.backend = C.c_void_p(h)
        for p, cpu in zip(self.parts, self.host_cpus):
            self.lib.gpbs_cpu_backend_map(self.backend, p, cpu)
        self.procs: Dict[int, subprocess.Popen] = {}
        self.counters_live: Dict[int, bool] = {}
        self.started = False

    def spawn(self, name: str, argv: List[str], slots: int = 1, weight: int = -1, cap: int = -1) -> int:
        t = self.engine.tenant_create(name, nslots=slots, weight=weight, cap=cap)
        p = subprocess.Popen(argv, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                             start_new_session=True)
        self.procs[t] = p
        rc = self.lib.gpbs_cpu_backend_add(self.backend, t, p.pid)
        self.counters_live[t] = rc == 0
        self.engine.wake(t)
        return t

    def start(self):
        self.engine.start()
        self.started = True
        return self

    def cpu_seconds(self) -> Dict[int, float]:
        return {t: proc_cpu_seconds(p.pid) for t, p in self.procs.items() if p.poll() is None}

    def gate_stats(self):
        s, pins = C.c_uint64(0), C.c_uint64(0)
        self.lib.gpbs_gate_stats(self.gate, C.byref(s), C.byref(pins))
        return {"signals": s.value, "pins": pins.value}

    def stop(self):
        if self.started:
            self.engine.stop()
            self.started = False
        if self.backend:
            self.lib.gpbs_cpu_backend_destroy(self.backend)
            self.backend = None
        if self.gate:
            self.lib.gpbs_gate_destroy(self.gate)  # SIGCONT everyone
            self.gate = None
        for p in self.procs.values():  # exact children only
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait(timeout=10)

    def close(self):
        self.stop()
        self.engine.close()
