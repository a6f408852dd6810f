"""Host-side race/memory checking (S12, the reference's debug=y latch and
lockdep analog): the native engine built with AddressSanitizer and with
ThreadSanitizer runs a credit workload -- including the real-time dispatcher
thread against concurrent API calls, the control-page bridge with its vPMU
mirror, and the gang shm transport through a re-formation -- with no
sanitizer report.  CPU only; GPU sanitizers are not used."""
import os
import subprocess
import sys

import pytest

from pbs_amd import build

WORKLOAD = r"""
import os, threading, time
from pbs_amd.core.engine import Engine
# simulated clock: credit, PBS adaptation, pools, pause, pin, trace, dumps
e = Engine(sim_clock=True, partitions=[(0, x, c) for x in range(4) for c in range(2)], coschedule=3)
e.tenant_create("Domain-0", nslots=1)
a = e.tenant_create("a", nslots=4); b = e.tenant_create("b", nslots=4, weight=512, cap=300)
e.wake(a); e.wake(b)
for i in range(2000):
    e.advance(e.now() + 50_000)
    if i % 100 == 0:
        e.pause(a); e.advance(e.now() + 10_000); e.unpause(a)
        e.pin(b, i % 4, [i % 8, (i + 3) % 8])
e.debug_keys("rqz"); e.trace(from_start=True)
assert e.check() == "", e.check()
# S4 pools side by side: credit2 and sedf, tenants moved between them
for name, sched, parts in (("c2", "credit2", (4, 5)), ("edf", "sedf", (6, 7))):
    p = e.pool_create(name, sched)
    for q in parts:
        e.pool_unassign(0, q); e.pool_assign(p, q)
c = e.tenant_create("c", nslots=2, pool=e.pool_find("c2")); d = e.tenant_create("d", nslots=2, pool=e.pool_find("edf"))
e.sched_ext_set(d, period_us=2000, slice_us=500, latency_us=200, extratime=1)
e.wake(c); e.wake(d)
for i in range(1500):
    e.advance(e.now() + 50_000)
    if i % 200 == 0:
        e.block(d); e.advance(e.now() + 5_000_000); e.wake(d)
        e.tenant_move(c, e.pool_find("edf") if i % 400 == 0 else e.pool_find("c2"))
e.debug_keys("rqz")
assert e.check() == "", e.check()
e.close()
# real clock: dispatcher thread vs. concurrent wake/block/adjust from 4 threads
r = Engine(partitions=[(0, x) for x in range(8)])
r.tenant_create("Domain-0", nslots=1)
ts = [r.tenant_create(f"t{i}", nslots=4) for i in range(4)]
r.start()
def hammer(t):
    for k in range(300):
        r.wake(t); r.block(t) if k % 3 == 0 else None
        r.sched_credit_set(t, weight=128 + k % 512)
        r.tenant_info(t)
th = [threading.Thread(target=hammer, args=(t,)) for t in ts]
[x.start() for x in th]; [x.join() for x in th]
# control-page bridge thread vs. a tenant writing its page
from pbs_amd import _native as N
import ctypes as C
lib = N.load_core()
ctl = C.c_void_p(lib.gpbs_ctl_create(b"san-%d" % os.getpid(), 4))
lib.gpbs_ctl_bind(ctl, r.h)
lib.gpbs_ctl_assign(ctl, 0, ts[0])
c4 = (C.c_uint64 * 4)(1, 2, 3, 4)
for k in range(400):
    lib.gpbs_ctl_set_work(ctl, 0, k % 2)
    lib.gpbs_ctl_report(ctl, 0, 1000 + k, 1 + k % 3, 0)
    lib.gpbs_ctl_heartbeat(ctl, 0, k, k)
    c4[0] += 1000; lib.gpbs_ctl_set_counters(ctl, 0, c4)
    lib.gpbs_ctl_wait_gate(ctl, 0, 10000)
    v4, mr, tsl, cl, ph, sq = (C.c_uint64 * 4)(), C.c_uint64(), C.c_uint32(), C.c_int32(), C.c_uint32(), C.c_uint32()
    lib.gpbs_ctl_read_vpmu(ctl, 0, v4, C.byref(mr), C.byref(tsl), C.byref(cl), C.byref(ph), C.byref(sq))
time.sleep(0.05)
lib.gpbs_ctl_close(ctl, 1)
# gang shm transport: three ranks as threads; rank 2 stops at epoch 20 and
# the other two re-form the gang without it and keep exchanging
gname = b"san-gang-%d" % os.getpid()
gh = [C.c_void_p(lib.gpbs_gang_shm_open(gname, k, 3, 4)) for k in range(3)]
res = {}
def grank(k):
    src, out = (C.c_int64 * 4)(k, k, k, k), (C.c_int64 * 12)()
    ep, done, reforms = 1, 0, 0
    while done < 60:
        if k == 2 and ep == 20:
            break
        # generous deadline / join window: ASan + the GIL on a loaded host
        # (pytest -n) must not look like a second failure
        rc = lib.gpbs_gang_shm_allgather(gh[k], ep, src, out, time.monotonic_ns() + 1_000_000_000)
        if rc in (-110, -117):  # deadline missed, or a peer already claimed the re-formation
            m, base = C.c_uint64(), C.c_uint64()
            rc = lib.gpbs_gang_shm_reform(gh[k], 2_000_000_000, time.monotonic_ns() + 6_000_000_000, C.byref(m),
                                          C.byref(base))
            assert rc == 0 and m.value == 3, (k, rc, m.value)
            ep, reforms = base.value, reforms + 1
            continue
        assert rc == 0, (k, rc)
        ep += 1
        done += 1
    res[k] = (done, reforms)
gt = [threading.Thread(target=grank, args=(k,)) for k in range(3)]
[x.start() for x in gt]; [x.join() for x in gt]
assert res[0] == (60, 1) and res[1] == (60, 1), res
for h in gh[::-1]:
    lib.gpbs_gang_shm_close(h)
# native gang coordinator threads (csrc/comm/gang_coord.cpp): three ranks'
# engines in one process, their C++ epoch loops racing stats/history readers
from pbs_amd.parallel.gang import GangCoordinator
engs, gcs = [], []
for k in range(3):
    ek = Engine(partitions=[(k, x) for x in range(2)], quantum_align_us=0)
    ek.tenant_create("Domain-0", nslots=1)
    tk = ek.tenant_create("coll", nslots=2)
    ek.start(); ek.wake(tk)
    engs.append(ek)
    gcs.append(GangCoordinator(ek, None, [tk], epoch_ms=1.0, share=0.5, transport="shm",
                               shm_name="san-gc-%d" % os.getpid(), rank=k, world=3, metric_tenants=[tk],
                               metric_every=1, deadline_ms=2000.0, native=True).start())
for _ in range(40):
    [(g.stats(), g.history, g.node_metrics) for g in gcs]
    time.sleep(0.005)
[g.stop() for g in gcs]
assert all(g.stats()["epochs"] >= 10 and g.stats()["timeouts"] == 0 for g in gcs), [g.stats() for g in gcs]
[(ek.stop(), ek.close()) for ek in engs]
r.stop(); r.close()
print("OK")
"""


def _run(kind):
    lib = build.build_core(sanitize=kind)
    rt = subprocess.run(["g++", f"-print-file-name=lib{'a' if kind == 'address' else 't'}san.so"],
                        capture_output=True, text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip(f"lib{kind} runtime not found")
    env = dict(os.environ, GPBS_CORE_LIB=lib, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0",
               TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=1")
    env.pop("GPBS_FAULT", None)
    out = subprocess.run([sys.executable, "-c", WORKLOAD], env=env, capture_output=True, text=True, timeout=600,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return out


def test_engine_under_address_sanitizer():
    out = _run("address")
    assert "ERROR: AddressSanitizer" not in out.stderr, out.stderr[-4000:]
    assert out.returncode == 0 and "OK" in out.stdout, out.stderr[-4000:]


def test_engine_under_thread_sanitizer():
    out = _run("thread")
    # python itself is not instrumented: only reports that involve libgpbs matter
    reports = [blk for blk in out.stderr.split("==================") if "WARNING: ThreadSanitizer" in blk]
    ours = [blk for blk in reports if "libgpbs" in blk]
    assert not ours, ours[0][-4000:]
    assert "OK" in out.stdout, out.stderr[-4000:]
