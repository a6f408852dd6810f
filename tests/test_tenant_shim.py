"""Tenant shim <-> gpbsd over the shared-memory control plane, multi-process
(CPU only): registration, launch gate, wait/hold/request reports (P2/P8/P7),
published counters reaching the scheduler's vPMU (C10) and its mirror back on
the tenant's page (S2/K13), heartbeat, and the
reaper's failure detection (S13) when a tenant process dies."""
import multiprocessing as mp
import os
import tempfile
import time

from pbs_amd.runtime.daemon import Daemon
from pbs_amd.runtime.tenant import half_cu_words, run_synthetic


def test_half_cu_words_cover_exactly_the_owned_halves():
    w = half_cu_words([(0, 0), (3, 1)])
    bits = [b for b in range(256) if (w[b // 32] >> (b % 32)) & 1]
    assert len(bits) == 2 * 16  # 16 CUs per half-XCD
    assert all((b % 8, ((b // 8) % 4) >> 1) in {(0, 0), (3, 1)} for b in bits)
    full = half_cu_words([(x, h) for x in range(8) for h in (0, 1)])
    assert full == [0xFFFFFFFF] * 8


def test_two_tenant_processes_share_the_gpu_through_the_control_plane():
    path = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
    # no reaper here: the tenants unregister without destroy and exit; their
    # engine state is inspected afterwards (the reaper has its own test)
    d = Daemon(path, gpus=[0], nctx=2, sim=False, profile="mi355x").start(reaper_s=0)
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=run_synthetic, args=(n, path, 1.5, q)) for n in ("alpha", "beta")]
        for p in ps:
            p.start()
        res = {}
        for _ in ps:
            r = q.get(timeout=60)
            res[r["name"]] = r
        for p in ps:
            p.join(timeout=30)
            assert p.exitcode == 0
        e = d.engine
        for name in ("alpha", "beta"):
            r = res[name]
            assert r["opens"] > 10 and r["loops"] > 10, r
            info = e.tenant_info(r["tenant"])
            assert info.run_ns > 0, name
            # published counters reached the scheduler (slot-0 vPMU mirror)
            assert e.slot_info(e.slot_id(r["tenant"], 0))["pmc"][0] > 0
            # ... and came back through the scheduler's metric path into the
            # tenant's own vPMU mirror (seqlock read of its control page):
            # cumulative counts, miss rate = misses per 100k instructions
            v = r["vpmu"]
            assert v["updates"] > 10 and v["inst"] > 0, v
            assert v["inst"] <= r["declared"][0] and v["inst"] >= 0.5 * r["declared"][0], (v, r["declared"])
            assert v["l2_misses"] <= r["declared"][3]
            want = r["declared"][3] * 100000 / r["declared"][0]
            assert abs(v["l2_misses"] * 100000 / v["inst"] - want) <= 0.05 * want, (v, want)
            assert v["tslice_us"] > 0
        z = e.debug_keys("z")
        assert "waits: n=" in z and "holds: n=" in z and "pending_requests=" in z
        assert e.perfc()["report_rx"] > 0
    finally:
        d.stop()


def test_reaper_destroys_tenant_whose_process_died():
    path = os.path.join(tempfile.mkdtemp(), "gpbsd.sock")
    d = Daemon(path, gpus=[0], nctx=2, sim=False, profile="mi355x").start(reaper_s=0.05)
    try:
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=run_synthetic, args=("doomed", path, 0.3), kwargs={"crash": True})
        p.start()
        p.join(timeout=60)
        deadline = time.monotonic() + 10
        while "doomed" not in d.reaped and time.monotonic() < deadline:
            time.sleep(0.05)
        assert "doomed" in d.reaped
        names = [d.engine.tenant_info(t).name for t in d.engine.tenants()]
        assert "doomed" not in names
        assert not d.pages  # page released
    finally:
        d.stop()


def test_se_mode_stream_uses_one_masked_queue_on_the_class_home_half(monkeypatch):
    """SE mode: a shim tenant launches on ONE CU-masked queue for its life --
    the home half of its class (compute {0,1}, memory {2,3}); a transitional
    layout on the other class's half, an unclassified tenant and a later
    class flip run on the unmasked stream (two processes that each moved
    their kernels between two masked queues collapsed together:
    profiles/llm5/config5_r3g_swap_nohwc.json)."""
    import torch

    from pbs_amd.ops import kernels as K
    from pbs_amd.runtime.tenant import TenantClient, se_cu_words
    made = []
    monkeypatch.setattr(K, "cumask_stream", lambda words, device=0: made.append(tuple(words)) or len(made))
    monkeypatch.setattr(torch.cuda, "ExternalStream", lambda h: ("masked", h))
    monkeypatch.setattr(torch.cuda, "current_stream", lambda: "unmasked")
    t = object.__new__(TenantClient)
    t.se_mode, t.spatial, t.gpu, t.one_queue, t._home, t._streams = True, True, 0, True, None, {}
    t.queue_probe, t._probers = 0, {}
    cls = {"v": -1}
    t.vpmu = lambda: {"class": cls["v"]}
    lo = [(x, c) for x in range(8) for c in (0, 1)]
    hi = [(x, c) for x in range(8) for c in (2, 3)]
    assert t.stream(lo) == "unmasked"          # not classified yet
    cls["v"] = 1                                # memory class: home {2,3}
    assert t.stream(lo) == "unmasked"          # transitional layout on the compute half
    assert t.stream(hi) == ("masked", 1) and made == [tuple(se_cu_words((2, 3)))]
    assert t.stream(lo + hi) == "unmasked"     # a set across both halves
    cls["v"] = 0                                # class flip: its home would be {0,1}
    assert t.stream(lo) == "unmasked" and len(made) == 1   # never a second masked queue
    t.one_queue, t._home = False, None          # pre-fix behaviour: any owned half gets its queue
    assert t.stream(lo) == ("masked", 2) and len(made) == 2


def test_queue_prober_explores_exploits_and_reexplores_on_drift():
    """Per SE half, K masked queues: explore each, exploit the fastest,
    explore again when the chosen one's slices drift above 1.6x its explored
    median (the head-of-line stall of a queue mapped onto a busy pipe)."""
    from pbs_amd.runtime.tenant import QueueProber
    speed = {0: 16.5, 1: 2.5, 2: 16.4}   # ms per slice on each queue
    p = QueueProber(3, explore=4, keep=3, drift=1.6, cooldown=10)
    seen = []
    for _ in range(9):
        seen.append(p.current())
        p.record(speed[p.current()])
    # queue 2 is left after one slice: 16.4 ms > 2 x queue 1's 2.5 ms
    assert seen == [0] * 4 + [1] * 4 + [2] and not p.exploring and p.current() == 1
    for _ in range(50):                  # steady: stays on the fast queue
        p.record(speed[p.current()])
    assert p.current() == 1 and p.explorations == 1
    speed[1] = 17.0                       # its pipe became busy: re-explore, queue 2 is now the fast one
    speed[2] = 2.6
    for _ in range(40):
        p.record(speed[p.current()])
    assert p.current() == 2 and p.explorations == 2
    # a re-exploration that picks the same queue backs the cooldown off
    c = p.cooldown
    speed[0] = speed[1] = 30.0
    speed[2] = 5.0                        # everything slower (more load), queue 2 still best
    for _ in range(200):
        p.record(speed[p.current()])
    assert p.current() == 2 and p.cooldown > c


def test_co_resident_stream_probes_k_unmasked_queues(monkeypatch):
    """Co-resident contexts (no CU mask): with queue_probe=K the shim keeps K
    streams of the tenant's priority and launches on the one QueueProber
    chose (two unmasked queues on one pipe block each other too: `none` is
    bimodal in config #5)."""
    import torch

    from pbs_amd.runtime.tenant import TenantClient
    made = []
    monkeypatch.setattr(torch.cuda, "Stream", lambda device=0, priority=0: made.append(priority) or f"q{len(made)}")
    t = object.__new__(TenantClient)
    t.se_mode, t.spatial, t.gpu, t.one_queue, t._home, t._streams = False, False, 0, False, None, {}
    t.queue_probe, t._probers, t.priority = 3, {}, 1
    parts = [(x, c) for x in range(8) for c in (0, 1)]
    assert t.stream(parts) == "q1" and made == [-1, -1, -1]
    pr = t._probers[("p", 0, 1)]
    for ms in (9.0, 9.0, 9.0, 9.0, 2.0, 2.0, 2.0, 2.0, 9.5):
        pr.record(ms)
    assert t.stream(parts) == "q2" and len(made) == 3


def test_slice_orders_queue_changes_and_times_gpu_work(monkeypatch):
    """when consecutive slices land on different queues (the
    prober rotating same-mask queues, or a layout change) the new queue
    waits for the old one's work, and a probed slice is timed after its
    stream synchronises (not at launch)."""
    import contextlib

    import torch

    from pbs_amd.runtime.tenant import QueueProber, TenantClient
    log = []

    class FakeStream:
        def __init__(self, name):
            self.name = name

        def __eq__(self, o):
            return isinstance(o, FakeStream) and o.name == self.name

        def __hash__(self):
            return hash(self.name)

        def wait_stream(self, o):
            log.append(("wait", self.name, o.name))

        def synchronize(self):
            log.append(("sync", self.name))

    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    t = object.__new__(TenantClient)
    t._last_stream, t._progress, t._probe_key = None, 0, None
    t.busy = lambda: None
    t.gate = lambda timeout_s=10.0: True
    t.report_wait = lambda ns: None
    pr = QueueProber(3, explore=1)
    t._probers = {("se", 2, 3): pr}
    qs = [FakeStream(f"q{i}") for i in range(3)]

    def stream(owned=None):
        t._probe_key = ("se", 2, 3)
        return qs[pr.current()]
    t.stream = stream
    for _ in range(3):
        with t.slice():
            log.append(("body", qs[pr.current()].name))
    # q0 -> q1 -> q2: each new queue waits for the previous one; every probed slice syncs
    assert ("wait", "q1", "q0") in log and ("wait", "q2", "q1") in log
    assert [e for e in log if e[0] == "sync"] == [("sync", "q0"), ("sync", "q1"), ("sync", "q2")]
    assert log.index(("wait", "q1", "q0")) < log.index(("body", "q1"))
    n_wait = sum(1 for e in log if e[0] == "wait")
    t.stream = lambda owned=None: qs[2]
    with t.slice():  # same queue again: no cross-queue wait
        pass
    assert sum(1 for e in log if e[0] == "wait") == n_wait


def test_queue_prober_started_on_a_known_winner_skips_exploration():
    """A prober started on a known-fast queue (start / ref_ms) exploits it at
    once and explores only if its first slices drift above 1.6x that time."""
    from pbs_amd.runtime.tenant import QueueProber
    mem = {"idx": 2, "ref_ms": 5.0}
    # remembered queue still fast: never explores
    p = QueueProber(3, start=mem["idx"], ref_ms=mem["ref_ms"])
    seen = []
    for _ in range(20):
        seen.append(p.current())
        p.record(5.2)
    assert seen == [2] * 20 and p.explorations == 0 and p.state() == {"idx": 2, "ref_ms": 5.0}
    # remembered queue now stalled (another mapping this run): explore after the probation
    speed = {0: 5.1, 1: 17.0, 2: 16.5}
    p = QueueProber(3, explore=2, start=2, ref_ms=5.0)
    seen = []
    for _ in range(12):
        seen.append(p.current())
        p.record(speed[p.current()])
    assert seen[:3] == [2, 2, 2] and p.explorations == 1 and p.current() == 0
    assert p.state()["idx"] == 0


def test_prober_leaves_a_stalled_queue_without_waiting_for_the_cooldown():
    """A queue that starts stalling mid-run (3x its explored time) is left
    within a few slices, not after the cooldown; a mild drift still waits."""
    from pbs_amd.runtime.tenant import QueueProber
    p = QueueProber(3, explore=2, keep=2, cooldown=100)
    for ms in (5.0, 5.0, 9.0, 9.0, 6.0, 6.0):  # queue 0 fastest
        p.record(ms)
    assert not p.exploring and p.current() == 0
    for _ in range(20):  # mild drift (1.3x): stays
        p.record(6.5)
    assert not p.exploring
    n = 0
    while not p.exploring and n < 50:  # stall (3x)
        p.record(15.0)
        n += 1
    assert p.exploring and n <= 8, n
