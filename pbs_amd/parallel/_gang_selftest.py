"""Worker for the multi-process gang test (tests/test_gang.py): one rank per
"GPU", a real-time engine per rank, a bandwidth hog plus a gang tenant, and a
GangCoordinator over gloo.  Samples which tenant runs on each partition and
returns per-epoch occupancy of the gang tenant."""
from __future__ import annotations

import os
import time


def worker(rank: int, world: int, port: int, q, seconds: float = 0.8, epoch_ms: float = 6.0):
    import torch.distributed as dist

    from pbs_amd.core.engine import Engine
    from pbs_amd.parallel.gang import FAVOUR, GangCoordinator
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(partitions=[(rank, x) for x in range(4)], quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    e.sched_params_set(0, 1000, 100)
    hog = e.tenant_create("hog", nslots=4)
    coll = e.tenant_create("coll", nslots=4)
    e.start()
    e.wake(hog)
    e.wake(coll)
    dist.barrier()
    g = GangCoordinator(e, None, [coll], epoch_ms=epoch_ms, share=0.5).start()
    samples = []  # (epoch, state, fraction of partitions running coll)
    t_end = time.monotonic() + seconds
    while time.monotonic() < t_end:
        ep = g.epoch - 1
        st = g.state.get(coll, 0)
        running = 0
        for k in range(4):
            if e.slot_info(e.slot_id(coll, k))["is_running"]:
                running += 1
        ep2 = g.epoch - 1
        if ep == ep2 and ep >= 0:
            samples.append((ep, st, running / 4.0))
        time.sleep(0.0005)
    g.stop()
    st = g.stats()
    e.stop()
    q.put({"rank": rank, "samples": samples, "history": g.history, "stats": st, "favour": FAVOUR})
    dist.destroy_process_group()


def atc_worker(rank: int, world: int, port: int, q, epoch_ms: float = 5.0, periods: int = 40):
    """Node-level sync over the gang epochs: an ATC pool per rank (rank 0's
    tenant reports heavy spin-waits, so its local minimum slice is small) and
    per-rank counters; returns each rank's applied slice and node metrics.

    Deterministic under any host load: the engines run on a simulated clock,
    so every ATC apply happens in the load phase below and the local minima
    are frozen before the gang starts; the check then waits for named gang
    epochs (three exchanges after the start on every rank), not wall time."""
    import torch.distributed as dist

    from pbs_amd.core.engine import Engine
    from pbs_amd.parallel.gang import GangCoordinator
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(sched="atc", sim_clock=True, partitions=[(rank, x) for x in range(2)], quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    t = e.tenant_create("t", nslots=2)
    e.wake(t)
    period_ns = 21_000_000  # the ATC apply period
    for k in range(1, periods + 1):
        if rank == 0:
            e.report_wait(t, 200_000)  # heavy lock-holder preemption symptom
        for s in range(2):  # modeled counters: rank r retires (r+1) x 1e6 instructions per ms
            e.set_pmc(e.slot_id(t, s), [k * (rank + 1) * 500_000, k * 1_000_000, k * 1000, k * 100 * (rank + 1)])
        e.advance(e.now() + period_ns)
    # one more count and up to the first metric tick after it: the period's
    # deltas (what the gang SUM-reduces) are non-zero when the clock stops
    k = periods + 1
    for s in range(2):
        e.set_pmc(e.slot_id(t, s), [k * (rank + 1) * 500_000, k * 1_000_000, k * 1000, k * 100 * (rank + 1)])
    for _ in range(100):
        e.advance(e.now() + 50_000)
        if e.tenant_info(t).pmc[0]:
            break
    local = e.atc_sync(0, 0)  # frozen from here on: the clock no longer moves
    dist.barrier()
    g = GangCoordinator(e, None, [t], epoch_ms=epoch_ms, share=0.0, atc_pool=0, metric_tenants=[t],
                        metric_every=1).start()
    t_end = time.monotonic() + 30.0
    while (g.metric_syncs < 3 or g.atc_global_us <= 0) and time.monotonic() < t_end:
        time.sleep(0.002)
    syncs = g.metric_syncs
    node = dict(g.node_metrics.get(t, {}))
    # one more named epoch past the one read, so both ranks' applies are in
    target = g.epoch + 2
    while g.epoch < target and time.monotonic() < t_end:
        time.sleep(0.002)
    g.stop()
    info = e.tenant_info(t)
    q.put({"rank": rank, "local_min": local, "tslice": info.tslice_us, "stats": g.stats(),
           "node": node, "syncs_seen": syncs})
    dist.destroy_process_group()


def metrics_sum_worker(rank: int, world: int, port: int, q, transport: str = "dist", shm_name: str = "",
                       epoch_ms: float = 4.0):
    """C11 exactness: each rank's engine (simulated clock, frozen after one
    metric period) holds fixed per-tenant counter deltas; after a few gang
    epochs every rank's node_metrics must be exactly the SUM of every rank's
    deltas for each metric tenant."""
    import torch.distributed as dist

    from pbs_amd.core.engine import Engine
    from pbs_amd.parallel.gang import GangCoordinator
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(sim_clock=True, partitions=[(rank, x) for x in range(2)], quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    ts = [e.tenant_create(n, nslots=2) for n in ("a", "b")]
    for t in ts:
        e.wake(t)
    e.advance(e.now() + 100_000)
    for i, t in enumerate(ts):  # rank- and tenant-specific counts, charged to slot 0
        e.set_pmc(e.slot_id(t, 0), [(rank + 1) * 1_000_003 * (i + 1), (rank + 7) * 999 * (i + 2),
                                    (rank + 3) * 77 * (i + 1), (rank + 2) * 13 * (i + 3)])
    for _ in range(100):  # up to the first metric tick after the counts: the deltas land in tenant_info().pmc
        e.advance(e.now() + 50_000)
        if all(e.tenant_info(t).pmc[0] for t in ts):
            break
    local = {t: list(e.tenant_info(t).pmc) for t in ts}
    g = GangCoordinator(e, None, [], epoch_ms=epoch_ms, share=0.0, metric_tenants=ts, metric_every=1,
                        transport=transport, rank=rank, world=world, shm_name=shm_name).start()
    t_end = time.monotonic() + 5.0
    while g.metric_syncs < 3 and time.monotonic() < t_end:
        time.sleep(0.005)
    node = {t: dict(g.node_metrics.get(t, {})) for t in ts}
    g.stop()
    totals = {t: dict(g.node_totals.get(t, {})) for t in ts}
    q.put({"rank": rank, "local": local, "node": node, "totals": totals, "syncs": g.metric_syncs,
           "still": {t: list(e.tenant_info(t).pmc) for t in ts},
           "vpmu": {t: list(e.tenant_vpmu(t).values()) for t in ts}})
    dist.destroy_process_group()


def hang_worker(rank: int, world: int, port: int, q, transport: str, shm_name: str, hang_rank: int,
                hang_ms: int = 1500, deadline_ms: float = 200.0, reform: bool = False):
    """One rank of the gang-deadline test: `hang_rank` stalls `hang_ms` before
    its first exchange (GPBS_FAULT rank_hang); the others must time out
    within the deadline, trace GANG_TIMEOUT and keep scheduling locally."""
    import torch.distributed as dist

    from pbs_amd.core.engine import Engine
    from pbs_amd.parallel.gang import GangCoordinator
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(partitions=[(rank, x) for x in range(2)], quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    coll = e.tenant_create("coll", nslots=2)
    if rank == hang_rank:
        e.fault_set(f"rank_hang=1000000:{hang_ms}")
    e.start()
    e.wake(coll)
    dist.barrier()
    t0 = time.monotonic()
    g = GangCoordinator(e, None, [coll], epoch_ms=5.0, transport=transport, shm_name=shm_name,
                        rank=rank, world=world, deadline_ms=deadline_ms, reform=reform,
                        start_grace_ms=deadline_ms).start()
    degraded_at = None
    # the hung rank stalls before EVERY exchange (ppm 1e6): it completes the
    # epoch the others abandoned, then misses the next one itself
    while time.monotonic() - t0 < (2 * hang_ms + 3 * deadline_ms) / 1e3 + 0.5:
        if g.degraded and degraded_at is None:
            degraded_at = time.monotonic() - t0
            run0 = e.tenant_info(coll).run_ns
            t_deg = time.monotonic()
        time.sleep(0.002)
    ran_after = None
    if degraded_at is not None:
        ran_after = (e.tenant_info(coll).run_ns - run0) / ((time.monotonic() - t_deg) * 1e9)
    recs = [r.event for r in e.trace(from_start=True)]
    q.put({"rank": rank, "degraded_at": degraded_at, "epochs": g.epoch, "stats": g.stats(),
           "history": [(ep, st) for ep, st in g.history][-400:],
           "perfc_timeout": e.perfc().get("gang_timeout", 0), "traced": "GANG_TIMEOUT" in recs,
           "ran_after": ran_after, "dmesg": e.dmesg()})
    q.close()
    q.join_thread()  # flush the result before the hard exit below
    e.stop()
    os._exit(0)  # a gloo collective abandoned at the deadline must not block exit


def node_worker(rank: int, world: int, name: str, q, seconds: float = 1.0, epoch_ms: float = 5.0, ready=None,
                native: bool = True):
    """One of `world` node-local scheduler ranks on the native shm gang
    transport (the 8-GPU node layout, rehearsed on CPU): every rank runs its
    own engine with a hog and a gang tenant; returns the decision history and
    the GANG_EPOCH records of its trace ring for the cross-rank check."""
    from pbs_amd.core.engine import Engine
    from pbs_amd.parallel.gang import GangCoordinator
    e = Engine(partitions=[(rank, x) for x in range(2)], quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    hog = e.tenant_create("hog", nslots=2)
    coll = e.tenant_create("coll", nslots=2)
    e.trace_set_mask(["GANG_EPOCH"])
    e.start()
    e.wake(hog)
    e.wake(coll)
    if ready is not None:  # every rank imported and built its engine (spawn start-up skew is seconds on a busy host)
        ready.wait(120)
    g = GangCoordinator(e, None, [coll], epoch_ms=epoch_ms, share=0.5, transport="shm", shm_name=name,
                        rank=rank, world=world, deadline_ms=5000.0, native=native).start()
    time.sleep(seconds)
    g.stop()
    recs = [r.a[1] for r in e.trace(max_records=1 << 16, from_start=True)
            if r.event == "GANG_EPOCH" and r.a[0] == coll]
    q.put({"rank": rank, "history": g.history, "stats": g.stats(), "trace_states": recs})
    e.stop()


# ---- scripts/microbench.py workers (module-level: spawn pickles them by name)
def gang_bench_worker(rank, world, name, iters, q):
    from pbs_amd.parallel.gang import _ShmTransport
    tr = _ShmTransport(name, rank, world, 16)
    lat = []
    vals = list(range(8))
    for i in range(iters):
        t0 = time.monotonic_ns()
        # the first exchange also absorbs the ranks' spawn start-up skew
        # (seconds on a host busy with other tests; dropped as warm-up below)
        r = tr.reduce_min(vals, t0 + (60_000_000_000 if i == 0 else 10_000_000_000))
        if r is None:
            q.put((rank, None))  # the parent fails at once instead of waiting out its queue timeout
            raise RuntimeError("gang shm timeout")
        lat.append(time.monotonic_ns() - t0)
    tr.close()
    q.put((rank, lat[iters // 10:]))  # drop warm-up


def spin_barrier_worker(rank, world, arr, iters, q):
    """Host-noise baseline for the gang gate (tests/test_microbench.py): the
    same back-to-back barrier among `world` processes, as a plain Python spin
    on a shared counter array -- no gang code at all.  A loaded host slows it
    the way it slows the native epoch, so the gate compares against it."""
    lat = []
    for i in range(1, iters + 1):
        t0 = time.monotonic_ns()
        arr[rank] = i
        deadline = t0 + (60_000_000_000 if i == 1 else 10_000_000_000)
        while min(arr[:world]) < i:
            if time.monotonic_ns() > deadline:
                q.put((rank, None))
                raise RuntimeError("spin barrier timeout")
        lat.append(time.monotonic_ns() - t0)
    q.put((rank, lat[iters // 10:]))


def sem_barrier_worker(rank, world, bar, iters, q):
    """The blocking counterpart of spin_barrier_worker: a multiprocessing
    Barrier (semaphores: a futex sleep and wake per crossing), which a loaded
    host slows the way it slows a native epoch that sleeps on its doorbell."""
    lat = []
    for _ in range(iters):
        t0 = time.monotonic_ns()
        bar.wait(60)
        lat.append(time.monotonic_ns() - t0)
    q.put((rank, lat[iters // 10:]))


def gloo_bench_worker(rank, world, port, iters, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = torch.zeros(8, dtype=torch.int64)
    lat = []
    for _ in range(iters):
        t0 = time.monotonic_ns()
        dist.all_reduce(buf, op=dist.ReduceOp.MIN)
        lat.append(time.monotonic_ns() - t0)
    dist.destroy_process_group()
    q.put((rank, lat[iters // 10:]))
