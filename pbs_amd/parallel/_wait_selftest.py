"""Workers for the K10 wait-latency tests (tests/test_waitprobe.py): gloo
ranks on the CPU stand in for the RCCL ranks of a collective tenant."""
from __future__ import annotations

import os
import time


def wait_worker(rank: int, world: int, port: int, q, lag_ms: float, board_name: str, nsteps: int = 24):
    """One rank of the collective tenant.  Rank 1 arrives ``lag_ms`` late at
    every all-reduce (its launch gate held it: the peer is descheduled).
    Rank 0's probe measures the wait on the arrival board and posts it into
    an ATC engine on a simulated clock, 4 collectives per 21 ms ATC period."""
    import torch
    import torch.distributed as dist

    from pbs_amd.core.engine import Engine
    from pbs_amd.runtime.waitprobe import ArrivalBoard, WaitProbe, engine_sink
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(sched="atc", sim_clock=True, partitions=[(rank, 0), (rank, 1)], atc={"wait_unit_ns": 8})
    e.tenant_create("Domain-0", nslots=1)
    t = e.tenant_create("coll", nslots=2)
    e.wake(t)
    board = ArrivalBoard(board_name, rank, world)
    dist.barrier()
    sink = engine_sink(e, t)
    waits = []  # every reported wait (ns), for a per-collective comparison

    def record(ns):
        waits.append(int(ns))
        return sink(ns)
    probe = WaitProbe(record, board=board)
    buf = torch.ones(1 << 14)
    now = 0
    traj = []
    for step in range(nsteps):
        if rank == 1 and lag_ms > 0:
            time.sleep(lag_ms / 1e3)
        probe.collective(dist.all_reduce, buf)
        now += 21_000_000 // 4
        e.advance(now)
        traj.append(e.tenant_info(t).tslice_us)
    # the same collectives through patch_dist (unmodified caller code)
    with probe.patch_dist():
        for _ in range(4):
            if rank == 1 and lag_ms > 0:
                time.sleep(lag_ms / 1e3)
            dist.all_reduce(buf)
    info = e.tenant_info(t)
    dist.barrier()
    board.close()
    q.put({"rank": rank, "traj": traj, "tslice": info.tslice_us, "spin_latency": info.spin_latency,
           "reports": info.report_count, "stats": probe.stats(), "waits": waits, "collectives": nsteps + 4})
    dist.destroy_process_group()


def gang_wait_worker(rank: int, world: int, port: int, q, shm_name: str, report_s: float = 0.3,
                     seconds: float = 1.2, epoch_ms: float = 5.0):
    """Wait-driven gang windows: rank 1's collective tenant reports heavy
    waits for ``report_s`` seconds, then none.  Every rank must switch the
    tenant's gang windows on (and back off after the hold) at the same epoch."""
    import torch.distributed as dist

    from pbs_amd.core.engine import Engine
    from pbs_amd.parallel.gang import GangCoordinator
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = Engine(partitions=[(rank, x) for x in range(2)], quantum_align_us=0)
    e.tenant_create("Domain-0", nslots=1)
    coll = e.tenant_create("coll", nslots=2)
    e.start()
    e.wake(coll)
    dist.barrier()
    g = GangCoordinator(e, None, [coll], epoch_ms=epoch_ms, share=0.5, transport="shm", shm_name=shm_name,
                        rank=rank, world=world, wait_driven=True, wait_on_frac=0.05, wait_hold_epochs=20).start()
    t0 = time.monotonic()
    while time.monotonic() - t0 < seconds:
        if rank == 1 and time.monotonic() - t0 < report_s:
            e.report_wait(coll, 1_000_000)  # 1 ms waited on a peer, every ms
        time.sleep(0.001)
    g.stop()
    st = g.stats()
    e.stop()
    q.put({"rank": rank, "history": g.history, "stats": st})
    dist.destroy_process_group()
