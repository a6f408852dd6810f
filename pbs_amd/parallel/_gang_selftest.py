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
