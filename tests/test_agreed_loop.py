"""N > 1 co-run: the all-reduce tenant's back-to-back loop must stop on the
same collective count on every rank, whatever moment each rank's main thread
raises its stop (a rank one collective ahead would otherwise wait in it
forever).  World 3 on gloo; the ranks stop at deliberately skewed times and
the collective itself is short, so without the agreed count a mismatch is
near certain."""
import multiprocessing as mp
import os
import socket


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import time

    import torch
    import torch.distributed as dist

    from pbs_amd.bench.corun import AgreedLoop
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctrl = dist.new_group(backend="gloo")
    coll = dist.new_group(backend="gloo")
    buf = torch.ones(1024)
    counts = []
    for rep in range(6):
        loop = AgreedLoop(lambda: dist.all_reduce(buf, group=coll)).start()
        time.sleep(0.05 + 0.013 * ((rank + rep) % world))  # skewed stops

        def agree(n):
            t = torch.tensor([n], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl)
            return int(t.item())
        counts.append(loop.stop(agree))
        assert loop.issued == counts[-1]
    t = torch.tensor(counts, dtype=torch.int64)  # a final collective on the coll group still matches
    dist.all_reduce(t, group=coll)
    q.put({"rank": rank, "counts": counts, "sum": t.tolist()})
    dist.destroy_process_group()


def test_agreed_loop_stops_every_rank_on_one_count():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 3, _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r = q.get(timeout=120)
        out[r["rank"]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    c0 = out[0]["counts"]
    assert all(out[r]["counts"] == c0 for r in out), out
    assert all(c > 0 for c in c0)
    assert out[0]["sum"] == [3 * c for c in c0]
