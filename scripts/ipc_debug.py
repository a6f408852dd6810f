"""IPC all-reduce tenant debug: 2 processes on one GPU, gated runs with
per-step flag dumps (run with torch.distributed env: RANK, WORLD_SIZE, ...)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
from pbs_amd.runtime.gpu import CTX, XCDS, GpuContext, Runner
from pbs_amd.parallel.ipc_coll import IpcColl
ctx = GpuContext(0, nctx=4)
coll = IpcColl(0, rank, world, 32 << 20)
r = Runner(ctx, "allreduce", 1, gate=False, engine_wake=False, coll=coll, chunk_bytes=1 << 18, timeout_ms=3000)
def log(*a):
    print(f"[r{rank} {time.perf_counter():.3f}]", *a, file=sys.stderr, flush=True)
def step(name, n):
    dist.barrier()
    t0 = time.perf_counter()
    r.submit(n)
    try:
        r.wait(10)
        ok = True
    except Exception as ex:
        ok = False
    st = r.stats()
    log(name, "ok" if ok else "FAIL", f"{(time.perf_counter()-t0)*1e3:.1f} ms units {st.units_done} launches {st.launches} relaunches {st.relaunches} flags {coll.flags()}")
    return ok
step("ungated x5", 5)
ctx.set_se_mode(True)
mine = [1 if c >= 2 else -1 for x in range(XCDS) for c in range(CTX)]
ctx.set_owners(mine)
r.set_gate(True)
ok = step("gated se23 x5", 5)
ok = ok and step("gated se23 x20", 20)
if ok:
    ctx.set_owners([1] * (XCDS * CTX))
    ok = step("gated all x20", 20)
if ok:  # revocation mid-run: rank r revokes every SE after (r + 1) x 20 ms for 50 ms
    ctx.set_owners(mine)
    dist.barrier()
    t0 = time.perf_counter()
    r.submit(400)
    time.sleep(0.002 * (rank + 1))
    ctx.set_owners([-1] * (XCDS * CTX))
    log("revoked", r.stats().units_done, coll.flags())
    time.sleep(0.05)
    log("before restore", r.stats().units_done, r.stats().relaunches, coll.flags())
    ctx.set_owners(mine)
    log("restored", r.stats().units_done, coll.flags())
    try:
        r.wait(15)
    except Exception as ex:
        ok = False
    st = r.stats()
    log("revocation", "ok" if ok else "FAIL", f"units {st.units_done} launches {st.launches} relaunches {st.relaunches} flags {coll.flags()}")
log("done", ok)
r.close(); coll.close(); ctx.close()
dist.barrier()
