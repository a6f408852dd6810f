"""IPC all-reduce tenant (csrc/hip/coll_kernels.hip) with 2 processes.

``one_device``: both ranks on one MI355X -- same-device IPC handles exercise
the whole multi-GPU path (handle export / open, the direct reduce-scatter +
all-gather kernel, the P2P-flag barrier between units, gating per
workgroup, revocation and relaunch, the agreed-count drain).
``peer_devices``: rank r on device r, so the peer
buffers are mapped over xGMI and the flags cross devices at system scope --
the 8-GPU bench's placement.  Skipped below two visible GPUs; each rank
records whether its device can access the peer's (hipDeviceCanAccessPeer).

The result is compared bit for bit with an fp32 torch reference of the same
reduction (bf16 inputs summed in fp32 in rank order, rounded to bf16).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import json, os, sys, time
sys.path.insert(0, %(root)r)
import torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
DEV = rank if %(peer)d else 0
torch.cuda.set_device(DEV)
dist.init_process_group("gloo")
from pbs_amd.runtime.gpu import CTX, XCDS, GpuContext, Runner
from pbs_amd.parallel.ipc_coll import IpcColl, agreed_drain
ctx = GpuContext(DEV, nctx=4)
nbytes = 32 << 20
coll = IpcColl(DEV, rank, world, nbytes)
g = torch.Generator(device="cuda").manual_seed(100 + rank)
x = torch.randn(nbytes // 2, device="cuda", dtype=torch.bfloat16, generator=g)
coll.fill(x, 0)
xs = [torch.empty_like(x.cpu()) for _ in range(world)]
dist.all_gather(xs, x.cpu())
acc = torch.zeros(x.numel(), dtype=torch.float32)
for t in xs:
    acc += t.float()
ref = acc.to(torch.bfloat16)
out = {"rank": rank, "device": DEV}
if %(peer)d:
    out["can_access_peer"] = bool(torch.cuda.can_device_access_peer(DEV, 1 - DEV))
T = 1
r = Runner(ctx, "allreduce", T, gate=False, engine_wake=False, coll=coll, chunk_bytes=1 << 18)
dist.barrier()
r.submit(1); r.wait(60); torch.cuda.synchronize()
dist.barrier()
o = coll.read(1).cpu()
out["exact"] = bool(torch.equal(o, ref))
out["max_abs_diff"] = float((o.float() - ref.float()).abs().max())
# gated, backlogged, with revocations: the tenant owns SEs {2,3}, loses them
# for a while (its workgroups leave, units are relaunched), gets them back
ctx.set_se_mode(True)
mine = [T if c >= 2 else -1 for x_ in range(XCDS) for c in range(CTX)]
ctx.set_owners(mine)
r.set_gate(True)
dist.barrier()
r.submit(40)
time.sleep(0.02 * (rank + 1))
ctx.set_owners([-1] * (XCDS * CTX))
time.sleep(0.05)
ctx.set_owners(mine)
try:
    r.wait(20)
except Exception as ex:
    st = r.stats()
    print(f"rank {rank} stuck: units {st.units_done} submitted {st.submitted} launches {st.launches} "
          f"relaunches {st.relaunches} waits_owner {st.waits_owner} owners {ctx.owners()[:8]}", file=sys.stderr, flush=True)
    raise
st = r.stats()
out["units"] = st.units_done
out["relaunches"] = st.relaunches
# unequal backlogs, stopped on an agreed count
r.submit(30 if rank == 0 else 10)
time.sleep(0.01)
def agree(n):
    t = torch.tensor([n], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())
out["agreed"] = agreed_drain(r, agree)
out["units_final"] = r.stats().units_done
torch.cuda.synchronize()
dist.barrier()
o = coll.read(1).cpu()
out["exact_after"] = bool(torch.equal(o, ref))
r.close(); coll.close(); ctx.close()
dist.barrier()
print("RESULT " + json.dumps(out), flush=True)
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("placement", ["one_device", "peer_devices"])
def test_ipc_allreduce_two_processes_exact_and_gated(placement):
    peer = placement == "peer_devices"
    if peer and torch.cuda.device_count() < 2:
        pytest.skip("rank-per-device placement needs two visible GPUs")
    world = 2
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", CODE % {"root": ROOT, "peer": int(peer)}], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs, logs = [], []
    for p in procs:
        try:
            so, se = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append((p.returncode, so, se))
    for rank, (rc, so, se) in enumerate(logs):
        assert rc == 0, "\n".join(f"--- rank {r} rc={c}\n{o[-1500:]}\n{e[-3000:]}" for r, (c, o, e) in enumerate(logs))
        outs.append(json.loads([x for x in so.splitlines() if x.startswith("RESULT ")][-1][7:]))
    print(json.dumps(outs, indent=1))
    for o in outs:
        assert o["exact"], o
        assert o["exact_after"], o
        assert o["units"] == 41, o  # 1 + 40, every unit completed through the revocation
        # rank 0 cannot run more than a unit or two past rank 1's: the drain
        # tops the laggard up to the agreed count instead of hanging rank 0
        assert o["units_final"] == o["agreed"] > 41, o
    assert outs[0]["agreed"] == outs[1]["agreed"]
    if peer:
        assert [o["device"] for o in outs] == [0, 1]
        assert all(o["can_access_peer"] for o in outs), outs
