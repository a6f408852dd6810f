"""Gang epoch exchange over xGMI (pbs_amd/parallel/gang.py
``_XgmiTransport``, csrc/hip/coll_kernels.hip ``k_gang_exchange``) with 2
processes: ``one_device`` puts both on one MI355X (same-device IPC handles
exercise the board mapping, the device-side publish / wait / copy and the
parity double buffering); ``peer_devices`` puts rank r on device r, so the
board crosses xGMI as on the 8-GPU node (skipped below two visible GPUs).  Checks every exchange's SUM
and MIN against the known per-rank values, reports the round-trip latency
next to the host shm transport, and checks that a rank whose peer stops
gets a timeout within its deadline instead of a hang.
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
from pbs_amd.parallel.gang import _XgmiTransport, _ShmTransport

def gather(obj):
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out

tr = _XgmiTransport(rank, world, 8, DEV, gather)
out = {"rank": rank, "bad": 0, "device": DEV}
lat = []
dist.barrier()
for k in range(1, 401):
    vals = [rank + 1, 10 * (rank + 1), k, -k * (rank + 1)]
    t0 = time.perf_counter_ns()
    s = tr.reduce_sum(vals, time.monotonic_ns() + int(2e9)) if k %% 2 else tr.reduce_min(vals, time.monotonic_ns() + int(2e9))
    lat.append(time.perf_counter_ns() - t0)
    want = [3, 30, 2 * k, -3 * k] if k %% 2 else [1, 10, k, -2 * k]
    if s != want:
        out["bad"] += 1
        if out["bad"] < 3:
            print("mismatch", k, s, want, file=sys.stderr, flush=True)
lat.sort()
out["p50_us"] = lat[len(lat) // 2] / 1e3
out["p99_us"] = lat[int(0.99 * (len(lat) - 1))] / 1e3
out["stats"] = tr.stats()
# the host shm transport, same exchange count, for comparison
sh = _ShmTransport(f"/gpbs-xgmi-test-{os.environ['MASTER_PORT']}", rank, world, 8)
dist.barrier()
lat = []
for k in range(400):
    t0 = time.perf_counter_ns()
    sh.reduce_sum([rank, k], time.monotonic_ns() + int(2e9))
    lat.append(time.perf_counter_ns() - t0)
lat.sort()
out["shm_p50_us"] = lat[len(lat) // 2] / 1e3
sh.close()
# a peer that stops: rank 0's next exchange times out at its deadline
dist.barrier()
if rank == 0:
    t0 = time.monotonic_ns()
    r = tr.reduce_sum([1, 1, 1, 1], time.monotonic_ns() + int(50e6))
    out["timeout_result"] = r
    out["timeout_ms"] = (time.monotonic_ns() - t0) / 1e6
dist.barrier()
tr.close()
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
def test_gang_exchange_over_xgmi_two_processes(placement):
    peer = placement == "peer_devices"
    if peer and torch.cuda.device_count() < 2:
        pytest.skip("rank-per-device placement needs two visible GPUs")
    world = 2
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", CODE % {"root": ROOT, "peer": int(peer)}], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    logs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append((p.returncode, so, se))
    outs = []
    for rank, (rc, so, se) in enumerate(logs):
        assert rc == 0, "\n".join(f"--- rank {r} rc={c}\n{o[-1500:]}\n{e[-3000:]}" for r, (c, o, e) in enumerate(logs))
        outs.append(json.loads([x for x in so.splitlines() if x.startswith("RESULT ")][-1][7:]))
    print(json.dumps(outs, indent=1))
    for o in outs:
        assert o["bad"] == 0, o
        assert o["stats"]["exchanges"] == 400, o
        assert o["p50_us"] < 1000, o
    assert [o["device"] for o in outs] == ([0, 1] if peer else [0, 0])
    assert outs[0]["timeout_result"] is None
    assert 45 <= outs[0]["timeout_ms"] < 500, outs[0]
