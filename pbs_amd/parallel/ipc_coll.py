"""All-reduce tenant over xGMI with IPC-mapped peer buffers (SURVEY §2.7 DP
tenant, §2.6 C16).

One process per GPU.  Every rank allocates its input, output and flag words
with hipMalloc (``gpbs_coll_create``), exports their IPC handles, exchanges
them over a host process group (gloo), and maps every peer's buffers
(``hipIpcOpenMemHandle``).  ``Runner(ctx, "allreduce", tenant, coll=...)``
then runs ``k_allreduce`` units (csrc/hip/coll_kernels.hip): a direct
reduce-scatter + all-gather over the xGMI mesh, gated per workgroup on the
partition table like every other gpbs tenant -- so the scheduler confines it
to the shader engines it owns and attributes its counters by ownership,
which RCCL's own kernels (on RCCL's internal streams) would escape.  Units
are collective (a P2P-flag barrier between units), so a rank never runs
ahead of a descheduled peer by more than one unit.

The same code runs with every rank on ONE GPU (same-device IPC handles):
that is how the CPU-less parts are tested (tests/test_gpu_ipc_coll.py).
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional

import torch

from ..ops.kernels import lib as hiplib


class IpcColl:
    def __init__(self, device: int, rank: int, world: int, nbytes: int, group=None,
                 gather: Optional[Callable] = None):
        """``gather(obj) -> list`` exchanges one picklable object per rank
        (default: ``torch.distributed.all_gather_object`` on ``group``)."""
        self.L = hiplib()
        self.device, self.rank, self.world = device, rank, world
        self.h = None
        align = 16 * world
        self.nbytes = (int(nbytes) + align - 1) // align * align
        if gather is None:
            import torch.distributed as dist

            def gather(obj):
                out = [None] * world
                dist.all_gather_object(out, obj, group=group)
                return out
        # Every rank makes exactly two exchanges whatever fails locally (its
        # handle or None, then its error or None), and all ranks raise
        # together: a rank that failed alone and moved on to the caller's
        # next collective would leave its peers waiting in this one (the
        # round-5 8-rank rehearsal hung that way).
        mine, err = None, None
        try:
            h = self.L.gpbs_coll_create(device, rank, world, self.nbytes)
            if not h:
                raise RuntimeError("gpbs_coll_create failed")
            self.h = C.c_void_p(h)
            nb = self.L.gpbs_coll_handle_bytes()
            buf = (C.c_char * nb)()
            if self.L.gpbs_coll_export(self.h, buf) != nb:
                raise RuntimeError("hipIpcGetMemHandle failed")
            mine = bytes(buf)
        except Exception as ex:  # noqa: BLE001 -- reported through the exchange
            err = f"rank {rank}: {ex}"
        allh = gather(mine)
        if err is None and any(hb is None for hb in allh):
            err = f"rank {rank}: a peer failed to export its buffers"
        if err is None:
            try:
                nb = self.L.gpbs_coll_handle_bytes()
                for peer, hb in enumerate(allh):
                    if peer == rank:
                        continue
                    arr = (C.c_char * nb).from_buffer_copy(hb)
                    rc = self.L.gpbs_coll_open(self.h, peer, arr)
                    if rc:
                        raise RuntimeError(f"hipIpcOpenMemHandle of rank {peer} failed ({rc})")
                if self.L.gpbs_coll_finalize(self.h):
                    raise RuntimeError("gpbs_coll_finalize failed")
            except Exception as ex:  # noqa: BLE001
                err = f"rank {rank}: {ex}"
        errs = [e for e in gather(err) if e]
        if errs:
            self.close()
            raise RuntimeError("IPC all-reduce setup failed: " + "; ".join(errs[:4]))
        self.desc = self.L.gpbs_coll_buffer(self.h, 3)

    def fill(self, t: torch.Tensor, which: int = 0):
        """Copy a bf16 device tensor into this rank's input (0) / output (1)."""
        t = t.contiguous()
        nb = t.numel() * t.element_size()
        if self.L.gpbs_coll_copy(self.h, which, C.c_void_p(t.data_ptr()), nb, 1):
            raise RuntimeError("gpbs_coll_copy failed")

    def read(self, which: int = 1) -> torch.Tensor:
        """This rank's output (1) / input (0) buffer as a new bf16 tensor."""
        t = torch.empty(self.nbytes // 2, dtype=torch.bfloat16, device=torch.device("cuda", self.device))
        if self.L.gpbs_coll_copy(self.h, which, C.c_void_p(t.data_ptr()), self.nbytes, 0):
            raise RuntimeError("gpbs_coll_copy failed")
        return t

    def flags(self):
        """This rank's flag words: word s = units rank s has finished (diagnostics)."""
        t = torch.zeros(8, dtype=torch.int32, device=torch.device("cuda", self.device))
        if self.L.gpbs_coll_copy(self.h, 2, C.c_void_p(t.data_ptr()), 32, 0):
            raise RuntimeError("gpbs_coll_copy failed")
        return t.cpu().tolist()[:self.world]

    def close(self):
        if getattr(self, "h", None):
            self.L.gpbs_coll_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def agreed_drain(runner, agree: Callable[[int], int], timeout_s: float = 120.0) -> int:
    """Stop a backlogged all-reduce runner on a unit count every rank agrees
    on.  Units are collective (unit k waits for every peer's unit k-1), so a
    rank that stopped after fewer units than a peer would leave that peer's
    in-flight unit waiting: drop the local backlog, take the MAX over ranks
    of the units launched, run the missing ones, then wait.  Returns the
    agreed count."""
    runner.cancel()
    launched = runner.stats().submitted
    target = max(int(agree(launched)), launched)
    if target > launched:
        runner.submit(target - launched)
    runner.wait(timeout_s)
    return target
