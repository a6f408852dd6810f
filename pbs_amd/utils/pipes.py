"""Masked-queue pipe pre-flight.

The SE-exclusive layouts rely on where the process's CU-masked queues land
on the command processor's pipes: hardware queues take the pipes
round-robin in creation order, and a CU-masked queue that shares a pipe
with a queue of the other class half lets a GEMM dispatch waiting for CUs
hold up the other half's dispatches (profiles/r5/pipe_probe.txt).  The
runtime therefore creates all of its masked queues in ONE burst
(csrc/hip/runtime.cpp MaskedPoolCore::prealloc, plan kPlan: compute half
on burst indexes 0, 4, 8 -- one pipe -- memory half on the other three)
and relies only on pipes RELATIVE to the burst's first queue.  That holds
whatever queues the process made before (RCCL's, the profiler's), as long
as no other queue is created in the middle of the burst.

``pipe_preflight`` makes the burst at a point of the bench's choosing --
after RCCL's communicators exist -- and checks it against the kernel
driver's view of the process: the KFD queue ids the process gained around
the burst must be exactly the pool's queues, one contiguous run (no
foreign queue in between, so creation order = pool order), and the pool's
recorded pipes / halves must match the plan.  The result is the rank's
pre-flight record; ``ok`` False marks the rank failed in the bench line.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence

# burst plan (csrc/hip/runtime.cpp kPlan): class half of burst index i
PLAN = (0, 1, 1, 1, 0, 1, 1, 1, 0, 1)
PIPES = 4


def kfd_queue_ids(pid: Optional[int] = None) -> Optional[List[int]]:
    """The hardware queue ids KFD holds for a process (None where sysfs does
    not expose them)."""
    try:
        return sorted(int(q) for q in os.listdir(f"/sys/class/kfd/kfd/proc/{pid or os.getpid()}/queues")
                      if q.isdigit())
    except OSError:
        return None


def check_burst(before: Optional[Sequence[int]], after: Optional[Sequence[int]], pool: Sequence[int],
                plan: Sequence[int] = PLAN) -> Dict:
    """Pure check of one burst.  before / after: KFD queue ids around it
    (None: not exposed); pool: gpbs_hip_masked_pool_prealloc's entries
    (pipe | half << 8) in creation order."""
    rec: Dict = {"pool_queues": len(pool), "plan_ok": False, "contiguous": None, "new_kfd_queues": None}
    pipes = [e & 0xFF for e in pool]
    halves = [(e >> 8) & 1 for e in pool]
    n = min(len(pool), len(plan))
    rec["plan_ok"] = len(pool) >= len(plan) and halves[:n] == list(plan[:n]) and \
        pipes[:n] == [i % PIPES for i in range(n)]
    # the compute half's queues share one pipe and no memory queue is on it
    cp = {p for p, h in zip(pipes, halves) if h == 0}
    mp = {p for p, h in zip(pipes, halves) if h == 1}
    rec["compute_pipes"], rec["memory_pipes"] = sorted(cp), sorted(mp)
    rec["pipes_disjoint"] = not (cp & mp)
    if before is not None and after is not None:
        new = sorted(set(after) - set(before))
        rec["new_kfd_queues"] = len(new)
        # KFD hands out the lowest free id: a burst with no foreign queue in
        # between is one run of ids (holes from destroyed queues below it
        # would be taken first, and then the run is still unbroken by others)
        rec["contiguous"] = len(new) == len(pool) and (not new or new == list(range(new[0], new[0] + len(new))))
    rec["ok"] = bool(rec["plan_ok"] and rec["pipes_disjoint"] and rec["contiguous"] is not False)
    return rec


def pipe_preflight(lib, device: int, list_qids: Callable[[], Optional[List[int]]] = kfd_queue_ids) -> Dict:
    """Make the process's masked-queue burst now and check it (see module
    doc).  A pool that already existed reports plan_ok from its record and
    contiguous None (the burst happened earlier)."""
    import ctypes as C
    before = list_qids()
    buf = (C.c_int * 64)()
    n = lib.gpbs_hip_masked_pool_prealloc(int(device), buf, 64)
    after = list_qids()
    if n < 0:
        return {"ok": False, "error": int(n)}
    pool = [int(buf[i]) for i in range(min(n, 64))]
    if before is not None and after is not None and set(after) == set(before):
        before = after = None  # the burst was made before this call: nothing to compare
    return check_burst(before, after, pool)
