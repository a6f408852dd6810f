"""Wait-latency producer: the guest spin-lock hook, rebuilt
for GPU tenants.

The reference counts how many times a guest vCPU spins on a contended ticket
lock and reports the count to the hypervisor (``vcrd_op(time, 1)``,
L:arch/x86/include/asm/spinlock.h:55-80 -> X:xen/common/sched_credit.c:249-259);
the ATC policy sizes every domain's slice from it
(X:xen/common/sched_credit_atc.c:210-229,291-460).  The lock-holder-preemption
symptom it measures -- a vCPU burning time waiting on a peer that is not
running -- has a direct analog for GPU tenants: an RCCL collective whose peer
rank is descheduled (its kernels spin on xGMI flags until the peer arrives),
and a host thread blocked in ``hipStreamSynchronize`` / ``hipEventSynchronize``
on work that is queued behind another tenant.

``WaitProbe`` times those waits and posts the excess as ``REPORT_WAIT``
records (ns):

* ``collective(op, tensor, ...)``: issues a ``torch.distributed`` collective
  and times it -- device time between HIP events recorded on the issuing
  stream around the call for GPU tensors (harvested later without a sync),
  host time to completion for CPU tensors (gloo).  The wait is the duration
  minus a per-(op, shape) baseline: a decaying minimum of the observed
  durations, i.e. the collective's uncontended cost.  What is left is time
  spent waiting for the slowest peer.
* ``sync(obj)``: host time blocked in ``synchronize()`` of a stream / event /
  the device, reported whole (a blocked host thread is pure wait).
* ``patch_dist()``: a context manager that routes ``dist.all_reduce`` /
  ``all_gather_into_tensor`` / ``reduce_scatter_tensor`` / ``broadcast`` /
  ``barrier`` through the probe, so unmodified training code is covered.

With an ``ArrivalBoard`` (ranks of one node) the wait is exact instead of
baseline-relative: every rank stamps its arrival at collective ``seq`` on the
node's shared monotonic clock in a small shared-memory board before issuing
it, and after completion reads everyone's stamp: ``wait = max(arrivals) -
own arrival``.  This is the one that stays correct when a peer is *always*
late (a constant skew would otherwise be learned as the baseline).

The sink is any ``f(wait_ns)``: ``TenantClient.report_wait`` (control-page
report ring, out of process) or ``lambda ns: engine.report_wait(tid, ns)``
(in process).  Reports below ``min_report_ns`` are dropped, as the guest
hook only calls ``vcrd_op`` when it spun at all (``if (time > 0)``).
"""
from __future__ import annotations

import contextlib
import threading
import time
from collections import deque
from typing import Callable, Deque, Dict, Optional, Tuple

REPORT_WAIT = 1


class ArrivalBoard:
    """Per-node collective arrival stamps: int64 [world, RING, 2] = (seq, t_ns)
    in POSIX shared memory.  Rank 0 creates the region (``name`` must be
    fresh and agreed by all ranks, e.g. a nonce broadcast by rank 0), the
    others attach (retrying until it exists)."""

    RING = 256

    def __init__(self, name: str, rank: int, world: int, create: Optional[bool] = None, timeout_s: float = 30.0):
        import numpy as np
        from multiprocessing import shared_memory
        self.rank, self.world, self.name = rank, world, name
        size = world * self.RING * 2 * 8
        create = (rank == 0) if create is None else create
        if create:
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=size)
        else:
            t_end = time.monotonic() + timeout_s
            while True:
                try:
                    self.shm = shared_memory.SharedMemory(name=name)
                    break
                except FileNotFoundError:
                    if time.monotonic() > t_end:
                        raise
                    time.sleep(0.005)
        try:  # lifetime is explicit (the creator unlinks in close()), not the resource tracker's
            from multiprocessing import resource_tracker
            resource_tracker.unregister(self.shm._name, "shared_memory")
        except Exception:
            pass
        self.owner = create
        self.a = np.ndarray((world, self.RING, 2), dtype=np.int64, buffer=self.shm.buf)
        if create:
            self.a[:] = -1
        self.seq = 0

    def arrive(self) -> tuple:
        """Stamp this rank's arrival at its next collective; returns (seq, t)."""
        self.seq += 1
        t = time.monotonic_ns()
        row = self.a[self.rank, self.seq % self.RING]
        row[1] = t          # stamp first, then publish the sequence number
        row[0] = self.seq   # (x86 stores are not reordered with other stores)
        return self.seq, t

    def wait_ns(self, seq: int, t_own: int) -> int:
        """After collective ``seq`` completed: max peer arrival - own arrival
        (peers whose stamp for ``seq`` was already overwritten are skipped)."""
        last = t_own
        slot = seq % self.RING
        for r in range(self.world):
            s, t = int(self.a[r, slot, 0]), int(self.a[r, slot, 1])
            if s == seq and t > last:
                last = t
        return last - t_own

    def close(self):
        try:
            del self.a
            self.shm.close()
            if self.owner:  # not shm.unlink(): that also unregisters from the tracker
                import _posixshmem
                _posixshmem.shm_unlink(self.shm._name)
        except Exception:
            pass


class WaitProbe:
    def __init__(self, sink: Callable[[int], object], min_report_ns: int = 2000, decay: float = 1.002,
                 max_pending: int = 256, board: Optional[ArrivalBoard] = None):
        self.sink = sink
        self.board = board
        self.min_report_ns = int(min_report_ns)
        self.decay = float(decay)
        self.base: Dict[Tuple, float] = {}
        self.pending: Deque = deque()
        self.max_pending = max_pending
        self.lock = threading.Lock()
        self.n_timed = 0
        self.n_reports = 0
        self.wait_ns_total = 0
        self.sync_ns_total = 0

    # ------------------------------------------------------------ baseline
    def _excess(self, key, dur_ns: float) -> int:
        """Duration minus the decaying-minimum baseline for this key."""
        b = self.base.get(key)
        if b is None or dur_ns < b:
            b = dur_ns
        self.base[key] = b * self.decay  # drift up slowly: a faster path is re-learned
        return int(max(0.0, dur_ns - b))

    def _post(self, wait_ns: int, sync: bool = False):
        self.n_timed += 1
        if sync:
            self.sync_ns_total += wait_ns
        if wait_ns < self.min_report_ns:
            return
        self.wait_ns_total += wait_ns
        self.n_reports += 1
        self.sink(int(wait_ns))

    # -------------------------------------------------------- collectives
    def collective(self, op: Callable, tensor, *args, **kw):
        """Run ``op(tensor, *args, **kw)`` (a torch.distributed collective)
        timed; returns what ``op`` returns."""
        key = (getattr(op, "__name__", str(op)), tuple(getattr(tensor, "shape", ())), str(getattr(tensor, "dtype", "")))
        if self.board is not None:  # exact: arrival skew on the node's clock
            seq, t_own = self.board.arrive()
            out = op(tensor, *args, **kw)
            if kw.get("async_op") and out is not None:
                out.wait()
            if getattr(tensor, "is_cuda", False):
                # every peer has stamped once the collective completed on the
                # device: harvest when the event after it has fired (no sync)
                import torch
                e1 = torch.cuda.Event()
                e1.record(torch.cuda.current_stream(tensor.device))
                with self.lock:
                    self.pending.append((("board", seq, t_own), None, e1))
                    if len(self.pending) > self.max_pending:
                        self.pending.popleft()
                self.poll()
            else:
                self._post(self.board.wait_ns(seq, t_own))
            return out
        if getattr(tensor, "is_cuda", False):
            import torch
            s = torch.cuda.current_stream(tensor.device)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            out = op(tensor, *args, **kw)
            if kw.get("async_op") and out is not None:
                out.wait()  # current stream waits on the collective's stream
            e1.record(s)
            with self.lock:
                self.pending.append((key, e0, e1))
                if len(self.pending) > self.max_pending:
                    self.pending.popleft()
            self.poll()
            return out
        t0 = time.monotonic_ns()
        async_op = kw.pop("async_op", False)
        work = op(tensor, *args, async_op=True, **kw)
        if work is not None and not async_op:
            work.wait()
        dur = time.monotonic_ns() - t0
        with self.lock:
            w = self._excess(key, dur)
        self._post(w)
        return work if async_op else None

    def poll(self) -> int:
        """Harvest completed GPU event pairs (no synchronisation); returns
        the number harvested."""
        n = 0
        while True:
            with self.lock:
                if not self.pending:
                    return n
                key, e0, e1 = self.pending[0]
                if not e1.query():
                    return n
                self.pending.popleft()
                if key[0] == "board":
                    w = self.board.wait_ns(key[1], key[2])
                else:
                    w = self._excess(key, e0.elapsed_time(e1) * 1e6)
            self._post(w)
            n += 1

    def flush(self):
        """Wait for every pending pair and harvest it (end of a run)."""
        with self.lock:
            last = self.pending[-1][2] if self.pending else None
        if last is not None:
            last.synchronize()
        self.poll()

    # ---------------------------------------------------------------- syncs
    def sync(self, obj=None):
        """``obj.synchronize()`` (stream / event; None = the device) timed."""
        t0 = time.monotonic_ns()
        if obj is None:
            import torch
            torch.cuda.synchronize()
        else:
            obj.synchronize()
        self._post(time.monotonic_ns() - t0, sync=True)

    # ------------------------------------------------------- dist patching
    @contextlib.contextmanager
    def patch_dist(self):
        """Route the common torch.distributed collectives through the probe."""
        import torch.distributed as dist
        names = ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast")
        saved = {n: getattr(dist, n) for n in names if hasattr(dist, n)}
        saved_barrier = dist.barrier

        def wrap(name, fn):
            def timed(tensor, *a, **k):  # keyed by the first (output) tensor's shape
                return self.collective(fn, tensor, *a, **k)
            timed.__name__ = name
            return timed

        def barrier(*a, **k):
            t0 = time.monotonic_ns()
            r = saved_barrier(*a, **k)
            with self.lock:
                w = self._excess(("barrier",), time.monotonic_ns() - t0)
            self._post(w)
            return r

        try:
            for n, fn in saved.items():
                setattr(dist, n, wrap(n, fn))
            dist.barrier = barrier
            yield self
        finally:
            for n, fn in saved.items():
                setattr(dist, n, fn)
            dist.barrier = saved_barrier

    def stats(self) -> Dict[str, float]:
        return {"timed": self.n_timed, "reports": self.n_reports, "wait_ns_total": self.wait_ns_total,
                "sync_ns_total": self.sync_ns_total, "pending": len(self.pending)}


def engine_sink(engine, tenant: int) -> Callable[[int], object]:
    """In-process sink: post straight into an Engine (REPORT_WAIT)."""
    return lambda ns: engine.report_wait(tenant, int(ns), REPORT_WAIT)
