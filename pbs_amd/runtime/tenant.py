"""Tenant shim: makes a torch process a gpbs tenant.

This is the guest side of the reference -- the Perfctr guest driver that
publishes counters through shared pages (S2, C10), the `vcrd_op` spin report
hypercall (P2, C7), the prepared lock-hold/I-O request hooks (P8, P7) and the
VIRQ upcall that wakes a descheduled vCPU (C9) -- rebuilt on the gpbsd control
plane:

* ``register`` over the daemon's Unix-socket RPC creates (or re-attaches to)
  the tenant and binds a 4 KiB control page in the daemon's POSIX shm region;
* a heartbeat thread keeps the daemon's failure detector quiet (S13);
* ``gate()`` blocks on the page's futex doorbell until the scheduler assigns
  the tenant at least one partition (the launch gate: no kernel preemption,
  the tenant stops launching at its next boundary);
* ``stream()`` returns a HIP stream whose CU mask covers exactly the
  (XCD, CU-half) partitions the tenant currently holds -- the actuation for
  third-party kernels (torch / hipBLASLt / RCCL) that cannot gate themselves
  through the partition table like the gpbs tenant kernels do;
* ``report_wait`` / ``report_hold`` / ``report_requests`` feed the spin-latency
  channel; ``wait_probe()`` produces the waits from timed RCCL collectives and
  stream/event syncs (K10, runtime/waitprobe.py), ``account`` publishes modeled counters (vPMU mirror), ``busy`` /
  ``idle`` set the has-work flag that wakes or blocks the tenant's slots.

    with TenantClient("llm-infer", slots=8) as t:
        for batch in loader:
            with t.slice() as s:         # waits for the gate, runs on s
                out = model(batch)
            t.account(flops=..., bytes=...)
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading
import time
from typing import Dict, List, Optional, Tuple

from .. import _native as N
from ..ctl.rpc import DEFAULT_SOCKET, Client

XCDS = 8
REPORT_WAIT, REPORT_HOLD, REPORT_REQUESTS = 1, 2, 3
# Modeled-counter units shared with the gpbs tenant kernels: one MFMA
# 16x16x32 bf16 = 16384 FLOP per instruction; 128-byte L2 lines.
FLOP_PER_INST = 16384
LINE = 128


def half_cu_words(owned: List[Tuple[int, int]]) -> List[int]:
    """CU-mask words (hipExtStreamCreateWithCUMask) covering the given
    (xcd, half) partitions: bit b = logical CU b/8 of XCD b%8, logical CU i on
    shader engine i%4, half = SE >> 1 (see csrc/hip/runtime.cpp)."""
    want = set(owned)
    words = [0] * 8
    for b in range(256):
        if (b % 8, ((b // 8) % 4) >> 1) in want:
            words[b // 32] |= 1 << (b % 32)
    return words


def se_cu_words(ses) -> List[int]:
    """CU-mask words covering shader engines `ses` of every XCD (logical CU i
    of an XCD on SE i % 4)."""
    want = set(ses)
    words = [0] * 8
    for b in range(256):
        if ((b // 8) % 4) in want:
            words[b // 32] |= 1 << (b % 32)
    return words


class QueueProber:
    """Choose, among K CU-masked queues of the same mask, the one whose slices
    run fastest, and re-choose when the chosen one degrades.

    Which hardware pipe a queue lands on is decided by the hardware scheduler
    from the node-wide queue set, not by the process.  Two processes whose
    active queues share a pipe measured a head-of-line stall: a decode-like
    step of 96 small GEMVs ran 16.5 ms instead of 2.5 ms next to a GEMM on
    the other shader engines, bimodally by run and unchanged for the whole
    run (scripts/queue_switch_probe.py, profiles/llm5/queue_switch_probe.json),
    which is config #5's collapse.  Equal masks, different queues: the fast
    and the slow queue differ only in where they were mapped.

    Explore each queue for ``explore`` slices (the median of its last
    ``keep``; a queue whose first slice is ``abort`` x slower than the best so
    far is left at once), exploit the fastest, and explore again when the exploited
    queue's EWMA exceeds ``drift`` x its explored median -- at most once per
    ``cooldown`` slices, doubling after every re-exploration that changed
    nothing.  Pure bookkeeping (CPU-testable); the caller times the slices."""

    def __init__(self, k: int, explore: int = 4, keep: int = 3, drift: float = 1.6, cooldown: int = 100,
                 abort: float = 2.0, start: Optional[int] = None, ref_ms: float = 0.0, probation: int = 3):
        self.k, self.explore, self.keep, self.drift = int(k), int(explore), int(keep), float(drift)
        self.abort = float(abort)
        self.cooldown0 = self.cooldown = int(cooldown)
        self.idx = 0
        self.exploring = True
        self.samples: List[List[float]] = [[] for _ in range(self.k)]
        self.ref = 0.0
        self.ewma = 0.0
        self.since = 0
        self.explorations = 0
        self.choices: List[int] = []
        # Remembered winner (a previous run's choice for this tenant and
        # mask): exploit it at once; if its first
        # `probation` slices run slower than drift x the remembered time,
        # explore after all.  Exploring costs one slow slice per stalled queue.
        self.probation = 0
        if start is not None and 0 <= int(start) < self.k and ref_ms > 0:
            self.idx, self.exploring = int(start), False
            self.ref = self.ewma = float(ref_ms)
            self.probation = int(probation)
            self._prob: List[float] = []

    def current(self) -> int:
        return self.idx

    @staticmethod
    def _median(xs: List[float]) -> float:
        xs = sorted(xs)
        n = len(xs)
        return xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])

    def record(self, ms: float):
        if self.exploring:
            self.samples[self.idx].append(ms)
            done = [self._median(x[-self.keep:]) for x in self.samples[:self.idx] if x]
            # a stalled queue shows on its first slice: leave it after one
            # (the stall costs one slow slice per exploration, not `explore`)
            stalled = bool(done) and ms > self.abort * min(done)
            if len(self.samples[self.idx]) < self.explore and not stalled:
                return
            if self.idx + 1 < self.k:
                self.idx += 1
                return
            meds = [self._median(x[-self.keep:]) if x else float("inf") for x in self.samples]
            best = min(range(self.k), key=lambda i: meds[i])
            prev = self.choices[-1] if self.choices else None
            if prev is not None and best == prev:
                self.cooldown *= 2  # nothing changed: back off
            else:
                self.cooldown = self.cooldown0
            self.idx, self.ref, self.ewma = best, meds[best], meds[best]
            self.exploring, self.since = False, 0
            self.choices.append(best)
            self.explorations += 1
            return
        if self.probation > 0:
            self._prob.append(ms)
            if len(self._prob) < self.probation:
                return
            self.probation = 0
            if self._median(self._prob) > self.drift * self.ref:  # the remembered queue is not fast here
                self.samples = [[] for _ in range(self.k)]
                self.idx, self.exploring = 0, True
                return
            self.choices.append(self.idx)
            return
        self.since += 1
        self.ewma = 0.8 * self.ewma + 0.2 * ms
        # a stall (abort x the explored time) re-explores at once; a milder
        # drift only after the cooldown.  Config #5 (s24): a queue that began
        # sharing a pipe with the trainer's ran 3x slower for 1.5 s while the
        # 100-slice cooldown ran out.
        severe = self.since >= 3 and self.ewma > self.abort * self.ref
        if severe or (self.since >= self.cooldown and self.ewma > self.drift * self.ref):
            self.samples = [[] for _ in range(self.k)]
            self.idx, self.exploring = 0, True

    def state(self) -> Optional[Dict[str, float]]:
        """The current choice, worth remembering once settled (None while exploring)."""
        if self.exploring or self.probation > 0 or self.ref <= 0:
            return None
        return {"idx": self.idx, "ref_ms": round(self.ref, 4)}


class TenantClient:
    def __init__(self, name: str, socket_path: str = DEFAULT_SOCKET, slots: int = 8, weight: int = -1,
                 cap: int = -1, pool=None, gpu: int = 0, heartbeat_s: float = 0.05, spatial: bool = True,
                 priority: int = 0, one_queue: bool = False, queue_probe: int = -1):
        self.name = name
        self.gpu = gpu
        self.spatial = spatial
        self.priority = priority
        self.rpc = Client(socket_path)
        r = self.rpc.call("register", name=name, slots=slots, weight=weight, cap=cap, pool=pool, pid=os.getpid())
        self.tenant: int = r["tenant"]
        self.page: int = r["page"]
        self.nctx: int = r.get("nctx", 2)
        self.se_mode: bool = bool(r.get("se_mode", False))
        # partition id -> (gpu, xcd, ctx)
        self.part: Dict[int, Tuple[int, int, int]] = {}
        for k, pid in r["partitions"].items():
            g, x, c = (int(v) for v in k.split(":"))
            self.part[int(pid)] = (g, x, c)
        self.lib = N.load_core()
        h = self.lib.gpbs_ctl_open(r["ctl"].encode())
        if not h:
            raise RuntimeError(f"cannot open control region {r['ctl']!r}")
        self.ctl = C.c_void_p(h)
        self._streams: Dict[Tuple, object] = {}
        self.one_queue = one_queue  # SE mode: one masked queue, on the class home half (see stream())
        self._home: Optional[Tuple[int, int]] = None
        # SE mode: K masked queues per half, the fastest chosen by measurement
        # (QueueProber); the slice body must end synchronised (the decode and
        # training loops do) for its time to mean anything
        self.queue_probe = int(queue_probe) if queue_probe >= 0 else (3 if self.se_mode else 0)
        self._probers: Dict[Tuple, QueueProber] = {}
        self._probe_key: Optional[Tuple] = None
        self._last_stream = None  # the stream of the previous slice (cross-queue ordering)
        self._progress = 0
        self._stop = threading.Event()
        self._hb = threading.Thread(target=self._beat, args=(heartbeat_s,), daemon=True, name=f"gpbs-hb-{name}")
        self._hb.start()
        self.counters = [0, 0, 0, 0]

    # ------------------------------------------------------------ liveness
    def _beat(self, period: float):
        while not self._stop.wait(period):
            self.lib.gpbs_ctl_heartbeat(self.ctl, self.page, time.monotonic_ns(), self._progress & 0xFFFFFFFF)

    def heartbeat(self):
        self.lib.gpbs_ctl_heartbeat(self.ctl, self.page, time.monotonic_ns(), self._progress & 0xFFFFFFFF)

    # ---------------------------------------------------------- assignment
    def assignment(self) -> Tuple[int, List[int], int]:
        """(gate, owned partition ids, epoch) -- one seqlock read."""
        m = (C.c_uint64 * 2)()
        ep = C.c_uint32(0)
        g = self.lib.gpbs_ctl_read_mask(self.ctl, self.page, m, C.byref(ep))
        ids = [i for i in range(128) if (m[i // 64] >> (i % 64)) & 1]
        return g, ids, ep.value

    def owned(self) -> List[Tuple[int, int]]:
        """(xcd, ctx) pairs of this tenant's GPU it currently holds."""
        _, ids, _ = self.assignment()
        return sorted({(x, c) for i in ids if i in self.part for (g, x, c) in [self.part[i]] if g == self.gpu})

    def gate(self, timeout_s: float = 10.0) -> bool:
        """Block until the scheduler lets this tenant launch (futex doorbell)."""
        rc = self.lib.gpbs_ctl_wait_gate(self.ctl, self.page, int(timeout_s * 1e9))
        if rc < 0:
            raise RuntimeError(f"wait_gate failed ({rc})")
        return rc == 1

    # ------------------------------------------------------------- streams
    def prepare_streams(self):
        """SE mode: create both class-half masked streams now, in a fixed
        order, before the tenant's own work creates queues (the queue set
        then no longer depends on which layout the first slices saw)."""
        import torch

        from ..ops import kernels as K
        for ses in ((0, 1), (2, 3)):
            if ("se",) + ses not in self._streams:
                self._streams[("se",) + ses] = torch.cuda.ExternalStream(
                    K.cumask_stream(se_cu_words(ses), device=self.gpu))

    def stream(self, owned: Optional[List[Tuple[int, int]]] = None):
        """torch stream masked to the CU halves this tenant holds.  The mask is
        quantised to {half 0, half 1, both} across all XCDs: a CU mask is a
        hardware-queue property, so every distinct mask costs a queue, and
        class placement keeps a tenant on one half anyway.  Co-resident
        contexts (``spatial=False``) always get the whole GPU, on a stream of
        the tenant's queue priority (``priority`` > 0: the command processor
        dispatches its workgroups ahead of normal-priority queues)."""
        import torch

        from ..ops import kernels as K
        parts = self.owned() if owned is None else owned
        if not parts:
            return torch.cuda.current_stream()
        if self.se_mode:  # exclusive shader engines: mask = the owned class half
            # Quantised to the class halves SEs {0,1} / {2,3}, as the native
            # runners do: every distinct CU mask is a hardware queue this
            # process keeps, and config #5 runs that saw five or six distinct
            # SE sets per tenant collapsed (profiles/llm5/config5_r3b_5rep.json).
            # A set that spans both halves runs unmasked (transitions only).
            #
            # One masked queue per tenant, on its class's home half only
            # (compute {0,1}, memory {2,3}: the budget layout's homes): two
            # processes that each moved their kernels from one CU-masked
            # queue to the other collapsed together -- decode 17 vs 5.7 ms per
            # step, the trainer 240 vs 188 ms -- and stayed collapsed on
            # disjoint masks, with no daemon at all (a static split that
            # starts on the swapped halves: profiles/llm5/config5_r3g_swap_nohwc.json).
            # A transitional layout (the tenant on the other class's half) and
            # a later class flip run unmasked instead.
            # A transitional set of three SEs runs on the half it holds whole
            # (round 6: run unmasked, it spread the decode tenant's kernels
            # over the trainer's SE for ~0.8 s of every config #5 start-up
            # while the two-tenant layout formed, profiles/r6/s37, s38).
            ses = {c for (_, c) in parts}
            if ses <= {0, 1}:
                ses = (0, 1)
            elif ses <= {2, 3}:
                ses = (2, 3)
            elif len(ses) == 3:
                ses = (0, 1) if {0, 1} <= ses else (2, 3)
            else:
                return torch.cuda.current_stream()
            if self.one_queue:
                cls = self.vpmu()["class"]
                home = (0, 1) if cls == 0 else (2, 3) if cls == 1 else None
                if home != ses or (self._home is not None and self._home != ses):
                    return torch.cuda.current_stream()
                self._home = ses
            if self.queue_probe > 1:
                pr = self._probers.get(ses)
                if pr is None:
                    pr = self._probers[ses] = QueueProber(self.queue_probe)
                    for i in range(self.queue_probe):  # all K at once: the set the prober chooses from
                        self._streams[("se",) + ses + (i,)] = torch.cuda.ExternalStream(
                            K.cumask_stream(se_cu_words(ses), device=self.gpu))
                self._probe_key = ses
                return self._streams[("se",) + ses + (pr.current(),)]
            s = self._streams.get(("se",) + ses)
            if s is None:
                s = torch.cuda.ExternalStream(K.cumask_stream(se_cu_words(ses), device=self.gpu))
                self._streams[("se",) + ses] = s
            return s
        halves = tuple(sorted({c for (_, c) in parts})) if self.spatial else (0, 1)
        if self.queue_probe > 1:  # K queues of this kind, the fastest by measurement (QueueProber)
            key = ("p",) + halves
            pr = self._probers.get(key)
            if pr is None:
                pr = self._probers[key] = QueueProber(self.queue_probe)
                for i in range(self.queue_probe):
                    if self.spatial:
                        h = K.cumask_stream(half_cu_words([(x, c) for x in range(XCDS) for c in halves]),
                                            device=self.gpu)
                        st = torch.cuda.ExternalStream(h)
                    else:
                        st = torch.cuda.Stream(device=self.gpu, priority=-1 if self.priority > 0 else 0)
                    self._streams[key + (i,)] = st
            self._probe_key = key
            return self._streams[key + (pr.current(),)]
        s = self._streams.get(halves)
        if s is None and not self.spatial:
            s = torch.cuda.Stream(device=self.gpu, priority=-1 if self.priority > 0 else 0)
            self._streams[halves] = s
        elif s is None:
            key = [(x, h) for x in range(XCDS) for h in halves]
            h = K.cumask_stream(half_cu_words(key), device=self.gpu)
            s = torch.cuda.ExternalStream(h)
            self._streams[halves] = s
        return s

    @contextlib.contextmanager
    def slice(self, timeout_s: float = 10.0):
        """Wait for the gate, mark the tenant busy, run the body on the
        tenant's CU-masked stream."""
        import torch
        self.busy()
        t0 = time.monotonic_ns()
        if not self.gate(timeout_s):
            raise TimeoutError(f"tenant {self.name}: gate closed for {timeout_s}s")
        waited = time.monotonic_ns() - t0
        self._probe_key = None
        s = self.stream()
        key = self._probe_key
        # A slice may land on another queue than the previous one (a layout
        # change, or the QueueProber rotating same-mask queues): nothing
        # orders two HIP queues, so the new one first waits for the old one's
        # work -- a body that does not end synchronised must not have its
        # kernels overtaken by the next slice's.
        prev = self._last_stream
        if prev is not None and s != prev:
            s.wait_stream(prev)
        t1 = time.perf_counter()
        with torch.cuda.stream(s):
            yield s
        if key is not None:
            # the prober compares queues by slice time: time the GPU work,
            # not its launch (the decode / training bodies end synchronised,
            # so this costs them nothing)
            s.synchronize()
            self._probers[key].record(1e3 * (time.perf_counter() - t1))
        self._last_stream = s
        self._progress += 1
        if waited > 0:
            self.report_wait(waited)

    # ------------------------------------------------------------- signals
    def busy(self):
        self.lib.gpbs_ctl_set_work(self.ctl, self.page, 1)

    def idle(self):
        self.lib.gpbs_ctl_set_work(self.ctl, self.page, 0)

    def report_wait(self, ns: int, gpu: Optional[int] = None):
        return self.lib.gpbs_ctl_report(self.ctl, self.page, int(ns), REPORT_WAIT, self.gpu if gpu is None else gpu)

    def wait_probe(self, min_report_ns: int = 2000):
        """K10 producer bound to this tenant's report ring: time RCCL
        collectives and stream/event syncs, post the waits (waitprobe.py)."""
        from .waitprobe import WaitProbe
        return WaitProbe(self.report_wait, min_report_ns=min_report_ns)

    def report_hold(self, ns: int):
        return self.lib.gpbs_ctl_report(self.ctl, self.page, int(ns), REPORT_HOLD, self.gpu)

    def report_requests(self, n: int = 1):
        return self.lib.gpbs_ctl_report(self.ctl, self.page, int(n), REPORT_REQUESTS, self.gpu)

    def account(self, flops: float = 0.0, bytes_moved: float = 0.0, busy_ns: int = 0, l2_bytes: float = 0.0):
        """Publish modeled counters (cumulative): instructions ~ MFMA issues,
        cycles ~ busy time, L2 references ~ lines touched, misses ~ HBM lines."""
        c = self.counters
        c[0] += int(flops / FLOP_PER_INST) + 1
        c[1] += int(busy_ns * 2.4)  # ~2.4 GHz shader clock
        c[2] += int((l2_bytes or bytes_moved) / LINE)
        c[3] += int(bytes_moved / LINE)
        arr = (C.c_uint64 * 4)(*c)
        self.lib.gpbs_ctl_set_counters(self.ctl, self.page, arr)

    def vpmu(self) -> dict:
        """The tenant's virtualized PMU as the scheduler sees it (control-page
        mirror, one seqlock read -- the Perfctr-xen guest read of its
        per-vCPU state page, L:drivers/perfctr/x86.c:252-277): cumulative
        INST / CYCLES / LLC refs / LLC misses the scheduler measured and
        attributed to this tenant (live hardware counters when the daemon runs
        them), last period's miss rate, current quantum, class and phase."""
        c4 = (C.c_uint64 * 4)()
        mr, ts, cls, ph, seq = C.c_uint64(0), C.c_uint32(0), C.c_int32(0), C.c_uint32(0), C.c_uint32(0)
        retries = self.lib.gpbs_ctl_read_vpmu(self.ctl, self.page, c4, C.byref(mr), C.byref(ts), C.byref(cls),
                                              C.byref(ph), C.byref(seq))
        if retries < 0:
            raise RuntimeError(f"read_vpmu failed ({retries})")
        return {"inst": c4[0], "cycles": c4[1], "l2_refs": c4[2], "l2_misses": c4[3], "miss_rate": mr.value,
                "tslice_us": ts.value, "class": cls.value, "phase": ph.value, "updates": seq.value,
                "retries": retries}

    # ------------------------------------------------------------ teardown
    def close(self, destroy: bool = True):
        if self._stop.is_set():
            return
        self._stop.set()
        self._hb.join(timeout=1.0)
        try:
            self.idle()
            self.rpc.call("unregister", name=self.name, destroy=destroy)
        except Exception:
            pass
        self.lib.gpbs_ctl_close(self.ctl, 0)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def run_synthetic(name: str, socket_path: str, seconds: float, result_q=None, slots: int = 4,
                  crash: bool = False, flops: float = 1e9, bytes_moved: float = 1e6):
    """A synthetic tenant loop (no GPU needed): gate, report, account, repeat.
    ``crash`` exits without unregistering (failure-detection test)."""
    t = TenantClient(name, socket_path, slots=slots)
    t.busy()
    opens = loops = 0
    t_end = time.monotonic() + seconds
    while time.monotonic() < t_end:
        t0 = time.monotonic_ns()
        if t.gate(timeout_s=0.5):
            opens += 1
        t.report_wait(time.monotonic_ns() - t0 + 1)
        t.report_hold(500)
        t.report_requests(1)
        t.account(flops=flops, bytes_moved=bytes_moved, busy_ns=100_000)
        loops += 1
        time.sleep(0.001)
    if crash:
        os._exit(0)
    time.sleep(0.01)  # one more metric period + mirror publication
    info = {"name": name, "tenant": t.tenant, "opens": opens, "loops": loops, "owned_seen": t.owned(),
            "declared": list(t.counters), "vpmu": t.vpmu()}
    t.close(destroy=False)
    if result_q is not None:
        result_q.put(info)
    return info


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="gpbs synthetic tenant")
    ap.add_argument("--name", required=True)
    ap.add_argument("--socket", default=DEFAULT_SOCKET)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--slots", type=int, default=4)
    a = ap.parse_args(argv)
    print(run_synthetic(a.name, a.socket, a.seconds, slots=a.slots))


if __name__ == "__main__":
    main()
