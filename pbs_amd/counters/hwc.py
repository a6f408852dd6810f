"""Live CDNA4 hardware counters (rocprofiler-sdk device counting service,
csrc/hip/hwc.cpp): the Perfctr-xen vPMU analog.

    from pbs_amd.counters import hwc
    hwc.init()            # BEFORE the HIP runtime initialises (first torch.cuda call)
    torch.cuda.set_device(0)
    hwc.start()
    per_xcd = hwc.sample()   # 8 x (INST, BUSY_CYCLES, L2_REQ, L2_MISS), cumulative

``GpuContext.set_hwc(True)`` then drives the scheduler's PBS metric with
hardware deltas attributed to tenants by partition OWNERSHIP: exact per
shader engine in the SE-exclusive mode, by owned time per XCD otherwise
(csrc/hip/runtime.cpp, hwc_attribute).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Tuple

from .. import _native as N

# PBS slots INST | CYCLES | LLC_REFS | LLC_MISSES on gfx950 (csrc/hip/hwc.cpp):
# SQ/TCP counters resolve per shader engine, TCC per XCD.
# "lean": 5 SQ + 1 TCP + 1 TCC counters.  A device-
# counting sample's cost grows with the counter RECORDS it returns (SQ: one per
# SE, TCP: one per CU, TCC: one per channel) and the memory-path (TCC) ones
# perturb the tenants most; measured with a backlogged GEMM alone
# (scripts/hwc_cost.py, profiles/r3/hwc_cost_gemm_r3a.jsonl): the round-2 "full"
# set (7 SQ + 2 TCP + 1 TCC) costs 3.9 % of the GEMM's throughput at a 1 ms
# period (324 us per sample), a 2 SQ + 1 TCP + 1 TCC set 0.75 % (188 us).
LEAN_SPEC = ("SQ_INSTS_VALU+SQ_INSTS_VMEM_RD+SQ_INSTS_VMEM_WR+SQ_INSTS_VALU_MFMA_MOPS_BF16|SQ_BUSY_CYCLES|"
             "TCP_TCC_READ_REQ|TCC_MISS")
FULL_SPEC = ("SQ_INSTS_VALU+SQ_INSTS_SALU+SQ_INSTS_VMEM_RD+SQ_INSTS_VMEM_WR+SQ_INSTS_LDS+"
             "SQ_INSTS_VALU_MFMA_MOPS_BF16|SQ_BUSY_CYCLES|"
             "TCP_TCC_READ_REQ+TCP_TCC_WRITE_REQ|TCC_MISS")
# "lean2": L2 request shares from SQ memory instructions (per SE) instead of
# TCP requests (per CU): 6 SQ + 1 TCC counters, no TCP
LEAN2_SPEC = ("SQ_INSTS_VALU+SQ_INSTS_SALU+SQ_INSTS_VALU_MFMA_MOPS_BF16|SQ_BUSY_CYCLES|"
              "SQ_INSTS_VMEM_RD+SQ_INSTS_VMEM_WR|TCC_MISS")
SPECS = {"lean": LEAN_SPEC, "full": FULL_SPEC, "lean2": LEAN2_SPEC}
# Measured on one MI355X, 4-tenant mix, gpbs vs the same layout without a
# sampler (profiles/r3/cmp_4mix_*.json, README "Sampler cost"): lean at 1 ms -5 %, lean at 4 ms
# -0.5 %, lean2 at 1 ms -2 % (131 us per sample).  Default: lean2, with the
# runtime's duty-cycle cap stretching the period to ~20 sample times.
# The PBS thresholds (pbs_amd/core/config.py, miss-rate threshold 2e4 per 1e5
# instructions) were re-checked against lean2's INST definition (no VMEM /
# LDS terms) on the round-4 8mix (profiles/r4/): hardware miss rates GEMM
# ~2.4e3, HBM stream ~1.0e5, reduce-copy ~4.4e4 -- an order of magnitude on
# either side of the threshold, the classes unchanged.
DEFAULT_SPEC = LEAN2_SPEC
XCDS = 8


def _lib():
    return N.load_hip(required=True)


def init(spec: Optional[str] = None, gpu: int = -1) -> bool:
    """Register the sampler with rocprofiler-sdk; must precede HIP init.
    ``spec``: a counter spec, a name in SPECS, or None (GPBS_HWC_SPEC, else
    DEFAULT_SPEC = lean2).  ``gpu`` >= 0 (LOCAL_RANK) is a cross-check only: the
    counted agent is the one at the current HIP device's PCI address (agent())."""
    import os
    spec = spec or os.environ.get("GPBS_HWC_SPEC") or DEFAULT_SPEC
    spec = SPECS.get(spec, spec)
    return _lib().gpbs_hwc_init_gpu(spec.encode(), int(gpu)) == 0


def trace_enable(on: bool = True) -> bool:
    """In-process kernel trace (rocprofiler-sdk kernel-dispatch records in
    this tool's own context, so it runs WITH the live counters -- rocprofv3
    cannot: its tool takes the SDK and the scheduler falls back to modeled
    counters).  Call before init()."""
    return bool(_lib().gpbs_hwc_trace_enable(1 if on else 0))


def trace_stats(reset: bool = False) -> Optional[dict]:
    """Per-kernel GPU time since the last reset: {"dispatches", "dropped",
    "span_ns", "kernels": [[name, calls, total_ns, max_ns], ...]} by total
    time; None if the trace is not running."""
    import json
    cap = 1 << 16
    for _ in range(4):
        buf = C.create_string_buffer(cap)
        n = _lib().gpbs_hwc_trace_stats(buf, cap, 1 if reset else 0)
        if n == -1:
            return None
        if n >= 0:
            return json.loads(buf.value.decode())
        cap = -n + 1024
    return None


def start() -> bool:
    """Start counting on the current HIP device's agent.  False if the
    service is not configured; raises if the configured agent (LOCAL_RANK)
    is not at this device's PCI address -- counting a neighbour's GPU is
    worse than not counting."""
    rc = _lib().gpbs_hwc_start()
    if rc == -3:
        raise RuntimeError("hardware counters: the configured rocprofiler agent is not at the current HIP "
                           "device's PCI address (LOCAL_RANK / visible-device mismatch)")
    return rc == 0


def active() -> bool:
    return bool(_lib().gpbs_hwc_active())


def sample() -> List[Tuple[int, int, int, int]]:
    arr = (C.c_uint64 * (XCDS * 4))()
    if _lib().gpbs_hwc_sample(arr, XCDS) < 0:
        raise RuntimeError("hardware counter sample failed (init/start?)")
    return [tuple(arr[x * 4:(x + 1) * 4]) for x in range(XCDS)]


def sample_se():
    """Cumulative counters per (XCD, SE) for the SE-resolved slots and per
    XCD for all: ([8][4][4], [8][4])."""
    se, xs = (C.c_uint64 * (XCDS * 4 * 4))(), (C.c_uint64 * (XCDS * 4))()
    if _lib().gpbs_hwc_sample_se(se, xs) < 0:
        raise RuntimeError("hardware counter sample failed (init/start?)")
    return ([[tuple(se[(x * 4 + e) * 4:(x * 4 + e + 1) * 4]) for e in range(4)] for x in range(XCDS)],
            [tuple(xs[x * 4:(x + 1) * 4]) for x in range(XCDS)])


def stop():
    _lib().gpbs_hwc_stop()


def agent() -> dict:
    """The GPU agent the counting context was started on: chosen by the PCI
    address of the current HIP device (hwc.cpp gpbs_hwc_start), with its
    enumeration index and whether LOCAL_RANK named another one."""
    buf = C.create_string_buffer(32)
    mm = C.c_int(0)
    idx = _lib().gpbs_hwc_agent(buf, 32, C.byref(mm))
    return {"agent_index": int(idx), "bdf": buf.value.decode() or None, "index_mismatch": bool(mm.value)}
