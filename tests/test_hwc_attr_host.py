"""The host attribution algorithm (csrc/hip/hwc_attr.h hwc_attr_host, the
oracle k_hwc_attribute is checked against on the GPU) on CPU: on 200 random
snapshot pairs -- owned, time-shared and idle partitions, idle whole XCDs,
three slot layouts, co-resident mode, clean windows on and off, class-share
intervals -- every counter slot's attributed counts plus its unexplained
counts equal the hardware sum, and no tenant's clean (metric) part exceeds
its attributed part."""
import ctypes as C

import pytest


def test_attribution_conserves_counts():
    from pbs_amd.ops import kernels as K
    try:
        L = K.lib()
    except Exception as ex:  # pragma: no cover - the HIP library must build here
        pytest.fail(f"libgpbs_hip.so: {ex}")
    out = (C.c_double * 2)()
    for seed in (1, 7, 42):
        assert L.gpbs_hip_hwc_attr_host_check(seed, 200, out) == 0
        assert out[0] < 1e-12, (seed, out[0])  # attributed + unexplained == hardware sum
        assert out[1] < 1e-12, (seed, out[1])  # clean part <= attributed part


def test_masked_queue_pool_policy():
    """The process-wide CU-masked queue pool (csrc/hip/runtime.cpp
    MaskedPoolCore) on fake handles: co-sharers of one layout share a queue,
    concurrent layouts on one mask each get their own below the budget, an
    exclusive acquire never lands on another key's queue, idle queues are
    re-keyed before new ones are made, masks and devices never mix, and past
    the budget a share across keys happens and is counted."""
    from pbs_amd.ops import kernels as K
    assert K.lib().gpbs_hip_masked_pool_selftest() == 0


def test_metric_fold_calibrated_fallback_keeps_the_class():
    """The PBS metric fold (csrc/hip/runtime.cpp hwc_fold, host only): a
    tenant whose modeled counters are off by 24x / 0.13x alternates between
    clean hardware windows and stale unclean periods; the fallback, scaled by
    its hardware/model ratio, delivers the hardware miss rate within 10 %, so
    its class holds.  Uncalibrated or fresh unclean periods are skipped and
    the edge of another tenure (a sliver) never counts."""
    from pbs_amd.ops import kernels as K
    assert K.lib().gpbs_hip_hwc_fold_selftest() == 0
    assert K.lib().gpbs_hip_hwc_fold_selftest() == 0  # a second call in the same process (fresh context)


def test_drained_bit_needs_the_opening_owner_to_be_the_clean_one():
    """The drained bit of a clean window (csrc/hip/hwc_attr.h
    hwc_drained_bits): set only when the partition's owner at the
    interval's first sample had held it a drain guard AND no owner change
    landed in the interval's first (100 - clean_pct) %, so a tenant that takes
    a partition over at the head of an interval never gets a clean window
    holding its predecessor's head and drain; a switch-aligned close (the
    change one guard before the closing sample) keeps its window."""
    from pbs_amd.ops import kernels as K
    for seed in (1, 5, 9):
        assert K.lib().gpbs_hip_hwc_drained_selftest(seed, 2000) == 0


def test_kernel_trace_is_off_unless_enabled_before_init():
    """The in-process kernel trace (csrc/hip/hwc.cpp Trace) only exists when
    enabled before the counter tool registers: here (no rocprofiler-sdk
    configuration in this process) its statistics read back as not running,
    and bench.py carries the switch into the co-run config."""
    from pbs_amd.bench.corun import CorunConfig
    from pbs_amd.counters import hwc
    assert hwc.trace_stats() is None
    assert CorunConfig().kernel_trace is False


def test_one_ms_cadence_from_the_calibrated_model_keeps_the_class():
    """The 1 ms metric cadence (csrc/hip/runtime.cpp cadence_tick, VERDICT r5
    item 3): between clean hardware windows 10 ms apart, every metric tick
    reports the tenant's modeled deltas x its hardware/model ratio -- the
    hardware miss rate within 10 %, so its class holds with ten times the
    metric periods; a calibrated tenant's clean window only re-anchors the
    ratio (nothing reported twice); a phase change in the model crosses the
    class threshold at the next tick."""
    from pbs_amd.ops import kernels as K
    assert K.lib().gpbs_hip_hwc_cadence_selftest() == 0
