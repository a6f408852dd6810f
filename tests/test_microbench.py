"""Perf-regression gates on the scheduler path (the analog
of L:drivers/perfctr/x86_tests.c:181-245).  Thresholds live in
scripts/microbench.py (about 3x the committed profiles/micro/microbench_r2.json)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("microbench", os.path.join(ROOT, "scripts", "microbench.py"))
MB = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MB)


def test_gang_epoch_barrier_latency():
    """Native shm gang epoch among 4 node-local ranks, back to back.  The
    ranks busy-poll: the gate is a latency bound only on a host with 4 idle
    CPUs (it is skipped when other work -- pytest -n -- occupies them)."""
    ncpu = len(os.sched_getaffinity(0))
    if ncpu < 4 or os.getloadavg()[0] > ncpu - 4:
        pytest.skip(f"host busy (load {os.getloadavg()[0]:.1f} on {ncpu} CPUs): latency gate not meaningful")
    # a preempted poller shows up as a p99 outlier: one re-measurement before
    # the gate fails (the p50 gate is what a real regression moves)
    for attempt in range(2):
        res = MB.bench_gang(worlds=(4,), iters=2000, gloo=False)
        g = MB.gates({"gang": res})
        if all(ok for _, _, ok in g.values()):
            break
    for k, (v, lim, ok) in g.items():
        assert ok, (k, v, lim, res)


@pytest.mark.gpu
def test_switch_actuation_latency():
    """Publish -> every workgroup of a 1024-workgroup grid observed the new
    epoch, host and device partition tables."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = MB.bench_switch(iters=200)
    for mode in ("host", "device", "bar"):
        assert res[mode]["n"] == 200, res
    g = MB.gates({"switch": res})
    for k, (v, lim, ok) in g.items():
        assert ok, (k, v, lim, res)


@pytest.mark.gpu
def test_counter_read_latency():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = MB.bench_hwc(iters=100)
    g = MB.gates({"hwc": res})
    for k, (v, lim, ok) in g.items():
        assert ok, (k, v, lim, res)
