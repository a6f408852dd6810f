"""GPU runtime tests: native runners under the engine-driven partition table."""
import time

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from pbs_amd.core.engine import Engine  # noqa: E402
from pbs_amd.runtime.gpu import GpuContext, Runner  # noqa: E402


def _engine(sched="credit", **kw):
    e = Engine(sched=sched, **kw)
    for x in range(8):
        e.pool_assign(0, e.partition_add(0, x))
    e.tenant_create("Domain-0", nslots=1)
    return e


def test_backlogged_tenants_share_by_weight():
    """Weight 512 vs 256, both backlogged on all 8 partitions: the credit
    scheduler gives the heavier tenant ~2x the partition time (csched_acct
    fair share, X:xen/common/sched_credit.c:1302-1519)."""
    e = _engine()
    e.sched_params_set(0, 1000, 100)
    a = e.tenant_create("gemm", nslots=8)
    b = e.tenant_create("hbm", nslots=8, weight=512)
    ctx = GpuContext(0, e)
    e.start()
    ra = Runner(ctx, "gemm", a, M=2048, N=2048, K=2048)
    rb = Runner(ctx, "stream", b, bytes=64 << 20)
    ra.submit(1 << 20)
    rb.submit(1 << 20)
    time.sleep(0.3)
    a0, b0 = e.tenant_info(a).run_ns, e.tenant_info(b).run_ns
    time.sleep(1.0)
    a1, b1 = e.tenant_info(a).run_ns, e.tenant_info(b).run_ns
    ra.cancel()
    rb.cancel()
    ra.wait(60)
    rb.wait(60)
    e.stop()
    ratio = (b1 - b0) / max(1, a1 - a0)
    assert 1.6 <= ratio <= 2.5, ratio
    assert ra.stats().units_done > 0 and rb.stats().units_done > 0
    for r in (ra, rb):
        r.close()
    ctx.close()
    e.close()


def test_runners_complete_under_gpbs():
    e = _engine()
    a = e.tenant_create("gemm", nslots=8)
    b = e.tenant_create("hbm", nslots=8, weight=512)
    ctx = GpuContext(0, e)
    e.start()
    ra = Runner(ctx, "gemm", a, M=2048, N=2048, K=2048)
    rb = Runner(ctx, "stream", b, bytes=256 << 20)
    ra.submit(40)
    rb.submit(40)
    ra.wait(120)
    rb.wait(120)
    e.stop()
    assert ra.stats().units_done == 40 and rb.stats().units_done == 40
    ia, ib = e.tenant_info(a), e.tenant_info(b)
    assert ia.run_ns > 0 and ib.run_ns > 0
    # counters flowed through the device metric path
    assert ctx.stats()["metric_calls"] > 0
    assert e.perfc()["metric_tick"] > 0
    assert ctx.read_counters(a)[0] > 0 and ctx.read_counters(b)[3] > 0
    assert e.check() == ""
    for r in (ra, rb):
        r.close()
    ctx.close()
    e.close()


def test_revocation_relaunch_completes_all_units():
    """Ownership flips every 200us while a GEMM runs: units are revoked
    mid-flight and resumed, and the result stays exact."""
    ctx = GpuContext(0)
    r = Runner(ctx, "gemm", 3, engine_wake=False, M=2048, N=2048, K=2048)
    stop = False
    import threading

    def flipper():
        i = 0
        while not stop:
            ctx.set_owners([3 if (x + i) % 2 == 0 else -1 for x in range(8)] if i % 3 else [-1] * 8)
            i += 1
            time.sleep(200e-6)
        ctx.set_owners([3] * 8)

    th = threading.Thread(target=flipper)
    th.start()
    r.submit(20)
    try:
        r.wait(120)
    finally:
        stop = True
        th.join()
    st = r.stats()
    assert st.units_done == 20
    a, b, c = r.buffers
    ref = a.float() @ b.float().t()
    assert (c.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    r.close()
    ctx.close()


def test_static_split_runs_concurrently():
    ctx = GpuContext(0)
    ctx.set_owners([1, 1, 1, 1, 2, 2, 2, 2])
    r1 = Runner(ctx, "gemm", 1, engine_wake=False, M=2048, N=2048, K=2048)
    r2 = Runner(ctx, "stream", 2, engine_wake=False, bytes=256 << 20)
    r1.submit(10)
    r2.submit(10)
    r1.wait(60)
    r2.wait(60)
    per1 = ctx.read_counters(1, per_xcd=True)
    per2 = ctx.read_counters(2, per_xcd=True)
    assert all(per1[x][0] == 0 for x in range(4, 8)) and all(per2[x][0] == 0 for x in range(4))
    r1.close()
    r2.close()
    ctx.close()


def _se(hwid):
    return (int(hwid) >> 13) & 7


def test_half_cu_mask_stream_confines_workgroups_to_one_half():
    from pbs_amd.ops import kernels as K
    for h in (0, 1):
        s = K.cumask_stream(K.half_cu_mask(h))
        out = K.census(1024, stream=s).cpu()
        torch.cuda.synchronize()
        K.lib().gpbs_gpu_stream_destroy(__import__("ctypes").c_void_p(s))
        assert (out[:, 3] == 0xC0FFEE).all()
        ses = {_se(v) for v in out[:, 1].tolist()}
        assert ses and all(se >> 1 == h for se in ses), (h, ses)
        assert len({int(x) for x in out[:, 0].tolist()}) == 8  # every XCD still used


def test_spatial_gate_follows_the_cu_half():
    from pbs_amd.ops import kernels as K
    ctx = GpuContext(0, None, nctx=2)
    ctx.set_spatial(True)
    # XCDs 0-5: tenant 1 on half 0, tenant 2 on half 1 (split); XCDs 6-7:
    # tenant 1 alone (unsplit: it gets the whole XCD)
    ctx.set_owners([t for x in range(6) for t in (1, 2)] + [1, -1, 1, -1])
    for me, half in ((1, 0), (2, 1)):
        out = K.census(2048, table=ctx.table, tenant=me, spatial=True).cpu()
        for xcc, hw, ok, magic in out.tolist():
            assert magic == 0xC0FFEE
            if xcc < 6:
                assert bool(ok) == ((_se(hw) >> 1) == half), (me, xcc, hex(hw))
            else:
                assert bool(ok) == (me == 1), (me, xcc)
    assert ctx.owners()[:2] == [1, 2]  # split bit hidden from readers
    ctx.close()


def test_four_context_table_gates_each_context():
    """kCtx = 4 co-resident issue contexts per XCD: a tenant holding only
    context c of XCD x runs there and nowhere else, for every c."""
    from pbs_amd.ops import kernels as K
    ctx = GpuContext(0, None, nctx=4)
    owners = [-1] * 32
    for x in range(8):
        owners[4 * x + (x % 4)] = 10 + (x % 4)  # tenant 10+c on context c of XCDs c and c+4
    ctx.set_owners(owners)
    assert ctx.owners() == owners
    for c in range(4):
        out = K.census(2048, table=ctx.table, tenant=10 + c).cpu()
        for xcc, _hw, ok, magic in out.tolist():
            assert magic == 0xC0FFEE
            assert bool(ok) == (xcc % 4 == c), (c, xcc)
    ctx.close()


def test_bar_table_gates_runners_and_census():
    """Table mode 'bar' (VRAM table written by the host through the BAR):
    a static XCD split confines each runner to its XCDs, and the census
    kernel reads the owners the host stored."""
    from pbs_amd.ops import kernels as K
    ctx = GpuContext(0, table_mode="bar")
    assert ctx.table_mode() == "bar"
    ctx.set_owners([1, 1, 1, 1, 2, 2, 2, 2])
    out = K.census(2048, table=ctx.table, tenant=2).cpu()
    for xcc, _hw, ok, magic in out.tolist():
        assert magic == 0xC0FFEE
        assert bool(ok) == (xcc >= 4), xcc
    r1 = Runner(ctx, "gemm", 1, engine_wake=False, M=2048, N=2048, K=2048)
    r2 = Runner(ctx, "stream", 2, engine_wake=False, bytes=256 << 20)
    r1.submit(10)
    r2.submit(10)
    r1.wait(60)
    r2.wait(60)
    per1 = ctx.read_counters(1, per_xcd=True)
    per2 = ctx.read_counters(2, per_xcd=True)
    assert all(per1[x][0] == 0 for x in range(4, 8)) and all(per2[x][0] == 0 for x in range(4))
    assert any(per1[x][0] > 0 for x in range(4)) and any(per2[x][0] > 0 for x in range(4, 8))
    r1.close()
    r2.close()
    ctx.close()


def test_hold_word_pauses_gate_hold_kernels_bounded():
    """GATE_HOLD: a kernel waits (bounded, ~0.25 ms per unit grab) while the
    table's hold word is set, and runs at full speed once it is cleared; the
    data is copied either way."""
    from pbs_amd.ops import kernels as K
    ctx = GpuContext(0, table_mode="bar")
    ctx.set_owners([5] * 8)
    x = torch.randn(1 << 20, device="cuda")
    y = torch.empty_like(x)

    def timed(hold):
        ctx.L.gpbs_gpu_force_hold(ctx.h, 1 if hold else 0)
        y.zero_()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.stream_copy(x, y, chunk_bytes=1 << 16, table=ctx.table, tenant=5, grid=64,
                      mode_extra=K.GATE_DEVTABLE | K.GATE_HOLD)
        e1.record()
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        return e0.elapsed_time(e1)

    timed(False)  # warm-up
    off = min(timed(False) for _ in range(3))
    on = timed(True)
    ctx.L.gpbs_gpu_force_hold(ctx.h, 0)
    after = min(timed(False) for _ in range(3))
    assert on > off + 0.2, (on, off)   # every grab waited out the bounded hold
    assert on < 20.0, on               # bounded: a stuck hold word cannot stall a tenant
    assert after < off + 0.1, (after, off)
    ctx.close()
