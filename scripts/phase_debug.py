"""Timeline of the live phase-change test (tests/test_gpu_phase.py) for
debugging: the same three tenants (GEMM, phase GEMM<->stream, HBM stream)
under the counter-driven SE budgets, with one row per poll -- units done,
owner waits, budget masks, the first XCD's owners, the runners' masked-queue
indexes, classes and miss rates.  Found the ~100 ms freeze of every runner at
the first SE-exclusive relayout (the lazy masked-queue burst,
profiles/r6/phase_debug_summary.txt).

    python scripts/phase_debug.py <repo root> <align 0|1>   (prints RESULT {json})
"""
import json
import sys
import time

ROOT = sys.argv[1]
ALIGN = int(sys.argv[2])
sys.path.insert(0, ROOT)

from pbs_amd.counters import hwc  # noqa: E402

assert hwc.init()
import torch  # noqa: E402

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
assert hwc.start()
from pbs_amd.bench.corun import BUDGET_OVERRIDES  # noqa: E402
from pbs_amd.core.config import MI355X_PROFILE  # noqa: E402
from pbs_amd.core.engine import Engine  # noqa: E402
from pbs_amd.runtime.gpu import GpuContext, Runner  # noqa: E402

prof = dict(MI355X_PROFILE)
prof.update(BUDGET_OVERRIDES)
e = Engine(**prof)
for x in range(8):
    for c in range(4):
        e.pool_assign(0, e.partition_add(0, x, c))
e.tenant_create("Domain-0", nslots=1)
g = e.tenant_create("gemm", nslots=32)
p = e.tenant_create("phase", nslots=32)
s = e.tenant_create("hbm", nslots=32)
ctx = GpuContext(0, nctx=4, table_mode="device")
ctx.set_se_mode(True)
ctx.attach(e, nctx=4)
ctx.set_hwc_sampler(align=ALIGN)
ctx.set_hwc(True)
e.start()
rg = Runner(ctx, "gemm", g, M=4096, N=4096, K=4096)
rp = Runner(ctx, "gemm", p, M=4096, N=4096, K=4096, alt=dict(kind="stream", bytes=1 << 30))
rs = Runner(ctx, "stream", s, bytes=1 << 30)
runners = (rg, rp, rs)
tids = (("gemm", g), ("phase", p), ("hbm", s))


def topup():
    for r, q in ((rg, 400), (rp, 400), (rs, 100)):
        st = r.stats()
        if st.submitted - st.units_done < q:
            r.submit(q)


def info():
    return {n: (e.lib.gpbs_tenant_class(e.h, t), e.tenant_info(t).budget_ctx) for n, t in tids}


TL = []
T00 = time.perf_counter()


def run_until(pred, limit_s):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < limit_s:
        topup()
        i = info()
        st = [r.stats() for r in runners]
        TL.append([round((time.perf_counter() - T00) * 1e3, 1)] + [x.units_done for x in st] +
                  [x.waits_owner for x in st] + [i[n][1] for n, _ in tids] + [ctx.owners()[:4]] +
                  [[ctx.L.gpbs_runner_queue(r.h) for r in runners]] + [[i[n][0] for n, _ in tids]] +
                  [[e.tenant_info(t).cache_miss_rate for _, t in tids]])
        if pred(i):
            return (time.perf_counter() - t0) * 1e3
        time.sleep(0.001)
    return -1.0


def compute_layout(i):
    return i["phase"][0] == 0 and i["phase"][1] in (1, 2) and i["gemm"][1] in (1, 2) and i["hbm"][1] == 12


def memory_layout(i):
    return i["phase"][0] == 1 and i["phase"][1] in (4, 8) and i["gemm"][1] == 3 and i["hbm"][1] in (4, 8)


out = {"metric_period_us": prof["metric_period_us"]}
out["settle_ms"] = run_until(compute_layout, 5.0)
e.perfc_reset()
rp.set_phase(1)
out["to_memory_ms"] = run_until(memory_layout, 3.0)
rp.set_phase(0)
out["to_compute_ms"] = run_until(compute_layout, 3.0)
out["hwc"] = ctx.hwc_stats()
for r in runners:
    r.cancel()
for r in runners:
    r.wait(120)
e.stop()
out["check"] = e.check()
for r in runners:
    r.close()
ctx.close()
e.close()
out["tl"] = TL
print("RESULT " + json.dumps(out))
