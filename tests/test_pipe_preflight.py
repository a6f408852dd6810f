"""Masked-queue pipe pre-flight (pbs_amd/utils/pipes.py)
on a fake library and fake KFD queue lists: a burst that took one
contiguous run of queue ids and follows the plan passes; a foreign queue
created in the middle of the burst (RCCL or the profiler making one on
another thread), a plan whose compute and memory queues share a pipe, or a
library error fail the rank; a pool made before the check reports no
comparison instead of a failure."""
import ctypes as C

from pbs_amd.bench.report import ranks_digest
from pbs_amd.utils.pipes import PLAN, check_burst, pipe_preflight


class FakeLib:
    def __init__(self, entries, rc=None):
        self.entries, self.rc = entries, rc

    def gpbs_hip_masked_pool_prealloc(self, device, out, mx):
        if self.rc is not None:
            return self.rc
        for i, e in enumerate(self.entries[:mx]):
            out[i] = e
        return len(self.entries)


def _plan_entries(plan=PLAN):
    return [(i % 4) | (h << 8) for i, h in enumerate(plan)]


def _qids(seq):
    it = iter(seq)
    return lambda: next(it)


def test_contiguous_burst_after_rccl_queues_passes():
    before = list(range(0, 14))  # 12 plain-stream queues + RCCL's two
    after = before + list(range(14, 24))
    rec = pipe_preflight(FakeLib(_plan_entries()), 0, _qids([before, after]))
    assert rec["ok"] and rec["contiguous"] and rec["plan_ok"] and rec["pipes_disjoint"], rec
    assert rec["new_kfd_queues"] == 10 and rec["compute_pipes"] == [0] and rec["memory_pipes"] == [1, 2, 3]


def test_foreign_queue_inside_the_burst_fails_the_rank():
    before = list(range(0, 14))
    after = before + list(range(14, 19)) + list(range(20, 25))  # id 19 went to another thread's queue
    rec = pipe_preflight(FakeLib(_plan_entries()), 0, _qids([before, after + [19]]))
    assert rec["new_kfd_queues"] == 11 and rec["contiguous"] is False and not rec["ok"], rec
    d = ranks_digest([{"rank": 0, "pipes": rec}, {"rank": 1, "pipes": {"ok": True}}])
    assert d["failures"] == [{"rank": 0, "why": ["pipes"]}]


def test_plan_with_a_shared_pipe_fails():
    bad = list(PLAN)
    bad[1] = 0  # a compute-half queue on pipe 1, which the memory half also uses
    rec = check_burst(list(range(4)), list(range(14)), _plan_entries(bad))
    assert not rec["plan_ok"] and not rec["pipes_disjoint"] and not rec["ok"], rec


def test_library_error_and_earlier_pool():
    assert pipe_preflight(FakeLib([], rc=-12), 0, _qids([[1], [1]])) == {"ok": False, "error": -12}
    rec = pipe_preflight(FakeLib(_plan_entries()), 0, _qids([list(range(30)), list(range(30))]))
    assert rec["ok"] and rec["contiguous"] is None and rec["new_kfd_queues"] is None, rec
    rec = pipe_preflight(FakeLib(_plan_entries()), 0, _qids([None, None]))  # sysfs not exposed
    assert rec["ok"] and rec["contiguous"] is None
