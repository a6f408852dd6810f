"""The IPC all-reduce tenant's setup fails on every rank together
(pbs_amd/parallel/ipc_coll.py): a rank whose buffer export fails still makes
both exchanges of the setup, so its peers never wait in a collective it
skipped (the round-5 8-rank rehearsal hung when one rank raised before the
handle exchange and went on to the caller's next collective).  Two ranks on
threads with a fake HIP library and an in-process exchange."""
import threading

import pytest


class _FakeLib:
    def __init__(self, fail_create_rank=-1, fail_open_rank=-1):
        self.fail_create_rank, self.fail_open_rank = fail_create_rank, fail_open_rank
        self.destroyed = []

    def gpbs_coll_create(self, device, rank, world, nbytes):
        return 0 if rank == self.fail_create_rank else 100 + rank

    def gpbs_coll_handle_bytes(self):
        return 8

    def gpbs_coll_export(self, h, buf):
        for i in range(8):
            buf[i] = b"x"
        return 8

    def gpbs_coll_open(self, h, peer, arr):
        return 5 if (h.value - 100) == self.fail_open_rank else 0

    def gpbs_coll_finalize(self, h):
        return 0

    def gpbs_coll_buffer(self, h, which):
        return 0

    def gpbs_coll_destroy(self, h):
        self.destroyed.append(h.value)


class _Exchange:
    """all_gather_object stand-in: rounds of one object per rank."""

    def __init__(self, world):
        self.world, self.cv, self.rounds = world, threading.Condition(), {}
        self.calls = [0] * world

    def gather_for(self, rank):
        def gather(obj):
            with self.cv:
                k = self.calls[rank]
                self.calls[rank] += 1
                slot = self.rounds.setdefault(k, [None] * self.world)
                slot[rank] = ("set", obj)
                self.cv.notify_all()
                ok = self.cv.wait_for(lambda: all(x is not None for x in slot), timeout=10)
                assert ok, "a rank never joined this exchange"
                return [x[1] for x in slot]
        return gather


@pytest.mark.parametrize("fail", ["create", "open", "none"])
def test_setup_raises_on_every_rank_together(monkeypatch, fail):
    import pbs_amd.parallel.ipc_coll as M
    lib = _FakeLib(fail_create_rank=1 if fail == "create" else -1, fail_open_rank=0 if fail == "open" else -1)
    monkeypatch.setattr(M, "hiplib", lambda: lib)
    ex = _Exchange(2)
    out = [None, None]

    def rank(r):
        try:
            M.IpcColl(0, r, 2, 1 << 20, gather=ex.gather_for(r))
            out[r] = "ok"
        except RuntimeError as e:
            out[r] = str(e)
    ths = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(20)
    assert ex.calls == [2, 2]  # both exchanges on both ranks, whatever failed
    if fail == "none":
        assert out == ["ok", "ok"]
    else:
        assert all(o.startswith("IPC all-reduce setup failed") for o in out), out
