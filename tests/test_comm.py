"""Communicator layer: LocalCommunicator, in-process groups, RCCL (world of one)."""
import threading

import pytest
import torch


def test_local_comm(C):
    c = C.LocalCommunicator()
    assert c.size() == 1 and c.rank() == 0
    assert c.all_gather([1, 2, 3]) == [1, 2, 3]
    assert c.all_reduce_sum([5]) == [5]
    s = torch.arange(10, dtype=torch.int64)
    r = torch.zeros(10, dtype=torch.int64)
    c.all_to_all_v(s, [10], r, [10])
    assert torch.equal(s, r)


@pytest.mark.parametrize("n", [2, 5])
def test_in_process_collectives(C, n):
    g = C.InProcessGroup(n)
    out, errs = [None] * n, []

    def work(r):
        try:
            c = g.communicator(r)
            ag = c.all_gather([r, r * 10])
            red = c.all_reduce_sum([r, 1])
            # rank r sends (p + 1) words to every peer p, valued r * 100 + p
            sc = [p + 1 for p in range(n)]
            send = torch.cat([torch.full((p + 1,), r * 100 + p, dtype=torch.int64) for p in range(n)])
            rc = [r + 1] * n
            recv = torch.zeros(sum(rc), dtype=torch.int64)
            c.all_to_all_v(send, sc, recv, rc)
            out[r] = (ag, red, recv)
        except Exception as e:
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    for r in range(n):
        ag, red, recv = out[r]
        assert ag == [v for q in range(n) for v in (q, q * 10)]
        assert red == [sum(range(n)), n]
        exp = torch.cat([torch.full((r + 1,), q * 100 + r, dtype=torch.int64) for q in range(n)])
        assert torch.equal(recv, exp)


@pytest.mark.gpu
def test_rccl_world_of_one(C, cuda):
    """Real RCCL library: init from a unique id, collectives, a join through it."""
    uid = C.rccl_unique_id()
    assert len(uid) == 128
    c = C.RcclCommunicator(uid, 0, 1, 0)
    assert c.name() == "rccl"
    assert c.all_gather([7, 8]) == [7, 8]
    assert c.all_reduce_sum([3]) == [3]
    c.barrier()
    s = torch.arange(1000, dtype=torch.int64, device="cuda")
    r = torch.zeros_like(s)
    c.all_to_all_v(s, [1000], r, [1000])
    assert torch.equal(s, r)
    ctx = C.ExecContext("device", 0, c)
    G = 1 << 18
    R = C.Relation(G, G, "device", 0)
    S = C.Relation(G, G, "device", 0)
    R.generate(C.GenSpec(seed=1), 0)
    S.generate(C.GenSpec(seed=2), 0)
    assert C.HashJoin(R, S, ctx, C.JoinConfig()).run()["global_matches"] == G
