"""N > 1 engine past 2^31 tuples per rank (BASELINE config 4's per-rank size:
1B x 16B over 8 GPUs puts ~2e9 outer tuples on every rank).

Two in-process ranks on the test GPU; every outer key is even and key
hashing is off, so with round-robin ownership of the 1024 network partitions
rank 0 owns every partition an outer key lands in and receives all 2.2e9
outer tuples: its window, wire segments, local items, split columns and
build/probe spans all run past 2^31 elements (the N = 1 analog is
test_bitmap_plans.py::test_key_only_outer_past_2g_elements).  Dense keys
(CompressedTuples) and sparse 63-bit keys (key-only words), sampled and
exact network passes; counts equal the closed form (every outer key matches
one inner key).
"""
import threading

import pytest
import torch

N_OUT = 2_200_000_000
G_R = 1 << 24


def run_two_ranks(C, R_parts, S_parts, cfg_fn):
    group = C.InProcessGroup(2)
    out, errs = [None] * 2, []

    def work(r):
        try:
            ctx = C.ExecContext("device", 0, group.communicator(r))
            R, S = R_parts[r], S_parts[r]
            cfg = C.JoinConfig()
            cfg_fn(cfg)
            j = C.HashJoin(C.Relation.from_tensor(R, G_R), C.Relation.from_tensor(S, N_OUT), ctx, cfg)
            out[r] = (j.run(), j.plan)
            del j, ctx
        except Exception as e:  # surface in the main thread
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(timeout=600) for t in ts]
    assert not errs, errs
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_rank_receives_past_2g_outer_tuples(C, cuda, sparse):
    g = torch.Generator(device="cuda").manual_seed(7)
    if sparse:
        inner = torch.randint(0, 1 << 61, (G_R,), device="cuda", generator=g).unique() * 2  # even 63-bit keys
    else:
        inner = torch.arange(G_R, device="cuda") * 2
    n_in = inner.numel()
    half_in, half_out = n_in // 2, N_OUT // 2
    R_parts = [torch.stack([inner[:half_in], torch.arange(half_in, device="cuda")], 1).contiguous(),
               torch.stack([inner[half_in:], torch.arange(half_in, n_in, device="cuda")], 1).contiguous()]
    S_parts = []
    for r in range(2):
        rid = torch.arange(r * half_out, (r + 1) * half_out, device="cuda")
        key = inner[torch.randint(0, n_in, (half_out,), device="cuda", generator=g)]
        S_parts.append(torch.stack([key, rid], 1))
        del rid, key
    torch.cuda.empty_cache()
    for mode in ("SAMPLED", "EXACT"):
        def cfg_fn(c):
            c.key_hashing = C.KeyHashing.OFF
            c.assignment = C.AssignmentPolicy.ROUND_ROBIN
            c.bitmap_join = False
            c.replicate_bitmap = C.PlanChoice.OFF
            c.network_histogram = getattr(C.HistogramMode, mode)
            c.chunks = 2
        out = run_two_ranks(C, R_parts, S_parts, cfg_fn)
        (r0, plan), (r1, _) = out
        assert plan.key_only == sparse, plan
        assert r0["outer_received"] == N_OUT and r0["outer_received"] > (1 << 31), r0["outer_received"]
        assert r1["outer_received"] == 0
        for res in (r0, r1):
            assert res["global_matches"] == N_OUT, (mode, sparse, res["global_matches"])
        if mode == "SAMPLED":
            assert r0["sampled_network"], r0
        torch.cuda.empty_cache()
    del R_parts, S_parts
    torch.cuda.empty_cache()
