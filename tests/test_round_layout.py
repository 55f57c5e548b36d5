"""Round-interleaved network windows (kernels.h RoundMap): the slot map, and
joins whose sampled single-rank windows use it, against the linear layout and
the exact oracle."""
import pytest

from test_join_engine import run_join


def test_round_map_is_a_piecewise_bijection(C):
    """lp = lv = 0 is the identity; otherwise slice i's logical positions
    i << lv | k land in 2^lp-slot pieces, piece j of every slice in round j,
    all slots distinct and inside roundSlots(max slice, lp, lns)."""
    slot = C.ops.round_slot
    for L in (0, 1, 77, 1 << 20, (1 << 33) + 5):
        assert slot(L, 0, 0, 0) == L
    lp, lv, lns = 2, 4, 3  # 8 slices of up to 16 positions, pieces of 4
    caps = [16, 13, 16, 9, 4, 16, 1, 12]
    seen = set()
    for i, cap in enumerate(caps):
        phys = [slot((i << lv) | k, lp, lv, lns) for k in range(cap)]
        for k, p in enumerate(phys):
            assert p == ((k >> lp) << (lns + lp)) | (i << lp) | (k & 3)
            if k & 3:
                assert p == phys[k - 1] + 1  # contiguous inside a piece
        seen.update(phys)
    assert len(seen) == sum(caps)
    assert max(seen) < C.ops.round_slots(max(caps), lp, lns) == 4 << (lns + lp)
    assert C.ops.round_slots(17, lp, lns) == 5 << (lns + lp)


def _cfg(C, lp, bitmap):
    cfg = C.JoinConfig()
    cfg.round_lp = lp
    cfg.bitmap_join = bitmap
    cfg.network_histogram = C.HistogramMode.SAMPLED
    return cfg


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_round_windows_two_level(C, cuda, sparse):
    """The two-level plan's sampled network windows (u32 fragments of dense
    keys, key-only words of sparse 63-bit keys): round-interleaved slices
    (both windows report it) give the same exact count as linear slices."""
    G_R = 1 << 22
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    for lp, want in ((9, 2), (0, 0)):
        inner = C.GenSpec(seed=1234)
        outer = C.GenSpec(distribution=C.KeyDistribution.UNIQUE, seed=4321)
        inner.sparse64 = outer.sparse64 = sparse
        R = C.Relation(G_R, G_R, "device", 0)
        S = C.Relation(G_R, G_R, "device", 0)
        R.generate(inner, 0)
        S.generate(outer, 0)
        j = C.HashJoin(R, S, ctx, _cfg(C, lp, False))
        assert j.plan.key_only == sparse, j.plan
        for _ in range(2):
            res = j.run()
            assert res["global_matches"] == G_R and res["round_windows"] == want, res
            assert res["network_fallbacks"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("dist", ["UNIQUE", "ZIPF", "UNIFORM"])
@pytest.mark.parametrize("bitmap", [False, True])
def test_round_windows_exact(C, cuda, dist, bitmap):
    """Round-interleaved and linear windows give the oracle's count for even
    and skewed outer relations, on the two-level and the bitmap plans (a
    window too uneven for rounds keeps linear slices)."""
    G_R, G_S = 1 << 21, 5 << 20
    for lp in (9, 0):
        res, exp, j = run_join(C, "cuda", G_R, G_S, dist, cfg=_cfg(C, lp, bitmap))
        assert j.plan.bitmap_join == bitmap
        assert res["global_matches"] == exp, (lp, res)
        if not bitmap and lp == 0:
            assert res["round_windows"] == 0
        if not bitmap and lp and dist != "ZIPF":
            assert res["round_windows"] == 2, res


@pytest.mark.gpu
@pytest.mark.parametrize("raw,sparse", [(True, False), (False, False), (True, True)])
def test_round_send_buffers_shuffle(C, cuda, raw, sparse):
    """N > 1 sampled shuffle (2 in-process ranks): the claim slices of each
    rank's send buffer are round-interleaved (both relations report it) and
    the runs are gathered (raw words) or packed (codec) through the same slot
    map; counts equal the oracle and the linear send buffers'."""
    from test_distributed import run_ranks
    G = 8_000_000
    got = {}
    for lp in (9, 0):
        def cfg_fn(c, lp=lp):
            c.network_histogram = C.HistogramMode.SAMPLED
            c.bitmap_join = False
            c.chunks = 1
            c.round_lp = lp
            c.wire_codec = C.WireCodecMode.OFF if raw else C.WireCodecMode.ON
        inner, outer = C.GenSpec(seed=1234), C.GenSpec(seed=99)
        inner.sparse64 = outer.sparse64 = sparse
        results, exp = run_ranks(C, 2, "device", G, G, cfg_fn, inner=inner, outer=outer)
        for res, plan in results:
            assert plan.sampled_network and res["network_fallbacks"] == 0, res
            assert res["round_windows"] == (2 if lp else 0), res
            if exp is not None:
                assert res["global_matches"] == exp
        got[lp] = results[0][0]["global_matches"]
    assert got[9] == got[0]


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [8, 11])
@pytest.mark.parametrize("sparse", [False, True])
def test_round_windows_network_bits(C, cuda, bits, sparse):
    """Round-interleaved windows at other fan-outs (G * F = 2048 or 16384
    slices per round): same count as linear slices, both windows rounded on
    the two-level plan."""
    G_R = 1 << 22
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    inner, outer = C.GenSpec(seed=5), C.GenSpec(seed=6)
    inner.sparse64 = outer.sparse64 = sparse
    R = C.Relation(G_R, G_R, "device", 0)
    S = C.Relation(G_R, G_R, "device", 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    for lp in (9, 0):
        cfg = _cfg(C, lp, False)
        cfg.network_bits = bits
        j = C.HashJoin(R, S, ctx, cfg)
        assert j.plan.network_bits == bits, j.plan
        res = j.run()
        info = {k: res[k] for k in ("global_matches", "round_windows", "network_fallbacks", "sampled_network")}
        assert res["global_matches"] == G_R and res["round_windows"] == (2 if lp else 0), (info, repr(j.plan))
