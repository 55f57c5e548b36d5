"""Count-only single-level bitmap plans (tasks/BitmapJoin) and the N > 1 plan
choice (replicated bitmaps vs tuple shuffle), plus the sparse 63-bit key
generator and the automatic wide format for keys that do not fit a
CompressedTuple.

In-process ranks share one process (threads); on the host they run the same
plan with exact partitioning and the host communicator's all-reduce, on the
device the RCCL-free in-process communicator stages the all-reduce through
the host.  Counts are checked against the exact oracle or a torch reference.
"""
import threading

import pytest
import torch

from conftest import devices


def run_ranks(C, n, loc, R_parts, S_parts, G_R, G_S, cfg_fn=None, runs=2):
    """R_parts / S_parts: per-rank [n_r, 2] int64 tensors (or generator specs)."""
    group = C.InProcessGroup(n)
    out, errs = [None] * n, []

    def work(r):
        try:
            comm = group.communicator(r)
            ctx = C.ExecContext(loc, 0 if loc == "device" else -1, comm)
            R, S = R_parts(r), S_parts(r)
            cfg = C.JoinConfig()
            if cfg_fn:
                cfg_fn(cfg)
            j = C.HashJoin(R, S, ctx, cfg)
            res = [j.run() for _ in range(runs)]
            out[r] = (res, j.plan)
        except Exception as e:  # surface in the main thread
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    [t.start() for t in ts]
    [t.join(timeout=600) for t in ts]
    assert not errs, errs
    return out


def generated(C, loc, spec, G, n):
    def make(r):
        rel = C.Relation(C.Relation.local_size_for(G, r, n), G, loc, 0)
        rel.generate(spec, C.Relation.local_offset_for(G, r, n))
        return rel
    return make


def force_replicated(c, C):
    c.replicate_bitmap = C.PlanChoice.ON


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("outer_dist", ["UNIQUE", "UNIFORM", "ZIPF"])
def test_replicated_bitmap_ranks(C, dev, n_ranks, outer_dist):
    loc = "device" if dev == "cuda" else "host"
    G_R, G_S = 300_007, 450_011
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(distribution=getattr(C.KeyDistribution, outer_dist), seed=99,
                      domain=0 if outer_dist == "UNIQUE" else G_R, zipf_theta=0.9)
    if outer_dist == "UNIQUE":
        G_S = G_R
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
    out = run_ranks(C, n_ranks, loc, generated(C, loc, inner, G_R, n_ranks), generated(C, loc, outer, G_S, n_ranks),
                    G_R, G_S, lambda c: force_replicated(c, C))
    for res_list, plan in out:
        assert plan.bitmap_join and plan.bitmap_replicated == (n_ranks > 1)
        for res in res_list:
            assert res["bitmap_join"] and res["global_matches"] == exp
            assert res["local_fallbacks"] == 0 and res["network_fallbacks"] == 0
            # the replicated plan keeps every tuple on its rank
            assert res["inner_received"] == res["inner_local"] and res["outer_received"] == res["outer_local"]
    assert sum(o[0][0]["local_matches"] for o in out) == exp


@pytest.mark.gpu
@pytest.mark.parametrize("nth,flat", [("256", "0"), ("256", "1"), ("1024", "0"), ("1024", "1")])
def test_bitmap_walk_variants(C, nth, flat):
    """Both slice walks of the bitmap kernels (one pipelined walk per claim
    slice / one flat walk over all slices of a partition) at both workgroup
    sizes give the exact count: short partitions (many empty and sub-vector
    slices, tails of 1-3 fragments) and long ones, N = 1 fused kernel and the
    replicated build / probe kernels at N = 2."""
    def cfg(c):
        force_replicated(c, C)
        c.bm_threads = int(nth)
        c.bm_flat = int(flat)
    for G_R, G_S, n_ranks in [(40_009, 70_001, 1), (1 << 20, 3 << 19, 1), (3_000_017, 1_000_003, 1),
                              (300_007, 450_011, 2)]:
        inner = C.GenSpec(seed=77)
        outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=5, domain=G_R)
        exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
        out = run_ranks(C, n_ranks, "device", generated(C, "device", inner, G_R, n_ranks),
                        generated(C, "device", outer, G_S, n_ranks), G_R, G_S, cfg)
        for res_list, plan in out:
            assert plan.bitmap_join
            for res in res_list:
                assert res["bitmap_join"] and res["global_matches"] == exp, (G_R, G_S, n_ranks, res)


@pytest.mark.gpu
@pytest.mark.parametrize("nb,dup", [(1, False), (3, False), (2, True)])
def test_bitmap_split_pieces(C, nb, dup):
    """21 fragment bits above the network digit (forced small digit): each
    partition is joined by two workgroups holding one 128 KiB piece of its
    fragment range each; counts are exact, and a repeated inner key still
    sends the join to the two-level plan."""
    G = 1 << (21 + nb)
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    inner = C.GenSpec(seed=3)
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=4, domain=G)
    R = C.Relation(G, G, "device", 0)
    S = C.Relation(G // 2, G // 2, "device", 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    exp = C.Relation.expected_matches(inner, G, outer, G // 2)
    if dup:
        import torch
        t = R.to_tensor()
        t[5, 0] = t[9, 0]  # one repeated inner key
        R = C.Relation.from_tensor(t.contiguous(), G)
        exp = None
    cfg = C.JoinConfig()
    cfg.network_bits = nb
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.plan.bitmap_join and j.plan.bitmap_bits == 21
    res = j.run()
    if dup:
        from helpers import ref_join_count
        exp = ref_join_count(R.to_tensor()[:, 0].cpu(), S.to_tensor()[:, 0].cpu())
        assert not res["bitmap_join"] and res["global_matches"] == exp
    else:
        assert res["bitmap_join"] and res["global_matches"] == exp
        assert j.run()["global_matches"] == exp


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [2, 4])
def test_replicated_bitmap_split_pieces(C, dev, n_ranks):
    """21 fragment bits on the replicated plan: each partition's bitmap is
    built and probed as two 128 KiB pieces (adjacent in the all-reduced
    array), in 1 and 3 all-reduce ranges; exact on every rank."""
    loc = "device" if dev == "cuda" else "host"
    nb = 2
    G_R, G_S = 1 << (21 + nb), 3 << (19 + nb)
    inner = C.GenSpec(seed=41)
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=42, domain=G_R)
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)

    for chunks in (1, 3):
        def cfg(c):
            force_replicated(c, C)
            c.network_bits = nb
            c.reduce_chunks = chunks
        out = run_ranks(C, n_ranks, loc, generated(C, loc, inner, G_R, n_ranks),
                        generated(C, loc, outer, G_S, n_ranks), G_R, G_S, cfg)
        for res_list, plan in out:
            assert plan.bitmap_join and plan.bitmap_replicated and plan.bitmap_bits == 21
            for res in res_list:
                assert res["bitmap_join"] and res["global_matches"] == exp, (chunks, res["global_matches"], exp)


@pytest.mark.gpu
@pytest.mark.parametrize("n_ranks", [1, 4])
@pytest.mark.parametrize("G_R,G_S", [(1000, 0), (37, 5000), (3, 3), (100_000, 1)])
def test_bitmap_tiny_and_empty_sides(C, n_ranks, G_R, G_S):
    """Tiny and empty relations (some ranks hold no tuples at all): the
    sampled layout falls back to exact counts, one-launch histograms and
    layouts of both sides, exact results."""
    inner = C.GenSpec(seed=8)
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=9, domain=G_R)
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S) if G_S else 0
    out = run_ranks(C, n_ranks, "device", generated(C, "device", inner, G_R, n_ranks),
                    generated(C, "device", outer, G_S, n_ranks), G_R, G_S, lambda c: force_replicated(c, C))
    for res_list, _ in out:
        for res in res_list:
            assert res["global_matches"] == exp, (G_R, G_S, n_ranks, res["global_matches"], exp)


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", ["1", "3", "7"])
def test_replicated_bitmap_reduce_ranges(C, chunks):
    """The replicated plan's all-reduce in k partition ranges (k not dividing
    the partition count), each range probed behind its own all-reduce: exact
    counts on every rank."""
    G_R, G_S, n = 1_000_003, 2_000_029, 4

    def cfg(c):
        force_replicated(c, C)
        c.reduce_chunks = int(chunks)
    inner = C.GenSpec(seed=11)
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=12, domain=G_R, zipf_theta=0.75)
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
    out = run_ranks(C, n, "device", generated(C, "device", inner, G_R, n), generated(C, "device", outer, G_S, n),
                    G_R, G_S, cfg)
    for res_list, plan in out:
        assert plan.bitmap_join and plan.bitmap_replicated
        for res in res_list:
            assert res["global_matches"] == exp and res["network_fallbacks"] == 0
    assert sum(o[0][0]["local_matches"] for o in out) == exp


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [2, 4])
def test_replicated_bitmap_cross_rank_duplicate_falls_back(C, dev, n_ranks):
    """A key held by two ranks sets the same bit twice: the all-reduced sum
    carries, the set-bit count falls below |R|, every rank agrees and the join
    finishes on the shuffle + two-level plan (exact count); later joins stay
    there."""
    loc = "device" if dev == "cuda" else "host"
    per = 20_000
    G = per * n_ranks
    keys = torch.arange(G, dtype=torch.int64)
    keys[per] = 7  # rank 1's first key duplicates rank 0's key 7
    outer_keys = torch.randint(0, G, (G,), generator=torch.Generator().manual_seed(3))
    exp = int((torch.bincount(keys, minlength=G)[outer_keys]).sum())
    tdev = "cuda" if dev == "cuda" else "cpu"

    def rel(src, r):
        k = src[r * per:(r + 1) * per]
        t = torch.stack([k, torch.arange(r * per, (r + 1) * per)], 1).contiguous().to(tdev)
        return C.Relation.from_tensor(t, G)

    out = run_ranks(C, n_ranks, loc, lambda r: rel(keys, r), lambda r: rel(outer_keys, r), G, G,
                    lambda c: force_replicated(c, C), runs=2)
    for (first, second), plan in out:
        assert first["local_fallbacks"] == 1 and not first["bitmap_join"]
        assert first["global_matches"] == exp
        assert second["local_fallbacks"] == 0 and not second["bitmap_join"] and second["global_matches"] == exp
        assert not plan.bitmap_join  # restored two-level plan


@pytest.mark.parametrize("dev", devices())
def test_bitmap_in_rank_duplicate_falls_back(C, dev):
    """A repeated inner key on one rank (N == 1 and N == 3, forced bitmap)."""
    loc = "device" if dev == "cuda" else "host"
    tdev = "cuda" if dev == "cuda" else "cpu"
    for n_ranks in (1, 3):
        per = 30_000
        G = per * n_ranks
        keys = torch.arange(G, dtype=torch.int64)
        keys[5] = keys[6]
        okeys = torch.arange(G, dtype=torch.int64).flip(0)
        exp = int(torch.bincount(keys, minlength=G)[okeys].sum())

        def rel(src, r):
            t = torch.stack([src[r * per:(r + 1) * per], torch.arange(r * per, (r + 1) * per)], 1).contiguous()
            return C.Relation.from_tensor(t.to(tdev), G)

        out = run_ranks(C, n_ranks, loc, lambda r: rel(keys, r), lambda r: rel(okeys, r), G, G,
                        lambda c: force_replicated(c, C))
        for (first, second), _ in out:
            assert first["local_fallbacks"] == 1 and first["global_matches"] == exp
            assert second["global_matches"] == exp


def test_plan_choice_cost_model(C):
    """N > 1: the planner prices both plans in link bytes per rank.  Dense 1B
    keys: the replicated bitmaps (2 (N-1)/N x 128 MiB) undercut the shuffle
    ((N-1)/N of 2B tuples / N) at every N <= 8; sparse keys cannot use
    bitmaps at all."""
    cfg = C.JoinConfig()
    for n in (2, 4, 8):
        p = C.make_plan(cfg, n, 1_000_000_000, 1_000_000_000, 999_999_999, 999_999_999)
        assert not p.bitmap_join  # make_plan alone is the two-level plan; HashJoin adds the bitmap choice
    # through the engine (host ranks, Auto): fields are filled, the choice stays off the host path
    G = 200_003
    inner = C.GenSpec(seed=1)
    out = run_ranks(C, 4, "host", generated(C, "host", inner, G, 4), generated(C, "host", C.GenSpec(seed=2), G, 4),
                    G, G, None, runs=1)
    for (res,), plan in out:
        assert not plan.bitmap_join  # Auto never picks it on the host path
        assert 0 < plan.replicated_link_bytes < plan.shuffle_link_bytes
        assert plan.link_gbps > 0
        assert res["global_matches"] == G


def test_sparse64_generator(C):
    """Sparse random 63-bit keys: unique, spread over [0, 2^63), foreign keys
    drawn from the same key set, oracle preserved."""
    n = 200_000
    spec = C.GenSpec(seed=5)
    spec.sparse64 = True
    t = C.ops.generate(n, 0, n, spec, "cpu")
    k = t[:, 0]
    assert int(k.min()) >= 0 and torch.unique(k).numel() == n
    assert int(k.max()) > (1 << 60)  # really sparse
    fk = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=9, domain=n)
    fk.sparse64 = True
    o = C.ops.generate(3 * n, 0, 3 * n, fk, "cpu")
    assert bool(torch.isin(o[:, 0], k).all())
    assert C.Relation.expected_matches(spec, n, fk, 3 * n) == 3 * n
    plain = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=9, domain=n)
    assert C.Relation.expected_matches(spec, n, plain, 3 * n) is None  # transforms must match


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["8s", "9s", "8w", "8", "7", "7s"])
def test_key_only_count_variants(C, variant):
    """Every key-only count kernel variant against a torch reference, with heavily repeated inner keys (Zipf over sparse
    63-bit keys: long overflow chains through the next buckets)."""
    from helpers import ref_join_count
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    for (G_R, G_S, theta) in [(200_003, 300_007, 0.99), (1 << 20, 1 << 21, 0.5)]:
        inner = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=31, domain=G_R // 4, zipf_theta=theta)
        inner.sparse64 = True
        outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=32, domain=G_R // 4, zipf_theta=0.8)
        outer.sparse64 = True
        R = C.Relation(G_R, G_R, "device", 0)
        S = C.Relation(G_S, G_S, "device", 0)
        R.generate(inner, 0)
        S.generate(outer, 0)
        cfg = C.JoinConfig()
        cfg.key_count = int(variant.rstrip("sw"))
        # 7: v2 span kernel; 8: quotient table (44-bit fragments: 63-bit keys
        # above 10 + 9 radix bits; unsplit words: v2); 9: counted tables
        # throughout; "s": over the split (u32 + u16) local output; "8w": 48-bit
        # fragments (8 + 7 radix bits) on counted tables
        split = variant.endswith("s") or variant == "8w"
        cfg.split_local = split
        if variant in ("8s", "9s"):
            cfg.network_bits, cfg.local_bits = 10, 9
        elif split:  # 63-bit keys: the fragment above 8 + 7 radix bits fits the 48-bit split
            cfg.network_bits, cfg.local_bits = 8, 7
        j = C.HashJoin(R, S, ctx, cfg)
        assert j.plan.key_only and j.plan.split_local == split
        exp = ref_join_count(R.to_tensor()[:, 0].cpu(), S.to_tensor()[:, 0].cpu())
        for _ in range(2):
            assert j.run()["global_matches"] == exp, (variant, G_R, theta)


@pytest.mark.gpu
@pytest.mark.parametrize("key_count", [8, 9])
def test_key_only_multi_segment_compaction(C, key_count):
    """Hot keys with hundreds of thousands of inner copies: their partitions
    hold more than BP_DEDUP_SEG_MIN (32K) inner words, so bpKeyDedup compacts
    them in several segments and bpKeyDedupMerge moves the segment lists
    together before the counted spans; exact against a torch reference."""
    from helpers import ref_join_count
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    G_R, G_S = 3_000_017, 2_000_003
    inner = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=41, domain=20_000, zipf_theta=0.99)
    inner.sparse64 = True
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=42, domain=20_000, zipf_theta=0.9)
    outer.sparse64 = True
    R = C.Relation(G_R, G_R, "device", 0)
    S = C.Relation(G_S, G_S, "device", 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    cfg = C.JoinConfig()
    cfg.key_count = key_count
    cfg.split_local = True
    cfg.network_bits, cfg.local_bits = 10, 9  # 63-bit keys: 44-bit fragments (split words, quotient-eligible)
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.plan.key_only and j.plan.split_local, j.plan
    exp = ref_join_count(R.to_tensor()[:, 0].cpu(), S.to_tensor()[:, 0].cpu())
    for _ in range(3):
        assert j.run()["global_matches"] == exp, key_count


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [(1 << 20, 3 << 20), (5_000, 3 << 20), (3 << 20, 5_000), (0, 1 << 20)])
def test_sampled_general_path_device_layout(C, sizes):
    """Single-rank sampled network pass of the general path (key-only words):
    slices laid out on the device from the sampled totals; a side too small
    to sample gets an exact histogram next to a sampled one; counts equal a
    torch oracle, no fallback."""
    from helpers import ref_join_count
    G_R, G_S = sizes
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    inner = C.GenSpec(seed=51)
    inner.sparse64 = True
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=52, domain=max(G_R, 1))
    outer.sparse64 = True
    R = C.Relation(G_R, G_R, "device", 0)
    S = C.Relation(G_S, G_S, "device", 0)
    if G_R:
        R.generate(inner, 0)
    S.generate(outer, 0)
    exp = ref_join_count(R.to_tensor()[:, 0].cpu(), S.to_tensor()[:, 0].cpu()) if G_R else 0
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    cfg.network_bits, cfg.local_bits = 10, 9
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.plan.key_only and j.plan.sampled_network, j.plan
    for _ in range(2):
        res = j.run()
        assert res["global_matches"] == exp, (sizes, res["global_matches"], exp)
        assert res["sampled_network"] and res["network_fallbacks"] == 0, res


@pytest.mark.gpu
def test_key_only_outer_past_2g_elements(C):
    """General path with the outer side's local output past 2^31 elements
    (1.6e9 outer tuples in a gapped sampled layout of ~2.6e9 slots): span
    offsets above 2^31 must reach the build/probe intact.  Regression: the
    wave-uniform span offset was rebuilt from two readfirstlane halves whose
    low half sign-extended, so every probe batch after the first read from
    16 GiB below the partition (1.5076e9 of 1.6e9 matches, no fault)."""
    G_R, G_S = 100_000_000, 1_600_000_000
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    inner = C.GenSpec(seed=61)
    inner.sparse64 = True
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=62, domain=G_R)
    outer.sparse64 = True
    R = C.Relation(G_R, G_R, "device", 0)
    S = C.Relation(G_S, G_S, "device", 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    cfg = C.JoinConfig()
    cfg.network_bits, cfg.local_bits = 10, 9  # ~3052 outer tuples per final partition: two probe batches
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.plan.key_only, j.plan
    res = j.run()
    assert res["global_matches"] == G_S, (res["global_matches"], G_S)
    del j, R, S
    ctx.reset_scratch()


KQ_M = 0xFFFFFFFF


def kq_salt(b):
    return ((b + 1) * 0x85EBCA77) & KQ_M


def kq_home(v, lo_bits=0):
    return ((((v * 0x9E3779B1) & KQ_M) >> 20) ^ lo_bits) & 0xFFF


def kq_fragment(b, e, s, tag=0):
    """The fragment (f = 32 + s bits) whose counted-table key is (bucket b,
    stored value e ^ salt(b), tag): key_tables.hip kqKey inverted."""
    lo = kq_home(e, b) | (tag << 12)
    return (e << s) | lo


def kq4_fragment(b, v, s=12):
    """The fragment whose quotient-table key is (home bucket b, stored value
    v): key_tables.hip kq4Key inverted (s = 12: 44-bit fragments)."""
    return (v << s) | kq_home(v, b)


def quotient_escape_fragments(n, first_bucket=0):
    """Fragments whose counted-table value e ^ salt(b) is that table's empty
    marker, one per bucket b (44-bit fragments: 63-bit keys above 10 + 9
    radix bits): e = ~salt(b)."""
    return [kq_fragment(b, ~kq_salt(b) & KQ_M, 12) for b in range(first_bucket, first_bucket + n)]


def quotient_crowd_fragments(n, bucket=17):
    """n distinct fragments with the same quotient-table home bucket: four
    fill its slots, the rest go to the overflow table (cap 384 per span)."""
    return [kq4_fragment(bucket, 0x9E370001 + 7919 * i) for i in range(n)]


def kc_bucket(frag, s=12):
    """The counted table's home bucket of a fragment (key_tables.hip kcBucket,
    3072 two-entry buckets)."""
    import numpy as np
    frag = np.asarray(frag, dtype=np.uint64)
    e = (frag >> np.uint64(s)) & np.uint64(KQ_M)
    lo = frag & np.uint64((1 << s) - 1)
    h = ((e * np.uint64(0x9E3779B1)) & np.uint64(KQ_M)) ^ ((lo * np.uint64(0x85EBCA77)) & np.uint64(KQ_M))
    h ^= h >> np.uint64(15)
    return (h * np.uint64(3072)) >> np.uint64(32)


def counted_crowd_fragments(n, bucket=3071):
    """n distinct 44-bit fragments with the same counted-table home bucket:
    two fill it, the rest walk on past the table's end (bucket 3071 is the
    last: the walk wraps to entry 0)."""
    import numpy as np
    rng = np.random.default_rng(n)
    out = []
    while len(out) < n:
        cand = rng.integers(0, 1 << 44, size=1 << 22, dtype=np.uint64)
        out = list(dict.fromkeys(out + [int(f) for f in cand[kc_bucket(cand) == bucket]]))
    return out[:n]  # (draw order: the largest keys set the plan's 63 key bits)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,dup,key_count,reruns",
                         [("crowd", 20, 1, 8, 0), ("crowd", 40, 3, 8, 0), ("crowd", 100, 1, 8, 0),
                          ("crowd", 400, 1, 8, 1), ("escape", 40, 1, 8, 0), ("escape", 20, 1, 9, 0),
                          ("escape", 300, 3, 9, 0), ("ccrowd", 300, 3, 9, 0), ("ccrowd", 2000, 1, 9, 0)])
def test_key_quotient_escapes(C, kind, n, dup, key_count, reruns):
    """Quotient / counted build/probe on adversarial keys, all in one final
    partition.  crowd: n keys share one quotient-table home bucket -- 4 in its
    slots, the rest in the overflow table of full fragments (up to 384 per
    span); 400 fill it: the count is void and the build/probe re-runs on
    counted tables (1 re-run).  escape: keys whose counted-table value is that
    table's empty marker -- counted tables hold them inline, the quotient
    table (no marker) as any other key.  ccrowd: n keys share the counted
    table's last home bucket -- two in it, the rest walk, wrapping to entry 0.  Repeated inner keys (dup 3) are seen
    at plan time or by the overflow chains.  Counts equal a torch oracle every
    time; later joins of the same HashJoin start where the first ended (no
    re-run)."""
    import torch
    from helpers import ref_join_count
    g = torch.Generator().manual_seed(n * 7 + dup + key_count)
    part = 0x2A5F3  # one (network, local) digit pair: the keys share a span
    frags = {"crowd": lambda: quotient_crowd_fragments(n), "ccrowd": lambda: counted_crowd_fragments(n),
             "escape": lambda: quotient_escape_fragments(n, first_bucket=17)}[kind]()
    esc = torch.tensor(frags, dtype=torch.int64)
    esc_keys = (esc << 19) | part
    other = torch.randint(1 << 40, (1 << 62) - 1, (400_000,), generator=g, dtype=torch.int64).unique()
    rk = torch.cat([esc_keys.repeat(dup), other])
    rk = rk[torch.randperm(rk.numel(), generator=g)]
    sk = torch.cat([esc_keys.repeat(5), other[torch.randint(0, other.numel(), (600_000,), generator=g)],
                    (esc + 1) << 19 | part])  # + near misses in the same span
    sk = sk[torch.randperm(sk.numel(), generator=g)]
    exp = ref_join_count(rk, sk)
    rows = lambda k: torch.stack([k, torch.arange(k.numel())], 1).contiguous().cuda()
    R, S = rows(rk), rows(sk)
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    cfg.network_bits, cfg.local_bits = 10, 9
    cfg.key_hashing = C.KeyHashing.OFF
    cfg.key_count = key_count
    j = C.HashJoin(C.Relation.from_tensor(R, R.shape[0]), C.Relation.from_tensor(S, S.shape[0]), ctx, cfg)
    assert j.plan.key_only and j.plan.split_local and j.plan.key_bits == 63, j.plan
    for i in range(2):
        res = j.run()
        assert res["global_matches"] == exp, (kind, n, dup, res["global_matches"], exp)
        assert res["reruns"] == (reruns if i == 0 else 0), (i, res["reruns"])


@pytest.mark.gpu
@pytest.mark.parametrize("key_count,frag_bits", [(8, 44), (9, 44), (8, 48)])
def test_key_tables_no_foreign_matches(C, key_count, frag_bits):
    """Quotient and counted tables store a key as (bucket, 32-bit value[, tag])
    that names it only in its home bucket.  Inner keys share home bucket h
    (quotient table: six, so two sit in the overflow table; counted tables:
    three, the third displaced); every outer probe key B(X, d) has home h + d
    and the SAME stored value and tag as inner key X: a table that compared an
    entry without its home would count B as X.  Exact counts against a torch
    oracle on the quotient table (44-bit fragments), counted tables
    (key_count 9) and the 48-bit counted path (8 + 7 radix bits)."""
    import torch
    from helpers import ref_join_count
    s = frag_bits - 32
    bits = 63 - frag_bits
    net = 10 if bits == 19 else 8
    part = 0x2A5F3 & ((1 << bits) - 1)
    g = torch.Generator().manual_seed(frag_bits * 10 + key_count)
    h = 1000
    quotient = key_count == 8 and frag_bits == 44
    n_in = 6 if quotient else 3
    tags = [0] * n_in if s <= 12 else [3, 3, 11]
    es = [0x80000000 | int(x) for x in torch.randint(0, 1 << 31, (n_in,), generator=g)]
    probes = []
    if quotient:
        inner = [kq4_fragment(h, e) for e in es]
        for e in es:
            for d in (1, 2, 3, 4):
                probes.append(kq4_fragment(h + d, e))
    else:
        inner = [kq_fragment(h, e, s, t) for e, t in zip(es, tags)]
        vs = [e ^ kq_salt(h) for e in es]
        for v, t in zip(vs, tags):
            for d in (1, 2, 3, 4):
                probes.append(kq_fragment(h + d, v ^ kq_salt(h + d), s, t))
    assert not set(probes) & set(inner)
    key = lambda f: (torch.tensor(f, dtype=torch.int64) << bits) | part
    other = torch.randint(1 << 40, (1 << 62) - 1, (200_000,), generator=g, dtype=torch.int64).unique()
    rk = torch.cat([key(inner), other])
    sk = torch.cat([key(probes).repeat(7), key(inner).repeat(3), other[:50_000]])
    exp = ref_join_count(rk, sk)
    assert exp == 3 * n_in + 50_000
    rows = lambda k: torch.stack([k, torch.arange(k.numel())], 1).contiguous().cuda()
    R, S = rows(rk), rows(sk)
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    cfg.network_bits, cfg.local_bits = net, bits - net
    cfg.key_hashing = C.KeyHashing.OFF
    cfg.key_count = key_count
    j = C.HashJoin(C.Relation.from_tensor(R, R.shape[0]), C.Relation.from_tensor(S, S.shape[0]), ctx, cfg)
    assert j.plan.key_only and j.plan.split_local and j.plan.key_bits == 63, j.plan
    for _ in range(2):
        res = j.run()
        assert res["global_matches"] == exp, (key_count, frag_bits, res["global_matches"], exp)
        assert res["reruns"] == 0, res


@pytest.mark.parametrize("dev", devices())
def test_sparse64_join_auto_wide(C, dev):
    """63-bit keys do not fit a CompressedTuple: the planner switches by itself
    (no assertion) to 8-byte key-only words for a count and to the wide
    format when materializing; both joins are exact."""
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    G_R, G_S = 150_000, 400_000
    inner = C.GenSpec(seed=21)
    inner.sparse64 = True
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=22, domain=G_R, zipf_theta=0.8)
    outer.sparse64 = True
    R = C.Relation(G_R, G_R, loc, 0)
    S = C.Relation(G_S, G_S, loc, 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    j = C.HashJoin(R, S, ctx, C.JoinConfig())
    assert j.plan.key_only and not j.plan.wide and not j.plan.bitmap_join and j.plan.key_bits == 63
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
    assert exp == G_S
    for _ in range(2):
        assert j.run()["global_matches"] == exp
    cfg = C.JoinConfig()
    cfg.materialize = True
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.plan.wide and not j.plan.key_only
    res = j.run()
    assert res["global_matches"] == exp == res["output_pairs"]
    pairs = j.output()
    Rt, St = R.to_tensor().cpu(), S.to_tensor().cpu()
    assert torch.equal(Rt[pairs[:, 0], 0], St[pairs[:, 1], 0])


@pytest.mark.gpu
@pytest.mark.parametrize("dup,bits", [(1, None), (37, None), (3000, None), (37, (10, 9)), (3000, (10, 9)),
                                      (200_000, (10, 9))])
def test_key_only_count_duplicates(C, cuda, dup, bits):
    """KCOUNT build/probe (key-only words, bucketized LDS table) with every
    inner key repeated `dup` times: long bucket pass-through chains (3000
    copies overflow hundreds of 4-slot buckets) and partial batches; the
    count equals a torch oracle."""
    import torch
    g = torch.Generator().manual_seed(dup)
    nb = 3_000_000 // dup + 1
    base = torch.randint(1 << 40, (1 << 62) - 1, (nb,), generator=g, dtype=torch.int64).unique()
    rk = base.repeat_interleave(dup)[:3_000_000]
    pick = torch.randint(0, base.numel(), (5_000_000,), generator=g)
    miss = torch.randint(1 << 40, (1 << 62) - 1, (1_000_000,), generator=g, dtype=torch.int64)
    sk = torch.cat([base[pick], miss])
    sk = sk[torch.randperm(sk.numel(), generator=g)]
    mult = torch.zeros(base.numel(), dtype=torch.int64)
    mult.index_add_(0, torch.searchsorted(base, rk), torch.ones_like(rk))
    pos = torch.searchsorted(base, sk).clamp(max=base.numel() - 1)
    exp = int(torch.where(base[pos] == sk, mult[pos], torch.zeros_like(pos)).sum())
    rows = lambda k: torch.stack([k, torch.arange(k.numel())], 1).contiguous().cuda()
    R, S = rows(rk), rows(sk)
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    if bits:  # 44-bit fragments: the quotient table, partitions of repeated keys on counted tables
        cfg.network_bits, cfg.local_bits = bits
    j = C.HashJoin(C.Relation.from_tensor(R, R.shape[0]), C.Relation.from_tensor(S, S.shape[0]), ctx, cfg)
    assert j.plan.key_only and not j.plan.bitmap_join, j.plan
    for _ in range(2):
        res = j.run()
        assert res["global_matches"] == exp, (dup, bits, res["global_matches"], exp)
        assert res["reruns"] == 0, res["reruns"]


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [2, 4])
def test_sparse64_key_only_ranks(C, dev, n_ranks):
    """Key-only words through the N-rank shuffle (exchange, local pass, KCOUNT
    build/probe), chunked exchange included; the wire codec carries only the
    key bits above the network digit (no rid, no rid base)."""
    loc = "device" if dev == "cuda" else "host"
    G_R, G_S = 120_011, 300_007
    inner = C.GenSpec(seed=31)
    inner.sparse64 = True
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=32, domain=G_R)
    outer.sparse64 = True

    def cfg_fn(c):
        c.chunks = 2
        c.wire_codec = C.WireCodecMode.ON
    out = run_ranks(C, n_ranks, loc, generated(C, loc, inner, G_R, n_ranks), generated(C, loc, outer, G_S, n_ranks),
                    G_R, G_S, cfg_fn)
    for res_list, plan in out:
        assert plan.key_only and not plan.bitmap_join
        assert list(plan.wire_bits) == [plan.key_bits - plan.network_bits] * 2, (plan.wire_bits, plan)
        for res in res_list:
            assert res["global_matches"] == G_S


def test_generated_relations_skip_planning_scans(C):
    """Generated relations carry their key bound and positional rids: the
    plan is identical to the one from a tensor (which is scanned)."""
    G = 100_000
    spec = C.GenSpec(seed=3)
    R = C.Relation(G, G, "host", 0)
    R.generate(spec, 0)
    S = C.Relation(G, G, "host", 0)
    S.generate(C.GenSpec(seed=4), 0)
    ctx = C.ExecContext("host", -1, C.LocalCommunicator())
    p1 = C.HashJoin(R, S, ctx, C.JoinConfig()).plan
    R2 = C.Relation.from_tensor(R.to_tensor(), G)
    S2 = C.Relation.from_tensor(S.to_tensor(), G)
    p2 = C.HashJoin(R2, S2, ctx, C.JoinConfig()).plan
    assert repr(p1) == repr(p2)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("mode", ["shuffle", "replicated", "shuffle-chunks3"])
def test_measurement_keys_two_ranks(C, dev, mode):
    """Every .perf key of the reference (performance/Measurements.cpp:136-542)
    is present and non-negative after a 2-rank join, on both N > 1 plans; the
    phases that ran are timed (> 0)."""
    loc = "device" if dev == "cuda" else "host"
    G = 400_009
    group = C.InProcessGroup(2)
    snaps, errs = [None, None], []

    def work(r):
        try:
            ctx = C.ExecContext(loc, 0 if loc == "device" else -1, group.communicator(r))
            R = C.Relation(C.Relation.local_size_for(G, r, 2), G, loc, 0)
            S = C.Relation(C.Relation.local_size_for(G, r, 2), G, loc, 0)
            R.generate(C.GenSpec(seed=1), C.Relation.local_offset_for(G, r, 2))
            S.generate(C.GenSpec(seed=2), C.Relation.local_offset_for(G, r, 2))
            cfg = C.JoinConfig()
            if mode == "replicated":
                cfg.replicate_bitmap = C.PlanChoice.ON
            else:
                cfg.bitmap_join = False
                cfg.chunks = 3 if mode.endswith("3") else 1
            res = C.HashJoin(R, S, ctx, cfg).run()
            assert res["global_matches"] == G
            snaps[r] = C.measurements.snapshot()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    assert not errs, errs
    keys = C.measurements.reference_keys()
    assert len(keys) == 46
    for snap in snaps:
        for k in keys:
            assert k in snap and snap[k] >= 0, k
        assert snap["JTOTAL"] > 0 and snap["CTOTAL"] > 0
        assert snap["MIMAINPART"] > 0 and snap["MOMAINPART"] > 0 and snap["BPTASKTIME"] > 0
        assert snap["MWINPUTCNT"] >= 1 and snap["MWINPUT"] > 0
        assert snap["BPBUILD"] > 0 and snap["BPPROBE"] > 0
        if mode != "replicated":
            assert snap["HILOCAL"] > 0 and snap["HOLOCAL"] > 0 and snap["HOGLOBAL"] > 0
            assert snap["LPPART"] > 0 and snap["LPHISTCOMP"] > 0 and snap["LPMEMSIZE"] > 0
            assert snap["MWINPUTCNT"] == 2 * (3 if mode.endswith("3") else 1)
