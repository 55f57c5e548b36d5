"""End-to-end HashJoin engine (single process) on host and device."""
import pytest

from conftest import devices


def run_join(C, dev, G_R, G_S, outer_dist="UNIQUE", cfg=None, theta=0.75):
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(distribution=getattr(C.KeyDistribution, outer_dist), seed=4321,
                      domain=0 if outer_dist == "UNIQUE" else G_R, zipf_theta=theta)
    R = C.Relation(G_R, G_R, loc, 0)
    S = C.Relation(G_S, G_S, loc, 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    j = C.HashJoin(R, S, ctx, cfg or C.JoinConfig())
    res = j.run()
    return res, C.Relation.expected_matches(inner, G_R, outer, G_S), j


@pytest.mark.gpu
def test_bitmap_mixed_cursor_widths(C, cuda):
    """1M inner x 2.2B outer: the outer side's claim slices need 8-byte
    cursors, so the inner side must use them too (the fused bitmap kernel
    reads both with one slice type; this used to fail a CHECK)."""
    cfg = C.JoinConfig()
    res, exp, j = run_join(C, "cuda", 1 << 20, 2_200_000_000, "UNIFORM", cfg=cfg)
    assert j.plan.bitmap_join
    assert res["global_matches"] == exp


@pytest.mark.parametrize("dev", devices())
def test_bitmap_key_shift_edge(C, dev):
    """key_shift + bitmap bits == 64 (2^20 dense keys, 10 network bits, 10
    bitmap bits, key_shift 54): the bitmap pass reads 4-byte key fragments,
    and partial probe batches must not count padding lanes as matches."""
    cfg = C.JoinConfig()
    cfg.key_shift = 54
    cfg.network_bits = 10  # (with fewer network bits the fragments outgrow the word: key-only plan)
    cfg.replicate_bitmap = C.PlanChoice.ON  # the host path takes the bitmap only when forced
    res, exp, j = run_join(C, dev, 1 << 20, (1 << 20) + 12_345, "UNIFORM", cfg=cfg)
    assert j.plan.bitmap_join and j.plan.key_shift + j.plan.bitmap_bits == 64, j.plan
    assert res["global_matches"] == exp


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("dist", ["UNIQUE", "UNIFORM", "ZIPF", "MODULO"])
@pytest.mark.parametrize("bitmap", [True, False])
def test_join_matches_oracle(C, dev, dist, bitmap):
    cfg = C.JoinConfig()
    cfg.bitmap_join = bitmap
    if bitmap:
        cfg.replicate_bitmap = C.PlanChoice.ON  # the host path takes it only when forced
    res, exp, j = run_join(C, dev, 300_000, 500_000 if dist != "UNIQUE" else 300_000, dist, cfg=cfg)
    assert res["global_matches"] == exp
    assert j.plan.bitmap_join == bitmap == res["bitmap_join"]


@pytest.mark.parametrize("dev", devices())
def test_join_single_level(C, dev):
    cfg = C.JoinConfig()
    cfg.two_level = False
    cfg.bitmap_join = False
    res, exp, j = run_join(C, dev, 200_000, 200_000, cfg=cfg)
    assert not j.plan.two_level
    assert res["global_matches"] == exp


@pytest.mark.parametrize("dev", devices())
def test_join_wide_and_materialize(C, dev):
    cfg = C.JoinConfig()
    cfg.format = C.TupleFormat.WIDE
    cfg.materialize = True
    res, exp, j = run_join(C, dev, 100_000, 100_000, cfg=cfg)
    assert res["global_matches"] == exp == res["output_pairs"]
    out = j.output()
    assert out.shape == (exp, 2)


@pytest.mark.parametrize("dev", devices())
def test_output_invalid_after_workspace_reuse(C, dev):
    """output() reads the pairs from the engine's workspace: once a later join
    on the same context has rewound it, the call raises instead of returning
    (or, on a freed device buffer, crashing on) whatever the memory holds now."""
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    G = 50_000
    R = C.Relation(G, G, loc, 0)
    S = C.Relation(G, G, loc, 0)
    R.generate(C.GenSpec(seed=1234), 0)
    S.generate(C.GenSpec(seed=4321), 0)
    cfg = C.JoinConfig()
    cfg.materialize = True
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.run()["output_pairs"] == G
    assert j.output().shape == (G, 2)
    j.run()
    assert j.output().shape == (G, 2)  # still the last run of this join
    ctx.reset_scratch()  # what the next join on the context does first
    with pytest.raises(RuntimeError, match="reused"):
        j.output()


@pytest.mark.parametrize("dev", devices())
def test_join_repeatable(C, dev):
    res, exp, j = run_join(C, dev, 200_000, 200_000)
    for _ in range(3):
        assert j.run()["global_matches"] == exp


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1 << 24, 128_000_000])
def test_join_large_device(C, cuda, G):
    res, exp, j = run_join(C, "cuda", G, G)
    assert res["global_matches"] == exp


@pytest.mark.gpu
def test_pinned_host_relations(C, cuda):
    """Relations in pinned host memory are joined in place by the device engine
    (zero-copy reads over the host link: inputs larger than HBM)."""
    n = 1 << 22
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    R = C.Relation(n, n, "pinned", 0)
    S = C.Relation(n, n, "pinned", 0)
    assert R.location() == "pinned"
    R.generate(C.GenSpec(seed=11), 0)
    S.generate(C.GenSpec(seed=12), 0)
    j = C.HashJoin(R, S, ctx, C.JoinConfig())
    assert j.run()["global_matches"] == n
    link = C.ops.bench_host_link(1 << 26, 0, 2)
    assert link["h2d_GBps"] > 1 and link["zero_copy_read_GBps"] > 1


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("fmt", ["COMPRESSED", "WIDE"])
@pytest.mark.parametrize("inner_dist", ["UNIQUE", "UNIFORM"])
def test_materialized_pairs_exact(C, dev, fmt, inner_dist):
    """Every materialized (rid_inner, rid_outer) pair joins equal keys, and the
    pair multiset is exactly the join (duplicate build keys exercise the
    more-than-two-matches path of the probe)."""
    import torch
    G_R, G_S = 150_000, 400_000
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    inner = C.GenSpec(distribution=getattr(C.KeyDistribution, inner_dist), seed=77,
                      domain=0 if inner_dist == "UNIQUE" else G_R // 4)
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=78, domain=G_R, zipf_theta=0.9)
    R = C.Relation(G_R, G_R, loc, 0)
    S = C.Relation(G_S, G_S, loc, 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    cfg = C.JoinConfig()
    cfg.format = getattr(C.TupleFormat, fmt)
    cfg.materialize = True
    j = C.HashJoin(R, S, ctx, cfg)
    res = j.run()
    Rt, St = R.to_tensor().cpu(), S.to_tensor().cpu()
    dom = int(max(Rt[:, 0].max(), St[:, 0].max())) + 1
    exp = int((torch.bincount(Rt[:, 0], minlength=dom) * torch.bincount(St[:, 0], minlength=dom)).sum())
    assert res["global_matches"] == exp == res["output_pairs"] and not res["output_overflow"]
    pairs = j.output()
    assert pairs.shape == (exp, 2)
    keyR = torch.empty(G_R, dtype=torch.int64)
    keyR[Rt[:, 1]] = Rt[:, 0]
    keyS = torch.empty(G_S, dtype=torch.int64)
    keyS[St[:, 1]] = St[:, 0]
    assert torch.equal(keyR[pairs[:, 0]], keyS[pairs[:, 1]])
    assert torch.unique(pairs[:, 0] * G_S + pairs[:, 1]).numel() == exp


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("fmt", ["COMPRESSED", "WIDE"])
def test_key_hashing(C, dev, fmt):
    """Structured low key bits (sparse TPC-H order keys use 8 of every 32
    values) switch the radix digits to a bijective key mix: AUTO detects it,
    results equal the raw-digit plan, and forcing ON keeps exact pairs."""
    import torch
    G_R, G_S = 1 << 17, 1 << 19
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    inner = C.GenSpec(C.KeyDistribution.UNIQUE, 5, 0, 0, 0.75, True)
    outer = C.GenSpec(C.KeyDistribution.MODULO, 6, G_R, 0, 0.75, True)
    R = C.Relation(G_R, G_R, loc, 0)
    S = C.Relation(G_S, G_S, loc, 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
    assert exp == G_S
    runs = {}
    for mode in ("AUTO", "OFF", "ON"):
        cfg = C.JoinConfig()
        cfg.format = getattr(C.TupleFormat, fmt)
        cfg.key_hashing = getattr(C.KeyHashing, mode)
        cfg.materialize = True
        j = C.HashJoin(R, S, ctx, cfg)
        runs[mode] = (j.plan.key_mix, j.run(), j.output())
    assert runs["AUTO"][0] and runs["ON"][0] and not runs["OFF"][0]
    for mode, (_, res, pairs) in runs.items():
        assert res["global_matches"] == exp, mode
        assert pairs.shape == (exp, 2)
    Rt, St = R.to_tensor().cpu(), S.to_tensor().cpu()
    keyR = torch.empty(G_R, dtype=torch.int64)
    keyR[Rt[:, 1]] = Rt[:, 0]
    keyS = torch.empty(G_S, dtype=torch.int64)
    keyS[St[:, 1]] = St[:, 0]
    pairs = runs["ON"][2]
    assert torch.equal(keyR[pairs[:, 0]], keyS[pairs[:, 1]])
    # dense keys keep raw digits
    D = C.Relation(G_R, G_R, loc, 0)
    D.generate(C.GenSpec(seed=9), 0)
    assert not C.HashJoin(D, D, ctx, C.JoinConfig()).plan.key_mix


@pytest.mark.gpu
@pytest.mark.parametrize("dist,fmt,mat", [("UNIQUE", "COMPRESSED", False), ("ZIPF", "COMPRESSED", False),
                                          ("MODULO", "WIDE", False), ("UNIFORM", "COMPRESSED", True)])
def test_sampled_network_pass(C, cuda, dist, fmt, mat):
    """Single-rank device joins size the network pass from a sampled histogram
    (no full histogram read); results equal the exact path."""
    G_R, G_S = 1 << 22, 3 << 21
    out = {}
    for mode in ("SAMPLED", "EXACT"):
        cfg = C.JoinConfig()
        cfg.network_histogram = getattr(C.HistogramMode, mode)
        cfg.local_histogram = getattr(C.HistogramMode, mode)
        cfg.format = getattr(C.TupleFormat, fmt)
        cfg.materialize = mat
        cfg.bitmap_join = False  # the two-level pass is under test here
        res, exp, j = run_join(C, "cuda", G_R, G_S, dist, cfg=cfg)
        assert j.plan.sampled_network == (mode == "SAMPLED")
        assert res["sampled_network"] == (mode == "SAMPLED") and res["network_fallbacks"] == 0
        assert res["sampled_local"] == (mode == "SAMPLED") and res["local_fallbacks"] == 0
        assert res["global_matches"] == exp
        for _ in range(2):
            assert j.run()["global_matches"] == exp
        out[mode] = j.output() if mat else None
    if mat:
        import torch
        a, b = (torch.sort(out[m][:, 0] * G_S + out[m][:, 1]).values for m in ("SAMPLED", "EXACT"))
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_sampled_network_single_level(C, cuda):
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    cfg.two_level = False
    cfg.bitmap_join = False
    res, exp, j = run_join(C, "cuda", 1 << 21, 1 << 21, cfg=cfg)
    assert j.plan.sampled_network and res["sampled_network"] and res["global_matches"] == exp


@pytest.mark.gpu
def test_sampled_network_overflow_falls_back(C, cuda):
    """Adversarial layout for the sample: every 4096-tuple tile holds a single
    network digit, so the sampled tiles (1 in 16 of each workgroup's range) miss
    most digits.  Slices overflow, the join re-runs exactly, and later joins
    stay on the exact path."""
    import torch
    n = 1 << 22
    i = torch.arange(n, device="cuda")
    keys = i * 512 + (i // 4096) % 512  # unique; low 9 bits = tile index mod 512
    R = torch.stack([keys, i], 1).contiguous()
    S = torch.stack([keys.flip(0), i], 1).contiguous()
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    cfg.key_hashing = C.KeyHashing.OFF
    cfg.network_bits = 9
    cfg.max_partition_blocks = 16  # 64 tiles per workgroup, 4 of them sampled
    j = C.HashJoin(C.Relation.from_tensor(R, n), C.Relation.from_tensor(S, n), ctx, cfg)
    res = j.run()
    assert res["network_fallbacks"] == 1 and not res["sampled_network"]
    assert res["global_matches"] == n
    res = j.run()
    assert res["network_fallbacks"] == 0 and res["global_matches"] == n


def test_sampled_network_host_is_exact(C):
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    res, exp, j = run_join(C, "cpu", 100_000, 100_000, cfg=cfg)
    assert not j.plan.sampled_network and not res["sampled_network"] and res["global_matches"] == exp


@pytest.mark.gpu
def test_sampled_local_overflow_falls_back(C, cuda):
    """Inside every network partition the local digits rise with input order,
    so the sampled first tile of each local work item sees only low digits:
    slots overflow, the local pass and build/probe are redone exactly, and
    later joins use the exact local pass."""
    import torch
    n = 1 << 26
    i = torch.arange(n, device="cuda")
    net, j = i % 512, i // 512
    keys = ((j % 256) << 18) | ((j // 256) << 9) | net  # unique; local digit = j // 256 rises with i
    R = torch.stack([keys, i], 1).contiguous()
    S = torch.stack([keys.flip(0), i], 1).contiguous()
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.EXACT
    cfg.local_histogram = C.HistogramMode.SAMPLED
    cfg.key_hashing = C.KeyHashing.OFF
    cfg.network_bits, cfg.local_bits = 9, 9
    cfg.bitmap_join = False
    j = C.HashJoin(C.Relation.from_tensor(R, n), C.Relation.from_tensor(S, n), ctx, cfg)
    res = j.run()
    assert res["local_fallbacks"] == 1 and not res["sampled_local"]
    assert res["global_matches"] == n
    res = j.run()
    assert res["local_fallbacks"] == 0 and not res["sampled_local"] and res["global_matches"] == n


@pytest.mark.gpu
@pytest.mark.parametrize("sampled", [True, False])
@pytest.mark.parametrize("G", [1 << 22, 20_000_003])
def test_split_local_output(C, cuda, sampled, G):
    """Split local pass output (u32 rid + u16 fragment columns): same counts
    and the same materialized pairs as the 8-byte layout, exact and sampled
    local passes, skewed outer side."""
    import torch
    out = {}
    for narrow in (True, False):
        cfg = C.JoinConfig()
        cfg.split_local = narrow
        cfg.materialize = True
        cfg.local_histogram = C.HistogramMode.SAMPLED if sampled else C.HistogramMode.EXACT
        res, exp, j = run_join(C, "cuda", G, G + 12345, "ZIPF", cfg=cfg, theta=0.6)
        assert j.plan.split_local == narrow
        assert res["global_matches"] == exp and res["local_fallbacks"] == 0
        p = j.output()
        out[narrow] = p[torch.argsort(p[:, 1] * (1 << 32) + p[:, 0])]
    assert torch.equal(out[True], out[False])


@pytest.mark.gpu
@pytest.mark.parametrize("local", ["SAMPLED", "EXACT"])
@pytest.mark.parametrize("dist", ["UNIQUE", "ZIPF", "MODULO"])
def test_fragment_two_level(C, cuda, dist, local):
    """Count-only two-level plan on fragments (JoinPlan::fragments): the
    sampled network pass writes u32 key fragments, the local pass only the
    u16 fragment column; counts equal the reference, duplicates included,
    repeated runs included."""
    cfg = C.JoinConfig()
    cfg.bitmap_join = False
    cfg.local_histogram = getattr(C.HistogramMode, local)
    G = 20_000_003
    res, exp, j = run_join(C, "cuda", G, G + 4321, dist, cfg=cfg, theta=0.9)
    assert j.plan.fragments and j.plan.sampled_network and j.plan.split_local, j.plan
    assert res["global_matches"] == exp and res["network_fallbacks"] == 0
    for _ in range(2):
        assert j.run()["global_matches"] == exp


@pytest.mark.gpu
def test_fragment_two_level_network_overflow(C, cuda):
    """A sampled network pass that overflows on the fragment plan re-runs on
    the exact 8-byte path (the local pass follows each window's format)."""
    import torch
    n = 1 << 22
    i = torch.arange(n, device="cuda")
    keys = i * 512 + (i // 4096) % 512
    R = torch.stack([keys, i], 1).contiguous()
    S = torch.stack([keys.flip(0), i], 1).contiguous()
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    cfg.key_hashing = C.KeyHashing.OFF
    cfg.network_bits, cfg.local_bits = 9, 6  # 31-bit keys: 16-bit fragments after both passes
    cfg.bitmap_join = False
    cfg.max_partition_blocks = 16
    j = C.HashJoin(C.Relation.from_tensor(R, n), C.Relation.from_tensor(S, n), ctx, cfg)
    assert j.plan.fragments, j.plan
    res = j.run()
    assert res["network_fallbacks"] == 1 and res["global_matches"] == n
    assert j.run()["global_matches"] == n


@pytest.mark.gpu
@pytest.mark.parametrize("dist", ["UNIQUE", "ZIPF", "MODULO"])
@pytest.mark.parametrize("split", [True, False])
def test_direct_count_table(C, cuda, dist, split):
    """Count-only build/probe with direct-addressed LDS counts (fragments of at
    most 13 bits) equals the hash-table path, duplicates on both sides included."""
    counts = {}
    for direct in (True, False):
        cfg = C.JoinConfig()
        cfg.bitmap_join = False
        cfg.direct_count = direct
        cfg.split_local = split
        G = 6_000_011
        res, exp, j = run_join(C, "cuda", G, G + 777, dist, cfg=cfg, theta=0.9)
        assert j.plan.key_bits - j.plan.network_bits - j.plan.local_bits <= 13
        assert res["global_matches"] == exp
        counts[direct] = res["global_matches"]
    assert counts[True] == counts[False]


@pytest.mark.gpu
@pytest.mark.parametrize("r_chunk", [0, 512])
def test_materialize_split_duplicates(C, cuda, r_chunk):
    """Materializing build/probe of the split layout (bpMatSplitKernel): 16
    duplicates of every inner key (chain re-walk for the extra matches) and,
    with r_chunk=512, inner partitions split over several LDS tables."""
    import torch
    G_R, G_S = 160_000, 300_000
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    inner = C.GenSpec(distribution=C.KeyDistribution.MODULO, seed=91, domain=G_R // 16)
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=92, domain=G_R // 8, zipf_theta=0.5)
    R = C.Relation(G_R, G_R, "device", 0)
    S = C.Relation(G_S, G_S, "device", 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    cfg = C.JoinConfig()
    cfg.materialize = True
    cfg.r_chunk = r_chunk
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.plan.split_local
    res = j.run()
    Rt, St = R.to_tensor().cpu(), S.to_tensor().cpu()
    dom = int(max(Rt[:, 0].max(), St[:, 0].max())) + 1
    exp = int((torch.bincount(Rt[:, 0], minlength=dom) * torch.bincount(St[:, 0], minlength=dom)).sum())
    assert res["global_matches"] == exp == res["output_pairs"] and not res["output_overflow"]
    pairs = j.output().cpu()
    keyR = torch.empty(G_R, dtype=torch.int64)
    keyR[Rt[:, 1]] = Rt[:, 0]
    keyS = torch.empty(G_S, dtype=torch.int64)
    keyS[St[:, 1]] = St[:, 0]
    assert torch.equal(keyR[pairs[:, 0]], keyS[pairs[:, 1]])
    assert torch.unique(pairs[:, 0] * G_S + pairs[:, 1]).numel() == exp


@pytest.mark.gpu
@pytest.mark.parametrize("r_chunk,cap", [(0, 0), (512, 1000), (2048, 0)])
def test_fused_row_materialization(C, cuda, r_chunk, cap):
    """join_materialized at N = 1: the split layout's materialize pass writes
    whole 80-byte rows (bpMatRowsKernel for inner chunks <= 1024, else
    bpMatSplitKernel<true>).  16 duplicates of every inner
    key (windows of more than 64 rows per wave), Zipf outer; the rows equal
    those of run() + materialize_payloads as a multiset, and a capacity that is
    too small (cap=1000) is re-run exactly sized."""
    import torch
    G_R, G_S = 160_000, 300_000
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    inner = C.GenSpec(distribution=C.KeyDistribution.MODULO, seed=91, domain=G_R // 16)
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=92, domain=G_R // 8, zipf_theta=0.5)
    R = C.Relation(G_R, G_R, "device", 0)
    S = C.Relation(G_S, G_S, "device", 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    rows_a = C.ops.generate_payload(G_R, 0, 0x51, "cuda:0")
    rows_b = C.ops.generate_payload(G_S, 0, 0x52, "cuda:0")
    cfg = C.JoinConfig()
    cfg.materialize = True
    cfg.r_chunk = r_chunk
    cfg.output_capacity = cap
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.can_fuse_rows
    res, rows = j.join_materialized(ctx, rows_a, 0, G_R, rows_b, 0, G_S)
    Rt, St = R.to_tensor().cpu(), S.to_tensor().cpu()
    dom = int(max(Rt[:, 0].max(), St[:, 0].max())) + 1
    exp = int((torch.bincount(Rt[:, 0], minlength=dom) * torch.bincount(St[:, 0], minlength=dom)).sum())
    assert res["rows_fused"] and not res["output_overflow"]
    assert res["global_matches"] == exp == res["output_pairs"] == rows.shape[0]
    cfg2 = C.JoinConfig()
    cfg2.materialize = True
    cfg2.r_chunk = r_chunk
    j2 = C.HashJoin(R, S, ctx, cfg2)
    res2 = j2.run()
    assert not res2["rows_fused"]
    ref = j2.materialize_payloads(ctx, rows_a, 0, G_R, rows_b, 0, G_S)

    def canon(t):
        t = t.cpu()
        return t[torch.argsort(t[:, 0] * G_S + t[:, 1])]

    assert torch.equal(canon(rows), canon(ref))


@pytest.mark.gpu
@pytest.mark.parametrize("dist", ["UNIQUE", "UNIFORM", "ZIPF"])
def test_bitmap_join(C, cuda, dist):
    """Single-level bitmap join (N == 1, counting, sampled network pass): one
    LDS bitmap per 1024-way network partition, no local pass; counts equal
    the oracle and the two-level path, foreign-key outer sides included."""
    G_R, G_S = 1 << 24, (1 << 24) + 4321
    counts = {}
    for bitmap in (True, False):
        cfg = C.JoinConfig()
        cfg.network_histogram = C.HistogramMode.SAMPLED
        cfg.bitmap_join = bitmap
        res, exp, j = run_join(C, "cuda", G_R, G_S, dist, cfg=cfg, theta=0.9)
        assert j.plan.bitmap_join == bitmap and res["bitmap_join"] == bitmap
        if bitmap:
            assert j.plan.network_bits == 10 and j.plan.bitmap_bits == j.plan.key_bits - 10
            assert res["local_fallbacks"] == 0 and res["local_items"] == 0
        assert res["global_matches"] == exp
        for _ in range(2):
            assert j.run()["global_matches"] == exp
        counts[bitmap] = res["global_matches"]
    assert counts[True] == counts[False]


@pytest.mark.gpu
def test_bitmap_join_duplicate_inner_falls_back(C, cuda):
    """A repeated inner key cannot be counted by a bitmap: the kernel flags it,
    the same join finishes on the two-level pass (exact count), and later
    joins skip the bitmap."""
    import torch
    n = 1 << 24
    i = torch.arange(n, device="cuda")
    keys = i.clone()
    keys[n // 2] = keys[n // 3]  # one duplicate inner key
    R = torch.stack([keys, i], 1).contiguous()
    S = torch.stack([i.flip(0), i], 1).contiguous()
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    j = C.HashJoin(C.Relation.from_tensor(R, n), C.Relation.from_tensor(S, n), ctx, cfg)
    assert j.plan.bitmap_join
    exp = n  # key n//2 lost its inner row, key n//3 matches twice
    res = j.run()
    assert res["local_fallbacks"] == 1 and not res["bitmap_join"] and res["global_matches"] == exp
    res = j.run()
    assert res["local_fallbacks"] == 0 and not res["bitmap_join"] and res["global_matches"] == exp


def test_bitmap_join_config_and_host_plan(C, monkeypatch):
    """The bitmap join is a device single-rank plan: on by default in the
    config, switchable through HPCJOIN_BITMAP_JOIN, never chosen on the host
    path (which runs the two-level pass)."""
    from hpcjoin.utils import config_from_dict, config_to_dict
    assert C.JoinConfig().bitmap_join is True
    monkeypatch.setenv("HPCJOIN_BITMAP_JOIN", "0")
    cfg = config_from_dict({})
    assert cfg.bitmap_join is False and config_to_dict(cfg)["bitmap_join"] is False
    cfg = C.JoinConfig()
    cfg.network_histogram = C.HistogramMode.SAMPLED
    res, exp, j = run_join(C, "cpu", 100_000, 100_000, cfg=cfg)
    assert not j.plan.bitmap_join and not res["bitmap_join"] and res["global_matches"] == exp
    assert "bitmap=0/0" in repr(j.plan)


@pytest.mark.parametrize("dev", devices())
def test_repeated_inner_keys_planned_before_first_join(C, dev):
    """Repeated inner keys are known at plan time -- from the generator
    (Zipf draws) or from a 64K-key sample of an external tensor -- so the
    first join neither attempts a bitmap plan and falls back nor (key-only
    words) starts on quotient tables: no fallback, no re-run, exact."""
    import torch
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    G = 300_000
    for sparse in (False, True):
        inner = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=5, domain=G, zipf_theta=0.9)
        outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=6, domain=G, zipf_theta=0.9)
        inner.sparse64 = outer.sparse64 = sparse
        R = C.Relation(G, G, loc, 0)
        S = C.Relation(G, G, loc, 0)
        R.generate(inner, 0)
        S.generate(outer, 0)
        from helpers import ref_join_count
        exp = ref_join_count(R.to_tensor()[:, 0].cpu(), S.to_tensor()[:, 0].cpu())
        j = C.HashJoin(R, S, ctx, C.JoinConfig())
        assert j.plan.inner_repeats and not j.plan.bitmap_join, j.plan
        assert j.plan_ms >= 0 and j.reserve_ms >= 0
        res = j.run()
        assert res["global_matches"] == exp and res["local_fallbacks"] == 0 and res["reruns"] == 0, res
    # external tensors: sampled
    tdev = "cuda" if dev == "cuda" else "cpu"
    i = torch.arange(G, dtype=torch.int64)
    for keys, rep in ((i % 1000, True), (i.flip(0), False)):
        t = torch.stack([keys, i], 1).contiguous().to(tdev)
        o = torch.stack([i, i], 1).contiguous().to(tdev)
        j = C.HashJoin(C.Relation.from_tensor(t, G), C.Relation.from_tensor(o, G), ctx, C.JoinConfig())
        assert j.plan.inner_repeats == rep, (rep, j.plan)
        from helpers import ref_join_count
        assert j.run()["global_matches"] == ref_join_count(keys, i)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("passes,outer_dist,sparse", [(3, "UNIQUE", False), (4, "ZIPF", False), (2, "UNIFORM", True)])
def test_capacity_spill_passes(C, dev, passes, outer_dist, sparse):
    """Capacity spill: the join runs in `passes` key-hash passes (pass k joins
    the tuples of both sides whose key hashes to k), each a complete join with
    ~1/passes of the workspace; the counts add up to the oracle and equal the
    single-pass join."""
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    G_R, G_S = 150_001, 400_003
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(distribution=getattr(C.KeyDistribution, outer_dist), seed=4321,
                      domain=0 if outer_dist == "UNIQUE" else G_R, zipf_theta=0.9)
    inner.sparse64 = outer.sparse64 = sparse
    if outer_dist == "UNIQUE":
        G_S = G_R
    R = C.Relation(G_R, G_R, loc, 0)
    S = C.Relation(G_S, G_S, loc, 0)
    R.generate(inner, 0)
    S.generate(outer, 0)
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
    got = {}
    for k in (1, passes):
        cfg = C.JoinConfig()
        cfg.passes = k
        j = C.HashJoin(R, S, ctx, cfg)
        assert j.spill_passes == k
        for _ in range(2):
            res = j.run()
            assert res["global_matches"] == exp, (k, res["global_matches"], exp)
            assert res["passes"] == k
        got[k] = res["local_matches"]
        del j
    assert got[1] == got[passes]


@pytest.mark.gpu
@pytest.mark.parametrize("sparse,outer_dist", [(False, "UNIQUE"), (False, "ZIPF"), (True, "UNIQUE")])
def test_capacity_spill_auto_budget(C, cuda, sparse, outer_dist):
    """workspace_budget below the plan's estimate: the planner spills by
    itself and the join stays exact.  Dense unique inner keys (the bitmap
    plan) spill by partition groups -- each group pass reads both relations
    once and writes only its network partitions' fragments; random 63-bit
    keys (the two-level plan) spill by key-hash passes."""
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    G = 1 << 24
    R = C.Relation(G, G, "device", 0)
    S = C.Relation(G, G, "device", 0)
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(distribution=getattr(C.KeyDistribution, outer_dist), seed=4321,
                      domain=0 if outer_dist == "UNIQUE" else G, zipf_theta=0.75)
    inner.sparse64 = outer.sparse64 = sparse
    R.generate(inner, 0)
    S.generate(outer, 0)
    exp = C.Relation.expected_matches(inner, G, outer, G)
    full = C.HashJoin(R, S, ctx, C.JoinConfig())
    est = full.workspace_estimate()
    single = full.run()["global_matches"]
    assert single == exp
    bitmap = full.plan.bitmap_join
    del full
    cfg = C.JoinConfig()
    cfg.workspace_budget = est // 4
    j = C.HashJoin(R, S, ctx, cfg)
    for _ in range(2):
        res = j.run()
        assert res["global_matches"] == exp, res
    if bitmap:
        assert j.spill_passes == 1 and res["group_passes"] >= 4, (res["group_passes"], est)
        assert j.spill_info["group_budget_bytes"] > 0 and res["bitmap_join"]
    else:
        assert j.spill_passes >= 4 and res["passes"] == j.spill_passes, (j.spill_passes, est)


@pytest.mark.gpu
def test_capacity_spill_skewed_inner_key_classes(C, cuda):
    """Zipf inner keys under a workspace budget: every copy of a
    hot key lands in one key-hash pass, so the largest pass is far above 1/K of
    the data.  The planner counts the passes, grows K until the largest one
    fits, and the join stays exact; a key too frequent for any pass count is
    refused with a clear message instead of failing an allocation."""
    import torch
    from helpers import ref_join_count
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    G = 1 << 22
    R = C.Relation(G, G, "device", 0)
    S = C.Relation(G, G, "device", 0)
    R.generate(C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=11, domain=4096, zipf_theta=0.9), 0)
    S.generate(C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=12, domain=4096), 0)
    exp = ref_join_count(R.to_tensor()[:, 0], S.to_tensor()[:, 0])
    est = C.HashJoin(R, S, ctx, C.JoinConfig()).workspace_estimate()
    cfg = C.JoinConfig()
    cfg.workspace_budget = est // 4
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.spill_passes >= 4
    assert j.run()["global_matches"] == exp
    # Two keys only: one key-hash class holds about half the tuples at any K.
    R2 = C.Relation(G, G, "device", 0)
    R2.generate(C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=13, domain=2), 0)
    est2 = C.HashJoin(R2, S, ctx, C.JoinConfig()).workspace_estimate()
    cfg.workspace_budget = est2 // 16
    with pytest.raises(RuntimeError, match="too frequent to spill"):
        C.HashJoin(R2, S, ctx, cfg)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("passes", [0, 3])
def test_materializing_spill_to_host_output(C, dev, passes):
    """A materializing join under a memory budget (passes 0 = the planner's
    choice from workspace_budget, or forced key-hash passes) writes the pairs
    of every pass straight into a caller-owned pinned host buffer
    (JoinConfig.output_host), the reference UVA driver's host output; the
    pair multiset equals the join."""
    import torch
    G_R, G_S = 120_000, 300_000
    loc = "device" if dev == "cuda" else "host"
    ctx = C.ExecContext(loc, 0 if loc == "device" else -1, C.LocalCommunicator())
    R = C.Relation(G_R, G_R, loc, 0)
    S = C.Relation(G_S, G_S, loc, 0)
    R.generate(C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=91, domain=G_R // 3), 0)
    S.generate(C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=92, domain=G_R, zipf_theta=0.9), 0)
    Rt, St = R.to_tensor().cpu(), S.to_tensor().cpu()
    dom = int(max(Rt[:, 0].max(), St[:, 0].max())) + 1
    exp = int((torch.bincount(Rt[:, 0], minlength=dom) * torch.bincount(St[:, 0], minlength=dom)).sum())
    out = C.pinned_pairs(exp + 4096) if dev == "cuda" else torch.zeros((exp + 4096, 2), dtype=torch.int64)
    cfg = C.JoinConfig()
    cfg.materialize = True
    cfg.output_host = out.data_ptr()
    cfg.output_capacity = out.shape[0]
    if passes:
        cfg.passes = passes
    elif dev == "cuda":
        probe = C.JoinConfig()
        probe.materialize = True
        probe.output_host = out.data_ptr()
        probe.output_capacity = out.shape[0]
        cfg.workspace_budget = C.HashJoin(R, S, ctx, probe).workspace_estimate() // 4
    else:
        pytest.skip("the automatic spill plans device workspaces only")
    j = C.HashJoin(R, S, ctx, cfg)
    assert j.spill_passes >= (passes or 2), j.spill_passes
    res = j.run()
    assert res["global_matches"] == exp == res["output_pairs"] and not res["output_overflow"]
    if dev == "cuda":
        torch.cuda.synchronize()
    pairs = out[:exp].clone()
    assert torch.equal(j.output(), pairs)
    keyR = torch.empty(G_R, dtype=torch.int64)
    keyR[Rt[:, 1]] = Rt[:, 0]
    keyS = torch.empty(G_S, dtype=torch.int64)
    keyS[St[:, 1]] = St[:, 0]
    assert torch.equal(keyR[pairs[:, 0]], keyS[pairs[:, 1]])
    assert torch.unique(pairs[:, 0] * G_S + pairs[:, 1]).numel() == exp
    # Too small a buffer is refused with a clear message, not written past.
    cfg.output_capacity = exp // 2
    with pytest.raises(RuntimeError, match="host output buffer"):
        C.HashJoin(R, S, ctx, cfg).run()
