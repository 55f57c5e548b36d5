"""Kernel-level numerics: every HIP kernel (device param, marked gpu) and its
host twin (host param) against plain PyTorch references."""
import pytest
import torch

from conftest import devices
from helpers import gen, ref_join_count, sorted_pairs, unpack


@pytest.mark.parametrize("dev", devices())
def test_generate_unique_is_permutation(C, dev):
    n = 100_003
    t = gen(C, n, device=dev)
    keys = t[:, 0].cpu()
    assert torch.equal(torch.sort(keys).values, torch.arange(n))
    assert torch.equal(t[:, 1].cpu(), torch.arange(n))


@pytest.mark.gpu
def test_generate_device_matches_host(C, cuda):
    for dist in ["UNIQUE", "MODULO", "UNIFORM", "DENSE"]:
        h = gen(C, 50_000, dist=dist, domain=40_000 if dist != "UNIQUE" else 0, global_size=200_000, offset=777)
        d = gen(C, 50_000, dist=dist, domain=40_000 if dist != "UNIQUE" else 0, global_size=200_000, offset=777,
                device="cuda")
        assert torch.equal(h, d.cpu()), dist


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("bits", [1, 5, 8, 11])
def test_net_histogram(C, dev, bits):
    t = gen(C, 300_001, device=dev)
    h = C.ops.net_histogram(t, bits)
    ref = torch.bincount((t[:, 0] & ((1 << bits) - 1)).cpu(), minlength=1 << bits)
    assert torch.equal(h.cpu(), ref)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("bits,max_blocks", [(5, 2048), (9, 2048), (10, 7), (11, 64)])
@pytest.mark.parametrize("key_bits", [30, 64])  # 30: digit carried in spare top bits; 64: LDS digit array
def test_net_partition_compressed(C, dev, bits, max_blocks, key_bits):
    n = 250_000 + 17
    t = gen(C, n, device=dev, dist="UNIFORM", domain=1 << 30)
    out, begin = C.ops.net_partition(t, bits, 32, False, max_blocks, key_bits)
    ref_sizes = torch.bincount((t[:, 0] & ((1 << bits) - 1)).cpu(), minlength=1 << bits)
    assert torch.equal(begin[1:] - begin[:-1], ref_sizes)
    k, r = unpack(out, bits, 32, begin)
    assert torch.equal(sorted_pairs(k.cpu(), r.cpu()), sorted_pairs(t[:, 0].cpu(), t[:, 1].cpu()))


@pytest.mark.parametrize("dev", devices())
def test_net_partition_wide(C, dev):
    n = 100_000
    t = gen(C, n, device=dev)
    t[:, 0] = t[:, 0] * 0x10001 + (1 << 40)  # keys far beyond the CompressedTuple range
    out, begin = C.ops.net_partition(t.contiguous(), 7, 64, True)
    p = torch.repeat_interleave(torch.arange(128), begin[1:] - begin[:-1])
    assert torch.equal((out[:, 0].cpu() & 127), p)
    assert torch.equal(torch.sort(out[:, 0].cpu()).values, torch.sort(t[:, 0].cpu()).values)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("bits", [0, 4, 9])
def test_local_partition(C, dev, bits):
    n, b1, ks = 400_000, 6, 32
    t = gen(C, n, device=dev, dist="UNIFORM", domain=1 << 28)
    v, b = C.ops.net_partition(t, b1, ks)
    v2, pb2 = C.ops.local_partition(v, b, ks, bits)
    F2 = 1 << bits
    assert pb2.numel() == (1 << b1) * F2 + 1 and int(pb2[-1]) == n
    sizes = (pb2[1:] - pb2[:-1]).cpu()
    q = torch.repeat_interleave(torch.arange((1 << b1) * F2), sizes)
    assert torch.equal(((v2.cpu() >> ks) & (F2 - 1)), q % F2)
    # network partition preserved
    assert torch.equal(torch.sort(v2.cpu()).values, torch.sort(v.cpu()).values)
    k1, _ = unpack(v, b1, ks, b.cpu())
    pk = torch.repeat_interleave(torch.arange(1 << b1), b[1:] - b[:-1])
    assert torch.equal(k1.cpu() & ((1 << b1) - 1), pk)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("dist", ["UNIQUE", "UNIFORM", "ZIPF"])
def test_build_probe_count(C, dev, dist):
    n_r, n_s, b1, b2, ks = 200_000, 300_000, 6, 5, 32
    R = gen(C, n_r, device=dev, seed=11)
    S = gen(C, n_s, device=dev, seed=12, dist=dist, domain=n_r if dist != "UNIQUE" else 0)
    ref = ref_join_count(R[:, 0].cpu(), S[:, 0].cpu())
    rv, rb = C.ops.net_partition(R, b1, ks)
    sv, sb = C.ops.net_partition(S, b1, ks)
    rv2, rpb = C.ops.local_partition(rv, rb, ks, b2)
    sv2, spb = C.ops.local_partition(sv, sb, ks, b2)
    res = C.ops.build_probe(rv2, sv2, rpb, spb, ks + b2, ks)
    assert res["matches"] == ref


@pytest.mark.parametrize("dev", devices())
def test_build_probe_skew_splits_items(C, dev):
    # 2 network partitions only: a few huge partitions force R- and S-chunking.
    n, b1, ks = 60_000, 1, 32
    R = gen(C, n, device=dev, seed=3)
    S = gen(C, 3 * n, device=dev, seed=4, dist="ZIPF", domain=n, theta=0.9)
    ref = ref_join_count(R[:, 0].cpu(), S[:, 0].cpu())
    rv, rb = C.ops.net_partition(R, b1, ks)
    sv, sb = C.ops.net_partition(S, b1, ks)
    res = C.ops.build_probe(rv, sv, rb, sb, ks, ks, r_chunk=1024, s_chunk=4096)
    assert res["matches"] == ref
    if dev == "cuda":
        assert res["work_items"] > 2


@pytest.mark.parametrize("dev", devices())
def test_build_probe_duplicates_inner(C, dev):
    # inner side with duplicate keys (multiset semantics)
    n = 50_000
    R = gen(C, n, device=dev, seed=5, dist="UNIFORM", domain=n // 4)
    S = gen(C, n, device=dev, seed=6, dist="UNIFORM", domain=n // 4)
    ref = ref_join_count(R[:, 0].cpu(), S[:, 0].cpu())
    rv, rb = C.ops.net_partition(R, 4, 32)
    sv, sb = C.ops.net_partition(S, 4, 32)
    res = C.ops.build_probe(rv, sv, rb, sb, 32, 32)
    assert res["matches"] == ref


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("wide", [False, True])
def test_build_probe_materialize(C, dev, wide):
    n = 80_000
    R = gen(C, n, device=dev, seed=7)
    S = gen(C, n, device=dev, seed=8, dist="UNIFORM", domain=n)
    if wide:
        rv, rb = C.ops.net_partition(R, 5, 64, True)
        sv, sb = C.ops.net_partition(S, 5, 64, True)
        res = C.ops.build_probe(rv, sv, rb, sb, 64, 64, wide=True, materialize=True, out_capacity=2 * n,
                                r_chunk=2048)
    else:
        rv, rb = C.ops.net_partition(R, 5, 32)
        sv, sb = C.ops.net_partition(S, 5, 32)
        res = C.ops.build_probe(rv, sv, rb, sb, 32, 32, materialize=True, out_capacity=2 * n, r_chunk=4096)
    assert res["matches"] == n and res["output_count"] == n
    pairs = res["pairs"][:n].cpu()
    # every pair joins: key(R[rid_r]) == key(S[rid_s])
    rk = R[:, 0].cpu()[pairs[:, 0]]
    sk = S[:, 0].cpu()[pairs[:, 1]]
    assert torch.equal(rk, sk)
    assert torch.equal(torch.sort(pairs[:, 1]).values, torch.arange(n))


@pytest.mark.gpu
def test_scan_u32(C, cuda):
    for n in [1, 100, 2048, 2049, 1_000_003]:
        x = torch.randint(0, 100, (n,), dtype=torch.int32, device="cuda")
        out = C.ops.scan_u32(x).cpu()
        ref = torch.zeros(n + 1, dtype=torch.int64)
        ref[1:] = torch.cumsum(x.cpu().long(), 0)
        assert torch.equal(out.long(), ref), n


@pytest.mark.parametrize("dev", devices())
def test_npj_count(C, dev):
    R = gen(C, 100_000, device=dev, seed=1)
    S = gen(C, 150_000, device=dev, seed=2, dist="ZIPF", domain=100_000)
    assert C.ops.npj_count(R, S) == 150_000


@pytest.mark.parametrize("dev", devices())
def test_npj_join_pairs(C, dev):
    """Materializing NPJ (duplicate inner keys: every copy pairs with every
    outer match) against the torch pair oracle."""
    from hpcjoin.models.npj import NoPartitionJoin
    from hpcjoin.utils import join_pairs_reference
    R = gen(C, 5_000, device=dev, seed=3, dist="ZIPF", domain=3_000)
    S = gen(C, 8_000, device=dev, seed=4, dist="ZIPF", domain=4_000)
    npj = NoPartitionJoin()
    pairs = npj.join(R, S).cpu()
    assert pairs.shape[0] == npj.count(R, S) > 0
    ref = join_pairs_reference(R.cpu(), S.cpu())
    got = pairs[torch.argsort(pairs[:, 0] * (1 << 32) + pairs[:, 1])]
    assert torch.equal(got, ref)
    assert npj.timings["join_ms"] > 0 and npj.throughput(R, S) > 0


@pytest.mark.gpu
def test_global_atomic_scatter_ablation(C, cuda):
    t = gen(C, 200_000, device="cuda")
    v, b = C.ops.net_partition(t, 6, 32)
    v2 = C.ops.net_scatter_global_atomic(t, 6, 32, b)
    assert torch.equal(torch.sort(v2.cpu()).values, torch.sort(v.cpu()).values)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("w,rid_bits", [(48, 27), (33, 20), (64, 32), (7, 3), (50, 29)])
def test_wire_codec_roundtrip(C, dev, w, rid_bits):
    """Bit-packed exchange format: segments of odd lengths with their own rid
    bases round-trip exactly, and the device packing equals the host's
    (independent bit-stream implementation) word for word."""
    import torch
    g = torch.Generator().manual_seed(w)
    key_shift = 32
    key_bits = w - rid_bits
    segs = [(0, 1, 5), (1, 64, 1000), (65, 130, 0), (300, 0, 7), (300, 1000, 1 << 20)]
    n = 1300
    rid = torch.zeros(n, dtype=torch.int64)
    frag = torch.randint(0, 1 << key_bits, (n,), generator=g, dtype=torch.int64)
    for off, cnt, base in segs:  # rids must stay below 2^key_shift
        base = base if rid_bits < 32 else 0
        rid[off:off + cnt] = base + torch.randint(0, 1 << rid_bits, (cnt,), generator=g, dtype=torch.int64)
    segs = [(off, cnt, base if rid_bits < 32 else 0) for off, cnt, base in segs]
    raw = rid | (frag << key_shift)
    host_wire = C.ops.wire_pack(raw, w, rid_bits, key_shift, segs)
    assert host_wire.numel() == sum((c + 63) // 64 * w for _, c, _ in segs)
    back = torch.full_like(raw, -1)
    C.ops.wire_unpack(host_wire, back, w, rid_bits, key_shift, segs)
    mask = back != -1
    assert mask.sum() == sum(c for _, c, _ in segs)
    assert torch.equal(back[mask], raw[mask])
    if dev == "cuda":
        dwire = C.ops.wire_pack(raw.cuda(), w, rid_bits, key_shift, segs)
        assert torch.equal(dwire.cpu(), host_wire)
        dback = torch.full_like(raw, -1).cuda()
        C.ops.wire_unpack(dwire, dback, w, rid_bits, key_shift, segs)
        assert torch.equal(dback.cpu(), back)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [-1, 0, 1, 2, 3])
def test_gather_rows_shapes(C, cuda, mode):
    """The random row gather (operator kernel and the microbenchmark shapes)
    equals torch indexing of the 32-byte rows."""
    import torch
    n = 100_003
    payload = C.ops.generate_payload(n, 0, 5, "cuda:0")
    rids = torch.randperm(n, device="cuda", dtype=torch.int64)
    out = C.ops.gather_rows(rids, 0, payload, mode)
    assert torch.equal(out, payload[rids])


@pytest.mark.gpu
def test_project_keys_and_global_bitmap_probe(C, cuda):
    """Streaming-ceiling and whole-key-space probe microbenchmark kernels
    compute what they claim (key >> shift; count of keys whose bit is set)."""
    import torch
    n = 1 << 18
    R = C.Relation(n, n, "device", 0)
    R.generate(C.GenSpec(seed=9), 0)
    t = R.to_tensor()
    for ipt in (1, 4, 8):
        assert torch.equal(C.ops.project_keys(t, 10, ipt).to(torch.int64) & 0xFFFFFFFF,
                           (t[:, 0] >> 10) & 0xFFFFFFFF)
    even = torch.arange(0, 1 << 18, 2, device="cuda")  # set the bits of even keys
    words = torch.zeros((1 << 18) // 32, dtype=torch.int64, device="cuda")
    words.index_add_(0, even >> 5, torch.ones_like(even) << (even & 31))  # distinct bits: sum == OR
    bm = words.to(torch.int32)
    got = int(C.ops.probe_bitmap_global(t, bm, (1 << 18) - 1, 8).item())
    assert got == int(((t[:, 0] & ((1 << 18) - 1)) % 2 == 0).sum().item())
