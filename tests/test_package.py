"""Python package surface: ops / models / utils / parallel, and the
measurement files (reference key names)."""
import os

import pytest
import torch

from conftest import devices


def test_compress_roundtrip():
    from hpcjoin.ops import compress, decompress
    keys = torch.randint(0, 1 << 36, (1000,), dtype=torch.int64)
    rids = torch.randint(0, 1 << 31, (1000,), dtype=torch.int64)
    for bits in (5, 10):
        v = compress(keys, rids, bits, 32)
        k, r = decompress(v, keys & ((1 << bits) - 1), bits, 32)
        assert torch.equal(k, keys) and torch.equal(r, rids)


@pytest.mark.parametrize("dev", devices())
def test_ops_pipeline_and_join(dev):
    from hpcjoin import ops
    from hpcjoin.utils import join_count_reference, join_pairs_reference
    R = ops.generate(40_000, "UNIQUE", seed=3, device=dev)
    S = ops.generate(60_000, "ZIPF", seed=4, domain=40_000, device=dev)
    exp = join_count_reference(R[:, 0], S[:, 0])
    assert exp == 60_000
    assert ops.join_count(R, S) == exp
    rv, rb = ops.radix_partition(R, 6)
    sv, sb = ops.radix_partition(S, 6)
    rv2, rb2 = ops.local_partition(rv, rb, 32, 4)
    sv2, sb2 = ops.local_partition(sv, sb, 32, 4)
    assert ops.build_probe_count(rv2, sv2, rb2, sb2, 36, 32) == exp
    assert ops.npj_count(R, S) == exp
    pairs = ops.join(R[:5000].contiguous(), S[:5000].contiguous()).cpu()
    ref = join_pairs_reference(R[:5000], S[:5000])
    got = pairs[torch.argsort(pairs[:, 0] * (1 << 32) + pairs[:, 1])]
    assert torch.equal(got, ref)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("theta,domain", [(0.99, 20), (1.1, 100), (1.5, 100)])
def test_zipf_frequencies(dev, theta, domain):
    """Zipf draws (theta on both sides of 1) against the exact law: the two
    hottest keys are exact in Gray et al.'s inverse, the rest within ~1.5%."""
    from hpcjoin import ops
    n = 400_000
    S = ops.generate(n, "ZIPF", seed=9, domain=domain, zipf_theta=theta, device=dev).cpu()
    freq = torch.sort(torch.unique(S[:, 0], return_counts=True)[1].double() / n, descending=True).values
    law = torch.arange(1, domain + 1, dtype=torch.float64) ** -theta
    law /= law.sum()
    assert freq.numel() <= domain
    assert abs(freq[0] - law[0]) < 0.004 and abs(freq[1] - law[1]) < 0.004
    assert (freq - law[:freq.numel()]).abs().max() < 0.015


def test_config_roundtrip(C, monkeypatch):
    from hpcjoin.utils import config_from_dict, config_to_dict
    cfg = config_from_dict({"network_bits": 7, "assignment": "round_robin", "materialize": True, "format": "wide"})
    d = config_to_dict(cfg)
    assert d["network_bits"] == 7 and d["assignment"] == "ROUND_ROBIN" and d["materialize"] and d["format"] == "WIDE"
    monkeypatch.setenv("HPCJOIN_CHUNKS", "3")
    assert config_from_dict({}).chunks == 3


def test_workload_presets(C):
    from hpcjoin.models import workloads as W
    assert W.get("node_1b").expected_matches() == 1_000_000_000
    assert W.get("zipf_1b_16b").expected_matches() == 16_000_000_000
    assert W.get("tpch_sf1000").expected_matches() == 6_000_000_000
    assert W.get("gpu_128m", 0.001).inner_size == 128_000


def test_radix_join_model_host(C):
    from hpcjoin.models import RadixHashJoin, workloads as W
    eng = RadixHashJoin(W.get("cpu_1m", 0.2), location="host")
    run = eng.run()
    assert run.correct and run.matches == 200_000
    b = eng.benchmark(steps=2, warmup=0)
    assert b["correct"]


def test_plan_is_deterministic(C):
    cfg = C.JoinConfig()
    p = C.make_plan(cfg, 8, 1_000_000_000, 1_000_000_000, 999_999_999, 999_999_999)
    assert (p.network_bits, p.local_bits, p.key_shift) == (9, 9, 32)
    p16 = C.make_plan(cfg, 8, 1_000_000_000, 16_000_000_000, 999_999_999, 16_000_000_000 - 1)
    assert p16.key_shift == 34  # 16B rids need 34 bits
    ko = C.make_plan(cfg, 1, 1000, 1000, (1 << 62), 1000)  # keys too wide for a CompressedTuple
    assert ko.key_only and not ko.wide and ko.key_shift == 0  # counting: 8-byte key-only words
    cfg.materialize = True
    wide = C.make_plan(cfg, 1, 1000, 1000, (1 << 62), 1000)
    assert wide.wide and wide.key_shift == 64  # materializing: the 16-byte Tuple format
    cfg.format = C.TupleFormat.WIDE
    with pytest.raises(RuntimeError):
        C.make_plan(cfg, 1, 1000, 1000, (1 << 64) - 1, 1000)  # the wide format reserves key 2^64-1


def test_measurement_files(C, tmp_path):
    from hpcjoin.utils import parse_perf_dir
    d = str(tmp_path / "exp")
    C.measurements.init(0, 1, "experiment", d)
    ctx = C.ExecContext("host", -1, C.LocalCommunicator())
    R = C.Relation(50_000, 50_000, "host", 0)
    S = C.Relation(50_000, 50_000, "host", 0)
    R.generate(C.GenSpec(seed=1), 0)
    S.generate(C.GenSpec(seed=2), 0)
    C.HashJoin(R, S, ctx, C.JoinConfig()).run()
    C.measurements.store_all()
    ranks = parse_perf_dir(d)
    perf, info = ranks[0]["perf"], ranks[0]["info"]
    for k in ("JTOTAL", "JHIST", "JMPI", "JPROC", "SWINALLOC", "HILOCAL", "HIGLOBAL", "LPELEMENTS", "BPPROBEELEM"):
        assert k in perf, k
    assert perf["RTUPLES"] == 50_000 and info["NUMNODES"] == 1
    snap = C.measurements.snapshot()
    assert snap["JTOTAL"] > 0
    assert C.result_counter() == 50_000


def test_reference_api_surface(C):
    """Reference entry points kept source-compatible (host path)."""
    R = C.Relation(1000, 1000, "host", 0)
    R.fill_unique_values(0, 0)
    t = R.to_tensor()
    assert torch.equal(torch.sort(t[:, 0]).values, torch.arange(1000))
    S = C.Relation(3000, 3000, "host", 0)
    S.fill_modulo_values(0, 0, 1000)
    ctx = C.ExecContext("host", -1, C.LocalCommunicator())
    j = C.HashJoin(R, S, ctx, C.JoinConfig())
    j.join()
    assert C.result_counter() == 3000


def test_arena_growth_and_generation(C):
    """Workspace arena rules (memory/Arena.h): growth -- a fallback allocation
    or a chunk added mid-join -- keeps generation() (peers' IPC mappings of
    the same join stay open, core/ExecContext::ipcImport); only frees bump
    it; reset() keeps the fallback allocations as chunks, so a repeated
    allocation sequence allocates nothing; ensure() with nothing handed out
    re-lays the chunks out as one chunk of the request instead of adding the
    request on top; trim gives the memory back."""
    MiB = 1 << 20
    ctx = C.ExecContext("host", -1, C.LocalCommunicator())
    g0 = ctx.workspace_generation()
    ctx.ensure_workspace(4 * MiB)
    assert ctx.workspace_capacity() == 4 * MiB and ctx.workspace_generation() == g0
    ctx.workspace_scratch(1 * MiB)
    ctx.workspace_scratch(8 * MiB)  # does not fit: a fallback allocation
    ctx.ensure_workspace(10 * MiB)  # in use: adds the 6 MiB shortfall, not 10
    assert ctx.workspace_capacity() == 10 * MiB and ctx.workspace_generation() == g0
    ctx.reset_scratch()  # the fallback becomes a chunk: nothing freed
    assert ctx.workspace_generation() == g0 and ctx.workspace_capacity() == 18 * MiB
    ctx.workspace_scratch(1 * MiB)
    ctx.workspace_scratch(8 * MiB)  # the same sequence fits the chunks again: no allocation
    assert ctx.workspace_capacity() == 18 * MiB and ctx.workspace_generation() == g0
    ctx.reset_scratch()
    assert ctx.trim_workspace(0) == 18 * MiB and ctx.workspace_capacity() == 0
    assert ctx.workspace_generation() == g0 + 1
    ctx.ensure_workspace(4 * MiB)
    assert ctx.workspace_generation() == g0 + 1
    ctx.ensure_workspace(8 * MiB)  # nothing handed out: one chunk of 8 MiB, not 4 + 8
    assert ctx.workspace_capacity() == 8 * MiB and ctx.workspace_generation() == g0 + 2
