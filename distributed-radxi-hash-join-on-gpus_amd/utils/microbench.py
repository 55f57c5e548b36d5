"""Per-phase micro-benchmarks (analog of the reference's partition-throughput
and build/probe-only drivers, /root/reference/operators/gpu/
small_data_optimized.cu:254-399 `shared_memory_PT` and :1731-2087
`simple_hash_join_SD_PT`, plus `UVA_benchmark1/2` for link bandwidth).

Each benchmark reports device time per call (median, hipEvents) and the
effective bandwidth of the bytes the phase must move at minimum, next to the
HBM copy ceiling measured in the same process.
"""
from __future__ import annotations

import statistics

import torch

from .._native import require_native


def _time(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b))
    return statistics.median(out)


def copy_ceiling(nbytes=4 << 30, iters=5):
    C = require_native()
    src = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
    dst = torch.empty_like(src)
    ms = C.ops.bench_copy_ms(src, dst, iters)
    rms = C.ops.bench_read_ms(src, iters)
    return {"copy_ms": ms, "copy_TBps": 2 * nbytes / ms / 1e9, "read_ms": rms, "read_TBps": nbytes / rms / 1e9}


def gen(n, seed=1, dist="UNIQUE", domain=0):
    C = require_native()
    spec = C.GenSpec(distribution=getattr(C.KeyDistribution, dist), seed=seed, domain=domain)
    return C.ops.generate(n, 0, n, spec, "cuda")


def partition_phase(n=1 << 28, bits=10, key_shift=32, iters=5):
    """Network pass (histogram + cursors + LDS scatter) on n 16-byte tuples."""
    C = require_native()
    t = gen(n)
    ms = _time(lambda: C.ops.net_partition(t, bits, key_shift), iters)
    return {"n": n, "bits": bits, "ms": ms, "tuples_per_s": n / ms / 1e6 * 1e3,
            "min_bytes_GB": n * (16 + 16 + 8) / 1e9}


def local_phase(n=1 << 28, b1=10, b2=9, iters=5):
    C = require_native()
    t = gen(n)
    v, b = C.ops.net_partition(t, b1, 32)
    ms = _time(lambda: C.ops.local_partition(v, b, 32, b2), iters)
    return {"n": n, "bits": b2, "ms": ms, "min_bytes_GB": n * 24 / 1e9}


def build_probe_phase(n=1 << 28, b1=10, b2=9, iters=5):
    C = require_native()
    R, S = gen(n, 1), gen(n, 2)
    rv, rb = C.ops.net_partition(R, b1, 32)
    sv, sb = C.ops.net_partition(S, b1, 32)
    rv2, rpb = C.ops.local_partition(rv, rb, 32, b2)
    sv2, spb = C.ops.local_partition(sv, sb, 32, b2)
    ms = _time(lambda: C.ops.build_probe(rv2, sv2, rpb, spb, 32 + b2, 32), iters)
    return {"n": n, "ms": ms, "min_bytes_GB": 2 * n * 8 / 1e9}


def npj_phase(n=1 << 26, iters=3):
    C = require_native()
    R, S = gen(n, 1), gen(n, 2)
    ms = _time(lambda: C.ops.npj_count(R, S), iters)
    return {"n": n, "ms": ms, "tuples_per_s": 2 * n / ms * 1e3}


GEOMETRIES = {0: "256x16", 1: "512x16", 2: "1024x8", 3: "1024x16", 4: "256x16+digarray", 5: "256x8",
              6: "claim256x16", 7: "claim512x16", 8: "claim1024x16", 9: "claim1024x8", 10: "frag-claim1024x16"}


def scatter_ablation(n=1 << 28, bits_list=(4, 8, 10), iters=5, geometries=(0,)):
    """Scatter kernel alone: real / coalesced write-out / no write-out, per
    workgroup geometry (threads x tuples-per-thread)."""
    C = require_native()
    t = gen(n)
    out = []
    for geo in geometries:
        for b in bits_list:
            row = {"geometry": GEOMETRIES[geo], "bits": b}
            try:
                for mode, name in ((0, "scatter_ms"), (1, "coalesced_ms"), (2, "no_write_ms"))[: (2 if 6 <= geo < 10 else 3)]:
                    row[name] = round(C.ops.bench_scatter_ms(t, b, mode, iters, 2048, geo), 4)
                row["scatter_TBps"] = round(n * (20 if geo == 10 else 24) / row["scatter_ms"] / 1e9, 3)
            except RuntimeError as e:  # e.g. LDS budget exceeded for this geometry
                row["error"] = str(e).split("(")[0]
            out.append(row)
    return out


def host_link(bytes_: int = 1 << 30, device: int = 0, iters: int = 5) -> dict:
    """Host-link ceilings: DMA H2D / D2H and in-place kernel reads of pinned
    host memory (the engine's path for relations kept in pinned memory)."""
    return dict(require_native().ops.bench_host_link(bytes_, device, iters))


def wire_phase(n=1 << 28, w=48, rid_bits=27, iters=5):
    """Wire codec (exchange bit-packing): pack and unpack of n CompressedTuples
    into w-bit wire values; HBM streaming, 8 + w/8 bytes per tuple each."""
    C = require_native()
    g = torch.Generator(device="cuda").manual_seed(1)
    rid = torch.randint(0, 1 << rid_bits, (n,), device="cuda", dtype=torch.int64, generator=g)
    frag = torch.randint(0, 1 << (w - rid_bits), (n,), device="cuda", dtype=torch.int64, generator=g)
    raw = rid | (frag << 32)
    r = C.ops.bench_wire(raw, w, rid_bits, 32, iters)
    moved = n * 8 + r["wire_bytes"]
    return {"n": n, "w": w, "pack_ms": r["pack_ms"], "unpack_ms": r["unpack_ms"],
            "pack_TBps": moved / r["pack_ms"] / 1e9, "unpack_TBps": moved / r["unpack_ms"] / 1e9,
            "wire_ratio": r["wire_bytes"] / (n * 8)}
