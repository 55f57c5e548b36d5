"""Tensor-level entry points of the gfx950 kernels (device tensors) and their
host twins (CPU tensors).  Tuples are int64 tensors of shape [n, 2] holding
(key, rid) — the 16-byte ``hpcjoin::data::Tuple`` layout.

    values, begin = radix_partition(tuples, bits=10)      # network pass
    v2, begin2 = local_partition(values, begin, 32, 9)   # local pass
    n = build_probe_count(rv, sv, rbeg, sbeg, 41, 32)    # LDS build/probe
    join_count(R, S)                                      # whole engine
"""
from __future__ import annotations

import torch

from .._native import require_native
from .tuples import compress, decompress, make_tuples  # noqa: F401


def _C():
    return require_native()


def generate(n: int, distribution: str = "UNIQUE", seed: int = 1234, domain: int = 0, global_offset: int = 0,
             global_size: int | None = None, zipf_theta: float = 0.75, device: str = "cpu") -> torch.Tensor:
    """Slice [global_offset, global_offset + n) of a synthetic relation (see Relation.generate)."""
    C = _C()
    spec = C.GenSpec(distribution=getattr(C.KeyDistribution, distribution.upper()), seed=seed, domain=domain,
                     zipf_theta=zipf_theta)
    return C.ops.generate(n, global_offset, global_size or n, spec, str(device))


def radix_histogram(tuples: torch.Tensor, bits: int) -> torch.Tensor:
    """Counts of ``key & (2^bits - 1)`` (LocalHistogram)."""
    return _C().ops.net_histogram(tuples.contiguous(), bits)


def radix_partition(tuples: torch.Tensor, bits: int, key_shift: int = 32, wide: bool = False,
                    key_bits: int = 64):
    """Network pass: returns (values, part_begin[F+1]); values are packed
    CompressedTuples (int64) unless ``wide`` (then [n, 2] tuples)."""
    return _C().ops.net_partition(tuples.contiguous(), bits, key_shift, wide, 2048, key_bits)


def local_partition(values: torch.Tensor, part_begin: torch.Tensor, shift: int, bits: int, wide: bool = False):
    """Local pass over a partition-major buffer: every input partition is split
    by ``(word >> shift) & (2^bits - 1)``; returns (values, part_begin[P*2^bits+1])."""
    return _C().ops.local_partition(values.contiguous(), part_begin, shift, bits, wide)


def build_probe(R, S, part_r, part_s, frag_shift: int, key_shift: int, wide=False, materialize=False,
                r_chunk=4096, s_chunk=65536, out_capacity=0) -> dict:
    """LDS hash build/probe over matching partitions; returns a dict with
    ``matches`` (and ``pairs`` / ``output_count`` when materializing)."""
    return _C().ops.build_probe(R, S, part_r, part_s, frag_shift, key_shift, wide, materialize, r_chunk, s_chunk,
                                out_capacity)


def build_probe_count(R, S, part_r, part_s, frag_shift: int, key_shift: int) -> int:
    return build_probe(R, S, part_r, part_s, frag_shift, key_shift)["matches"]


def npj_count(R: torch.Tensor, S: torch.Tensor) -> int:
    """No-partitioning join baseline (one global hash table)."""
    return _C().ops.npj_count(R.contiguous(), S.contiguous())


def npj_join(R: torch.Tensor, S: torch.Tensor) -> torch.Tensor:
    """(inner rid, outer rid) pairs of the no-partitioning hash join, [matches, 2] int64."""
    return _C().ops.npj_join(R.contiguous(), S.contiguous())


def _engine(inner: torch.Tensor, outer: torch.Tensor, config=None):
    C = _C()
    on_dev = inner.is_cuda
    dev = (inner.device.index or 0) if on_dev else -1
    ctx = C.ExecContext("device" if on_dev else "host", dev, C.LocalCommunicator())
    R = C.Relation.from_tensor(inner.contiguous(), inner.shape[0])
    S = C.Relation.from_tensor(outer.contiguous(), outer.shape[0])
    return C.HashJoin(R, S, ctx, config or C.JoinConfig())


def join_count(inner: torch.Tensor, outer: torch.Tensor, config=None) -> int:
    """|inner join outer| on key, single process, full engine."""
    return _engine(inner, outer, config).run()["global_matches"]


def join(inner: torch.Tensor, outer: torch.Tensor, config=None) -> torch.Tensor:
    """Materialized join: int64 [m, 2] of (inner rid, outer rid)."""
    C = _C()
    cfg = config or C.JoinConfig()
    cfg.materialize = True
    j = _engine(inner, outer, cfg)
    j.run()
    return j.output()
