from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch

from .._native import require_native


@dataclass
class NoPartitionJoin:
    """Single-GPU no-partitioning hash join (NPJ): one open-addressing table of
    the inner keys in HBM (64-bit CAS inserts, linear probing), probed by every
    outer tuple with random HBM reads -- the baseline the radix join is
    measured against.

    Reference: the dormant ``simple_hash_join*`` drivers and their
    ``build_kernel`` / ``probe_kernel`` (operators/gpu/small_data_optimized.cu:1731-1823,
    kernels_optimized.cu:1250-1377), which build one table and write (rid, rid)
    pairs through a global output cursor.  Here ``count()`` is the count-only
    probe and ``join()`` the materializing one (count pass, exact output
    allocation, then one cursor claim per outer tuple with matches,
    ``csrc/kernels/npj.hip``); both run on host tensors too (C++ reference
    path).  ``timings`` keeps the last call's wall times in ms.
    """

    timings: dict = field(default_factory=dict)

    def _timed(self, name, fn, *args):
        dev = args[0].is_cuda
        if dev:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(*(a.contiguous() for a in args))
        if dev:
            torch.cuda.synchronize()
        self.timings[name] = (time.perf_counter() - t0) * 1e3
        return out

    def count(self, inner: torch.Tensor, outer: torch.Tensor) -> int:
        """Number of (inner, outer) pairs with equal keys."""
        return self._timed("count_ms", require_native().ops.npj_count, inner, outer)

    def join(self, inner: torch.Tensor, outer: torch.Tensor) -> torch.Tensor:
        """Every match as (inner rid, outer rid), [matches, 2] int64, unordered."""
        return self._timed("join_ms", require_native().ops.npj_join, inner, outer)

    def throughput(self, inner: torch.Tensor, outer: torch.Tensor, key: str = "count_ms") -> float:
        """Input tuples per second of the last timed call (G tuples/s)."""
        ms = self.timings.get(key)
        return (inner.shape[0] + outer.shape[0]) / ms / 1e6 if ms else float("nan")
