from __future__ import annotations

from dataclasses import dataclass

import torch

from .._native import require_native


@dataclass
class NoPartitionJoin:
    """Single-GPU no-partitioning hash join: one open-addressing table in HBM
    (reference: operators/gpu/kernels_optimized.cu:1250-1377 build_kernel /
    probe_kernel, small_data_optimized.cu:1731-2087 simple_hash_join*).  Kept
    as the baseline the radix join is measured against."""

    def count(self, inner: torch.Tensor, outer: torch.Tensor) -> int:
        return require_native().ops.npj_count(inner.contiguous(), outer.contiguous())
