"""Tuple / CompressedTuple layouts in plain torch (reference:
/root/reference/data/Tuple.h, data/CompressedTuple.h,
tasks/NetworkPartitioning.cpp:128-129)."""
from __future__ import annotations

import torch


def make_tuples(keys: torch.Tensor, rids: torch.Tensor | None = None) -> torch.Tensor:
    """[n, 2] int64 (key, rid); rids default to 0..n-1."""
    keys = keys.to(torch.int64)
    if rids is None:
        rids = torch.arange(keys.numel(), dtype=torch.int64, device=keys.device)
    return torch.stack([keys, rids.to(torch.int64)], dim=1).contiguous()


def compress(keys: torch.Tensor, rids: torch.Tensor, network_bits: int, key_shift: int = 32) -> torch.Tensor:
    """value = rid | ((key >> network_bits) << key_shift)."""
    return rids.to(torch.int64) | ((keys.to(torch.int64) >> network_bits) << key_shift)


def decompress(values: torch.Tensor, partition: torch.Tensor | int, network_bits: int, key_shift: int = 32):
    """(key, rid) given the network partition each value was routed to."""
    rid = values & ((1 << key_shift) - 1)
    key = ((values >> key_shift) << network_bits) | partition
    return key, rid
