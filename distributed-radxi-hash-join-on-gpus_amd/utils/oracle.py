"""Independent join oracles in plain torch (no engine code involved)."""
from __future__ import annotations

import torch


def join_count_reference(inner_keys: torch.Tensor, outer_keys: torch.Tensor) -> int:
    """Exact |R join S| = sum over S of the multiplicity of its key in R."""
    r = inner_keys.cpu().to(torch.int64)
    s = outer_keys.cpu().to(torch.int64).contiguous()
    if r.numel() == 0 or s.numel() == 0:
        return 0
    uk, cnt = torch.unique(r, return_counts=True)
    idx = torch.searchsorted(uk, s).clamp(max=uk.numel() - 1)
    hit = uk[idx] == s
    return int(cnt[idx][hit].sum().item())


def join_pairs_reference(inner: torch.Tensor, outer: torch.Tensor) -> torch.Tensor:
    """Sorted (inner rid, outer rid) pairs of an equi-join on column 0 (small inputs)."""
    r, s = inner.cpu(), outer.cpu()
    order = torch.argsort(r[:, 0])
    rk, rr = r[order, 0], r[order, 1]
    lo = torch.searchsorted(rk, s[:, 0].contiguous(), right=False)
    hi = torch.searchsorted(rk, s[:, 0].contiguous(), right=True)
    pairs = []
    for i in torch.nonzero(hi > lo).flatten().tolist():
        for j in range(lo[i], hi[i]):
            pairs.append((int(rr[j]), int(s[i, 1])))
    out = torch.tensor(sorted(pairs), dtype=torch.int64).reshape(-1, 2)
    return out
