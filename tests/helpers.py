"""Shared test helpers: plain PyTorch references for every kernel."""
import torch


def gen(C, n, seed=1234, dist="UNIQUE", domain=0, device="cpu", offset=0, global_size=None, theta=0.75):
    spec = C.GenSpec(distribution=getattr(C.KeyDistribution, dist), seed=seed, domain=domain, zipf_theta=theta)
    return C.ops.generate(n, offset, global_size or n, spec, device)


def unpack(values, bits, key_shift, part_begin):
    """CompressedTuple -> (key, rid) using the partition each value lives in."""
    F = part_begin.numel() - 1
    sizes = (part_begin[1:] - part_begin[:-1]).to(values.device)
    part = torch.repeat_interleave(torch.arange(F, device=values.device), sizes)
    key = ((values >> key_shift) << bits) | part
    rid = values & ((1 << key_shift) - 1)
    return key, rid


def sorted_pairs(keys, rids):
    k = keys * (1 << 32) + rids  # keys and rids < 2^31 in tests
    return torch.sort(k).values


def ref_join_count(r_keys, s_keys):
    """Exact |R join S| with torch: sum over S of multiplicity in R."""
    uk, cnt = torch.unique(r_keys, return_counts=True)
    idx = torch.searchsorted(uk, s_keys)
    idx = idx.clamp(max=uk.numel() - 1)
    hit = uk[idx] == s_keys
    return int(cnt[idx][hit].sum().item())
