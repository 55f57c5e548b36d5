"""Readers for the per-rank measurement files (<rank>.perf: KEY<TAB>value<TAB>unit,
<rank>.info: KEY<TAB>value), the format of /root/reference/performance/Measurements.cpp."""
from __future__ import annotations

import os


def read_kv_file(path: str) -> dict:
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) >= 2:
                try:
                    out[parts[0]] = float(parts[1])
                except ValueError:
                    out[parts[0]] = parts[1]
    return out


def parse_perf_dir(directory: str) -> dict:
    """{rank: {"perf": {...}, "info": {...}}} for every <rank>.perf in directory."""
    ranks = {}
    for name in os.listdir(directory):
        stem, ext = os.path.splitext(name)
        if ext in (".perf", ".info") and stem.isdigit():
            ranks.setdefault(int(stem), {})[ext[1:]] = read_kv_file(os.path.join(directory, name))
    return ranks
