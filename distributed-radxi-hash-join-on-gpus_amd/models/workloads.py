"""Workload presets: the BASELINE.json configurations plus scaled variants.

Key domain (BASELINE.md caveat): "uniform int64 keys" are drawn from a domain
that fits the 8-byte CompressedTuple (keys < 2^(64 - keyShift + networkBits));
the ``wide`` format carries full 64-bit keys end to end.
"""
from __future__ import annotations

from dataclasses import dataclass

from .._native import require_native


@dataclass(frozen=True)
class Workload:
    name: str
    inner_size: int
    outer_size: int
    outer_distribution: str = "UNIQUE"   # UNIQUE | UNIFORM | ZIPF | MODULO | DENSE
    zipf_theta: float = 0.75
    inner_seed: int = 1234
    outer_seed: int = 4321
    wide: bool = False
    materialize: bool = False
    payload_bytes: int = 0               # late-materialized payload per side (TPC-H-like)
    tpch_sparse: bool = False            # TPC-H O_ORDERKEY layout on both sides
    gpus: int = 1
    description: str = ""

    def specs(self):
        C = require_native()
        inner = C.GenSpec(C.KeyDistribution.UNIQUE, self.inner_seed, 0, 0, 0.75, self.tpch_sparse)
        dist = getattr(C.KeyDistribution, self.outer_distribution)
        outer = C.GenSpec(dist, self.outer_seed,
                          0 if self.outer_distribution in ("UNIQUE", "DENSE") else self.inner_size, 0,
                          self.zipf_theta, self.tpch_sparse)
        return inner, outer

    def expected_matches(self) -> int | None:
        C = require_native()
        i, o = self.specs()
        return C.Relation.expected_matches(i, self.inner_size, o, self.outer_size)

    def join_config(self):
        """Default JoinConfig for this workload, HPCJOIN_<FIELD> environment
        overrides applied (utils.config.config_from_dict)."""
        from ..utils.config import config_from_dict
        C = require_native()
        cfg = config_from_dict()
        if self.wide:
            cfg.format = C.TupleFormat.WIDE
        cfg.materialize = self.materialize
        return cfg

    def relations(self, info, location: str):
        """This rank's slices of both relations, generated in place."""
        C = require_native()
        i, o = self.specs()
        dev = info.local_rank if location == "device" else 0
        R = C.Relation(C.Relation.local_size_for(self.inner_size, info.rank, info.world), self.inner_size, location, dev)
        S = C.Relation(C.Relation.local_size_for(self.outer_size, info.rank, info.world), self.outer_size, location, dev)
        R.generate(i, C.Relation.local_offset_for(self.inner_size, info.rank, info.world))
        S.generate(o, C.Relation.local_offset_for(self.outer_size, info.rank, info.world))
        return R, S

    def scaled(self, factor: float) -> "Workload":
        return Workload(**{**self.__dict__, "name": f"{self.name}@{factor:g}",
                           "inner_size": max(1024, int(self.inner_size * factor)),
                           "outer_size": max(1024, int(self.outer_size * factor))})


B = 1_000_000_000
PRESETS = {
    # BASELINE.json configs
    "cpu_1m": Workload("cpu_1m", 1_000_000, 1_000_000, description="config 1: single-thread host reference path"),
    "gpu_128m": Workload("gpu_128m", 128_000_000, 128_000_000, description="config 2: 1 x MI355X"),
    "node_1b": Workload("node_1b", B, B, gpus=8, description="config 3: 1B x 1B, 8 x MI355X, RCCL all-to-allv"),
    "zipf_1b_16b": Workload("zipf_1b_16b", B, 16 * B, "ZIPF", 0.75, gpus=8,
                            description="config 4: 1B x 16B Zipf(0.75) foreign keys, LPT assignment"),
    "tpch_sf1000": Workload("tpch_sf1000", 1_500_000_000, 6_000_000_000, "MODULO", materialize=True,
                            payload_bytes=32, tpch_sparse=True, gpus=8,
                            description="config 5: orders x lineitem (4 lineitems per order), 32-byte payloads "
                                        "gathered by rid after the join (late materialization)"),
    # the reference's default workload: 20M x 20M per rank (main.cpp:70-71)
    "reference_default": Workload("reference_default", 20_000_000, 20_000_000,
                                  description="reference main.cpp default per rank"),
}


def get(name: str, scale: float = 1.0) -> Workload:
    w = PRESETS[name]
    return w if scale == 1.0 else w.scaled(scale)
