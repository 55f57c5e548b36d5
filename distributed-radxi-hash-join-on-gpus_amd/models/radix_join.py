from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch

from .._native import require_native
from ..parallel import DistInfo, init_distributed, make_context
from . import workloads as W


@dataclass
class JoinRun:
    """Result of RadixHashJoin.run(): the native JoinResult plus oracle check."""
    result: dict
    expected: int | None
    wall_ms: float

    @property
    def matches(self) -> int:
        return self.result["global_matches"]

    @property
    def correct(self) -> bool | None:
        return None if self.expected is None else self.matches == self.expected


@dataclass
class RadixHashJoin:
    """The distributed radix hash join engine on one rank.

    >>> eng = RadixHashJoin(W.get("gpu_128m"))      # generates the rank's slices
    >>> run = eng.run()                             # one full join
    >>> run.matches, run.correct
    """
    workload: W.Workload
    config: object = None
    location: str = "auto"
    info: DistInfo = field(default_factory=lambda: None)

    def __post_init__(self):
        C = require_native()
        if self.location == "auto":
            self.location = "device" if torch.cuda.is_available() else "host"
        self.info = self.info or init_distributed(device=self.location == "device")
        self.ctx, self.comm = make_context(self.info, self.location)
        self.config = self.config or self.workload.join_config()
        self.inner, self.outer = self.workload.relations(self.info, self.location)
        self.engine = C.HashJoin(self.inner, self.outer, self.ctx, self.config)

    @property
    def plan(self):
        return self.engine.plan

    def run(self) -> JoinRun:
        t0 = time.perf_counter()
        res = self.engine.run()
        return JoinRun(res, self.workload.expected_matches(), (time.perf_counter() - t0) * 1e3)

    def output(self) -> torch.Tensor:
        """Materialized (inner rid, outer rid) pairs of the last run (config.materialize)."""
        return self.engine.output()

    def benchmark(self, steps: int = 5, warmup: int = 1) -> dict:
        for _ in range(warmup):
            self.run()
        runs = [self.run() for _ in range(steps)]
        ms = sorted(r.result["join_ms"] for r in runs)
        tuples = self.workload.inner_size + self.workload.outer_size
        return {"workload": self.workload.name, "median_ms": ms[len(ms) // 2],
                "gtuples_per_s": tuples / (ms[len(ms) // 2] * 1e6), "correct": all(r.correct is not False for r in runs),
                "plan": repr(self.plan)}
