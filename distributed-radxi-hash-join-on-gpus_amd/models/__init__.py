"""Join "model families" and workload presets.

* :class:`RadixHashJoin` — the distributed two-pass radix hash join engine
  (histogram -> RCCL exchange -> local radix pass -> LDS build/probe).
* :class:`NoPartitionJoin` — the global-hash-table baseline (the reference's
  simple_hash_join* family).
* :mod:`workloads` — the BASELINE.json configurations (CPU 1M plumbing,
  128M single GPU, 1B node-wide, 1B x 16B Zipf skew, TPC-H-like with
  32-byte payloads) and scaled-down variants for tests.
"""
from .radix_join import JoinRun, RadixHashJoin  # noqa: F401
from .npj import NoPartitionJoin  # noqa: F401
from . import workloads  # noqa: F401
from .tpch import TpchJoin  # noqa: F401
