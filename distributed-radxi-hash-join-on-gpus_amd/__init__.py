"""hpcjoin — MI355X-native distributed radix hash join.

The compute path is the native core in ``csrc/`` (hand-written gfx950 HIP
kernels + C++ runtime + RCCL), exposed as ``hpcjoin._C``.  This package adds
the Python surface: launch/bootstrap (``parallel``), join "model" families
(``models``), tensor-level kernel entry points (``ops``) and the oracle,
config and reporting helpers (``utils``).

Import as ``import hpcjoin`` from the repository root (see ``hpcjoin.py``).
"""
from __future__ import annotations

import os as _os

import torch as _torch  # noqa: F401  -- load torch's HIP runtime / RCCL before the extension

from ._native import native, native_available, require_native  # noqa: F401

__version__ = "0.1.0"
PACKAGE_DIR = _os.path.dirname(_os.path.abspath(__file__))

if native_available():
    _C = native()
    JoinConfig = _C.JoinConfig
    JoinPlan = _C.JoinPlan
    GenSpec = _C.GenSpec
    Relation = _C.Relation
    HashJoin = _C.HashJoin
    ExecContext = _C.ExecContext
    KeyDistribution = _C.KeyDistribution
    AssignmentPolicy = _C.AssignmentPolicy
    TupleFormat = _C.TupleFormat
    LocalCommunicator = _C.LocalCommunicator
    RcclCommunicator = _C.RcclCommunicator
    ProcessGroupCommunicator = _C.ProcessGroupCommunicator
    measurements = _C.measurements
