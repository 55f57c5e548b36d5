"""Runtime JoinConfig <-> dict / environment (the reference configures
everything at compile time: core/Configuration.h + CMake -D macros)."""
from __future__ import annotations

import os

from .._native import require_native

_FIELDS = ["network_bits", "local_bits", "two_level", "key_shift", "materialize", "output_capacity", "build_target",
           "r_chunk", "s_chunk", "chunks", "checks", "max_partition_blocks", "sample_stride", "local_sample_stride", "round_lp", "local_item_tiles", "local_geometry",
           "split_local", "direct_count", "split_histogram", "pipeline_outer", "bitmap_join", "skew_split",
           "reserve_workspace", "passes", "workspace_budget", "link_gbps_per_peer", "codec_extra_ps_per_tuple",
           # kernel-shape variants (sweeps / A-B tests; JoinConfig.variants in C++)
           "net_ipt", "net_threads", "bm_threads", "bm_flat", "reduce_chunks", "key_count", "rows_lds", "mat_variant"]
_FLOATS = ("link_gbps_per_peer", "codec_extra_ps_per_tuple")
_BOOLS = ("two_level", "materialize", "checks", "split_local", "direct_count", "split_histogram", "pipeline_outer",
          "bitmap_join", "skew_split", "reserve_workspace")


def config_to_dict(cfg) -> dict:
    d = {f: getattr(cfg, f) for f in _FIELDS}
    d["assignment"] = str(cfg.assignment).split(".")[-1]
    d["format"] = str(cfg.format).split(".")[-1]
    d["key_hashing"] = str(cfg.key_hashing).split(".")[-1]
    d["network_histogram"] = str(cfg.network_histogram).split(".")[-1]
    d["local_histogram"] = str(cfg.local_histogram).split(".")[-1]
    d["wire_codec"] = str(cfg.wire_codec).split(".")[-1]
    d["replicate_bitmap"] = str(cfg.replicate_bitmap).split(".")[-1]
    d["exchange"] = str(cfg.exchange).split(".")[-1]
    return d


def config_from_dict(d: dict | None = None, env_prefix: str = "HPCJOIN_"):
    """JoinConfig from a dict, overridden by HPCJOIN_<FIELD> environment variables."""
    C = require_native()
    cfg = C.JoinConfig()
    merged = dict(d or {})
    for f in _FIELDS + ["assignment", "format", "key_hashing", "network_histogram", "local_histogram", "wire_codec",
                        "replicate_bitmap", "exchange", "verify_exchange"]:
        v = os.environ.get(env_prefix + f.upper())
        if v is not None:
            merged[f] = v
    for k, v in merged.items():
        if k == "assignment":
            cfg.assignment = getattr(C.AssignmentPolicy, str(v).upper())
        elif k == "format":
            cfg.format = getattr(C.TupleFormat, str(v).upper())
        elif k == "key_hashing":
            cfg.key_hashing = getattr(C.KeyHashing, str(v).upper())
        elif k in ("network_histogram", "local_histogram"):
            setattr(cfg, k, getattr(C.HistogramMode, str(v).upper()))
        elif k in _BOOLS:
            setattr(cfg, k, v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes"))
        elif k == "wire_codec":
            cfg.wire_codec = getattr(C.WireCodecMode, str(v).upper())
        elif k in ("replicate_bitmap", "verify_exchange"):
            setattr(cfg, k, getattr(C.PlanChoice, str(v).upper()))
        elif k == "exchange":
            cfg.exchange = getattr(C.ExchangeMode, str(v).upper())
        elif k in _FLOATS:
            setattr(cfg, k, float(v))
        elif k in _FIELDS:
            setattr(cfg, k, int(v))
        else:
            raise KeyError(f"unknown JoinConfig field {k}")
    return cfg
