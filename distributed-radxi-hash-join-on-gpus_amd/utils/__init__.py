"""Oracle, runtime configuration and reporting helpers."""
from .oracle import join_count_reference, join_pairs_reference  # noqa: F401
from .config import config_from_dict, config_to_dict  # noqa: F401
from .perf import parse_perf_dir, read_kv_file  # noqa: F401
