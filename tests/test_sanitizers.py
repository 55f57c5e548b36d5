"""Host runtime under AddressSanitizer+UBSan and ThreadSanitizer (SURVEY §5:
the reference has no race detection).  GPU sanitizers are unavailable on the
MI355X pool, so the sanitized binary drives the host path: in-process ranks
(threads), chunked exchange, wide + materialized joins, key hashing, late
materialization and fault propagation (csrc/apps/host_selftest.cpp)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "distributed-radxi-hash-join-on-gpus_amd")


@pytest.mark.parametrize("kind", ["address", "thread"])
def test_host_runtime_sanitized(kind):
    sys.path.insert(0, PKG)
    try:
        import _build
    finally:
        sys.path.remove(PKG)
    exe = _build.build_sanitized(kind)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=0")
    p = subprocess.run([str(exe), "--ranks", "4", "--size", "60000"], env=env, capture_output=True, text=True,
                       timeout=600)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "ALL OK" in out
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "runtime error" not in out  # UBSan
