"""Standalone CMake build (the reference's build system is CMake): the
runtime library, both apps, and the CTest host self-test."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "distributed-radxi-hash-join-on-gpus_amd")


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None, reason="cmake/ninja missing")
def test_cmake_build_and_ctest():
    bdir = os.path.join(PKG, "build", "cmake")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    subprocess.run(["cmake", "-S", PKG, "-B", bdir, "-G", "Ninja"], check=True, capture_output=True, timeout=600)
    jobs = str(min(16, os.cpu_count() or 4))
    r = subprocess.run(["cmake", "--build", bdir, "-j", jobs], capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert os.path.exists(os.path.join(bdir, "hjoin_bench"))
    r = subprocess.run(["ctest", "--output-on-failure"], cwd=bdir, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
