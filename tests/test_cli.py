"""Standalone C++ driver (build/bin/hjoin_bench, no Python/torch) and bench.py."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "distributed-radxi-hash-join-on-gpus_amd", "build", "bin", "hjoin_bench")


def _last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_hjoin_bench_host(tmp_path):
    assert os.path.exists(BIN), "run __graft_entry__.build() first"
    r = subprocess.run([BIN, "--host", "--inner", "200000", "--outer", "300000", "--dist", "zipf", "--iters", "2",
                        "--warmup", "0", "--perf-dir", str(tmp_path / "perf")],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stdout + r.stderr
    j = _last_json(r.stdout)
    assert j["correct"] is True and j["matches"] == 300000
    assert "[RESULTS] Tuples:" in r.stdout
    assert (tmp_path / "perf" / "0.perf").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--two-level-only"]])
def test_hjoin_bench_device(extra):
    r = subprocess.run([BIN, "--inner", "16777216", "--outer", "16777216", "--iters", "3", *extra],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert _last_json(r.stdout)["correct"] is True


def test_bench_py_cpu_contract():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    j = _last_json(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in j, k
    assert j["correct"] is True and j["n_gpus"] == 1 and j["steps"] == 2
    assert "value_note" in j  # which plan `value` measures (N > 1: replicated bitmaps, not the shuffle)


def test_bench_py_stalled_rank_exits_with_site(tmp_path):
    """bench.py --gpus 2 (its own spawner, gloo on the CPU) with rank 1 stalled
    at `network`: both ranks end within the watchdog timeout, the job exits
    non-zero, and the failing rank's message names rank, phase and site."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", HPCJOIN_STALL="network:1",
               HPCJOIN_COMM_TIMEOUT_S="5")
    env.pop("WORLD_SIZE", None)
    import time
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert r.returncode != 0, r.stdout + r.stderr
    assert "WATCHDOG" in r.stderr and "phase 'network'" in r.stderr, r.stderr[-3000:]
    assert "bench.py: rank" in r.stderr and "failed after" in r.stderr, r.stderr[-3000:]
    assert time.time() - t0 < 200


def test_bench_py_wall_budget_skips_secondary():
    """A spent wall budget skips the secondary measurements (and says so)
    instead of running past the driver's limit; the headline is printed."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1",
                        "--budget-s", "0"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    j = _last_json(r.stdout)
    assert j["correct"] is True and j["general_path"] is None
    assert "general_path" in j["skipped"] and "wall budget" in j["skipped"]["general_path"]
