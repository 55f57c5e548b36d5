"""Failure detection and fault injection (absent in the reference,
where MPI errors are fatal and most CUDA errors are unchecked).

A rank that fails mid-join (here: an injected fault) aborts its communicator;
peers blocked in a collective must raise promptly instead of hanging, and a
lone rank waiting on a barrier must time out.
"""
import os
import subprocess
import sys
import threading
import time

import pytest

from conftest import ROOT, devices


def _join_ranks(C, n, loc, fault_phase, fault_rank, G=1 << 16):
    group = C.InProcessGroup(n)
    errs = [None] * n

    def work(r):
        try:
            C.fault.arm(fault_phase, fault_rank)
            comm = group.communicator(r)
            ctx = C.ExecContext(loc, 0 if loc == "device" else -1, comm)
            R = C.Relation(C.Relation.local_size_for(G, r, n), G, loc, 0)
            S = C.Relation(C.Relation.local_size_for(G, r, n), G, loc, 0)
            R.generate(C.GenSpec(seed=1), C.Relation.local_offset_for(G, r, n))
            S.generate(C.GenSpec(seed=2), C.Relation.local_offset_for(G, r, n))
            C.HashJoin(R, S, ctx, C.JoinConfig()).run()
        except Exception as e:  # noqa: BLE001
            errs[r] = e
        finally:
            C.fault.arm("", -1)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    t0 = time.time()
    [t.start() for t in ts]
    [t.join(timeout=60) for t in ts]
    assert not any(t.is_alive() for t in ts), "a rank hung after its peer failed"
    return errs, group, time.time() - t0


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("phase", ["histogram", "network", "local", "build_probe"])
def test_injected_fault_fails_all_ranks(C, dev, phase):
    C.fault.set_comm_timeout_ms(30_000)
    try:
        errs, group, dt = _join_ranks(C, 3, "device" if dev == "cuda" else "host", phase, 1)
    finally:
        C.fault.set_comm_timeout_ms(0)
    assert isinstance(errs[1], C.fault.InjectedFault) and phase in str(errs[1])
    assert group.aborted()
    # Peers either fail through the abort, or (build_probe: no collective left
    # before the final all-reduce) fail in that all-reduce.  Nobody succeeds
    # with a partial result and nobody waits for the 30 s watchdog.
    for r in (0, 2):
        assert errs[r] is not None and "abort" in str(errs[r]), errs[r]
    assert dt < 25


def test_barrier_timeout(C):
    C.fault.set_comm_timeout_ms(300)
    try:
        group = C.InProcessGroup(2)
        comm = group.communicator(0)
        t0 = time.time()
        with pytest.raises(RuntimeError, match="timed out"):
            comm.barrier()  # rank 1 never arrives
        assert 0.25 < time.time() - t0 < 5
        assert group.aborted()
        with pytest.raises(RuntimeError, match="abort"):
            group.communicator(1).barrier()
    finally:
        C.fault.set_comm_timeout_ms(0)


def test_fault_injection_from_env():
    """HPCJOIN_FAULT=<phase>[:<rank>] arms a fault without code changes (CLI / bench)."""
    code = ("import hpcjoin; from hpcjoin import ops; R = ops.generate(4096); S = ops.generate(4096, seed=3); "
            "ops.join_count(R, S)")
    env = dict(os.environ, HPCJOIN_FAULT="network:0", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "injected fault at phase 'network'" in p.stderr
    env["HPCJOIN_FAULT"] = "network:5"  # other rank: no fault
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr


def test_stalled_rank_ends_every_rank():
    """A rank that stops making progress at `network` (HPCJOIN_STALL) must not
    leave the job hanging until an outer kill: with HPCJOIN_COMM_TIMEOUT_S set
    (bench.py sets 120 s for N > 1) every rank exits non-zero within the
    timeout, and each message names its rank, phase, wait site and last
    completed collective."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world, timeout_s = 3, 4
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", HPCJOIN_STALL="network:1",
               HPCJOIN_COMM_TIMEOUT_S=str(timeout_s))
    script = os.path.join(ROOT, "tests", "stall_worker.py")
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, "-u", script], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=120))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    wall = time.time() - t0
    for r, (p, (out, err)) in enumerate(zip(procs, outs)):
        assert p.returncode != 0, (r, out, err)
        line = next((l for l in err.splitlines() if l.startswith("RANK_FAILED")), "")
        assert f"rank={r}" in line and "WATCHDOG" in line and f"[rank {r}]" in line, (r, err[-2000:])
        assert "phase 'network'" in line and "last completed collective" in line, line
        after = float(line.split("after=")[1].split("s ")[0])
        assert after < 3 * timeout_s + 5, line  # bounded by the timeout, not by an outer kill
    assert "injected stall at phase 'network'" in [e for _, e in outs][1]
    assert wall < 100
