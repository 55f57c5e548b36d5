"""Distributed join paths.

* in-process ranks (threads sharing one process; host buffers here, device
  buffers on the GPU box) exercise the full N-rank exchange logic;
* a real multi-process run over torch.distributed (gloo) drives the
  ProcessGroupCommunicator on the host path.
"""
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

from conftest import ROOT, devices


def run_ranks(C, n_ranks, loc, G_R, G_S, cfg_fn=None, outer_dist="UNIQUE", theta=0.75, outputs=None, peaks=None,
              inner=None, outer=None):
    group = C.InProcessGroup(n_ranks)
    inner = inner or C.GenSpec(seed=1234)
    outer = outer or C.GenSpec(distribution=getattr(C.KeyDistribution, outer_dist), seed=4321,
                               domain=0 if outer_dist == "UNIQUE" else G_R, zipf_theta=theta)
    results, errors = [None] * n_ranks, []

    def rank_main(r):
        try:
            comm = group.communicator(r)
            ctx = C.ExecContext(loc, 0 if loc == "device" else -1, comm)
            R = C.Relation(C.Relation.local_size_for(G_R, r, n_ranks), G_R, loc, 0)
            S = C.Relation(C.Relation.local_size_for(G_S, r, n_ranks), G_S, loc, 0)
            R.generate(inner, C.Relation.local_offset_for(G_R, r, n_ranks))
            S.generate(outer, C.Relation.local_offset_for(G_S, r, n_ranks))
            cfg = C.JoinConfig()
            if cfg_fn:
                cfg_fn(cfg)
            j = C.HashJoin(R, S, ctx, cfg)
            res = j.run()
            res2 = j.run()  # repeatable
            assert res2["global_matches"] == res["global_matches"]
            results[r] = (res, j.plan)
            if outputs is not None:
                outputs[r] = j.output()
            if peaks is not None:
                peaks[r] = ctx.workspace_peak()
        except Exception as e:  # surface in the main thread
            errors.append((r, repr(e)))

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(n_ranks)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=600)
    assert not errors, errors
    return results, C.Relation.expected_matches(inner, G_R, outer, G_S)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [2, 3, 4, 8])
def test_in_process_ranks(C, dev, n_ranks):
    loc = "device" if dev == "cuda" else "host"
    results, exp = run_ranks(C, n_ranks, loc, 200_003, 300_007, outer_dist="UNIFORM")
    assert all(r[0]["global_matches"] == exp for r in results)
    assert sum(r[0]["local_matches"] for r in results) == exp
    # every tuple ends up on exactly one owner
    assert sum(r[0]["inner_received"] for r in results) == 200_003
    assert sum(r[0]["outer_received"] for r in results) == 300_007


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("policy", ["ROUND_ROBIN", "LPT"])
def test_in_process_chunked_exchange(C, dev, chunks, policy):
    loc = "device" if dev == "cuda" else "host"

    def cfg_fn(cfg):
        cfg.bitmap_join = False  # the tuple exchange is under test
        cfg.chunks = chunks
        cfg.assignment = getattr(C.AssignmentPolicy, policy)
        cfg.max_partition_blocks = 16  # several blocks per chunk even at this size

    results, exp = run_ranks(C, 4, loc, 500_000, 500_000, cfg_fn)
    assert all(r[0]["global_matches"] == exp for r in results)


@pytest.mark.gpu
@pytest.mark.parametrize("n_ranks,chunks,fmt", [(2, 1, "COMPRESSED"), (4, 3, "COMPRESSED"), (3, 2, "WIDE")])
def test_in_process_sampled_local_pass(C, cuda, n_ranks, chunks, fmt):
    """The sampled local pass on multi-rank windows (segments per chunk and
    source).  The sampled network pass (tasks/SampledShuffle) needs the wire
    codec, which wide tuples do not have: those stay on the exact exchange."""

    def cfg_fn(cfg):
        cfg.bitmap_join = False
        cfg.local_histogram = C.HistogramMode.SAMPLED
        cfg.network_histogram = C.HistogramMode.SAMPLED
        cfg.chunks = chunks
        cfg.format = getattr(C.TupleFormat, fmt)

    results, exp = run_ranks(C, n_ranks, "device", 3_000_017, 4_000_037, cfg_fn, outer_dist="ZIPF", theta=0.8)
    for res, plan in results:
        assert res["global_matches"] == exp
        sampled = fmt != "WIDE"
        assert res["sampled_local"] and res["sampled_network"] == sampled and plan.sampled_network == sampled
        assert res["local_fallbacks"] == 0 and res["network_fallbacks"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n_ranks,chunks,opts", [(2, 1, ""), (3, 3, "mat"), (4, 2, "zipf"), (8, 1, ""),
                                                  (4, 2, "hot"), (3, 2, "sparse"), (2, 1, "raw"),
                                                  (3, 2, "rawmat"), (4, 2, "rawsparse"), (4, 2, "rawhot")])
def test_sampled_shuffle(C, cuda, n_ranks, chunks, opts):
    """N > 1 sampled network pass (tasks/SampledShuffle): no exact pre-read of
    either relation; slices sized from a 1-in-S tile sample, exact fills
    all-gathered per chunk, filled runs packed onto the wire -- or, with the
    codec off ("raw": what the cost model picks on fast links), gathered and
    received straight into the window with no unpack pass.  Counts equal the
    oracle and the exact exchange; materialized pairs are the same set."""
    import torch
    G_R, G_S = 1_500_007, 2_500_009
    inner = outer = None
    raw = opts.startswith("raw")
    opts = opts[3:] if raw else opts
    if opts == "hot":
        G_R, G_S = 200_000, 2_000_000
        outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=79, domain=5, zipf_theta=0.99)
    if opts == "sparse":  # the general path: key-only words, key fragment on the wire
        inner, outer = C.GenSpec(seed=1234), C.GenSpec(seed=99)
        inner.sparse64 = outer.sparse64 = True
    got = {}
    for mode in ("SAMPLED", "EXACT"):
        pairs = [None] * n_ranks

        def cfg_fn(c, mode=mode):
            c.network_histogram = getattr(C.HistogramMode, mode)
            c.bitmap_join = False
            c.chunks = chunks
            c.materialize = opts == "mat"
            c.wire_codec = C.WireCodecMode.OFF if raw else C.WireCodecMode.ON
            if opts == "hot":
                c.key_hashing = C.KeyHashing.OFF

        results, exp = run_ranks(C, n_ranks, "device", G_R, G_S, cfg_fn, outer_dist="ZIPF" if opts == "zipf" else "UNIFORM",
                                 theta=0.9, outputs=pairs if opts == "mat" else None, inner=inner, outer=outer)
        for res, plan in results:
            assert plan.sampled_network == (mode == "SAMPLED")
            assert (list(plan.wire_bits) == [0, 0]) == raw, plan
            assert res["sampled_network"] == (mode == "SAMPLED") and res["network_fallbacks"] == 0, res
            if exp is not None:
                assert res["global_matches"] == exp
            if opts == "hot":
                assert res["split_partitions"] >= 1
        got[mode] = results[0][0]["global_matches"]
        if opts != "hot":  # (a split partition's inner side is replicated to its helpers)
            assert sum(r[0]["inner_received"] for r in results) == G_R
        assert sum(r[0]["outer_received"] for r in results) == G_S
        if opts == "mat":
            p = torch.cat([x.cpu() for x in pairs])
            got[mode + "pairs"] = p[torch.argsort(p[:, 1] * (1 << 32) + p[:, 0])]
    assert got["SAMPLED"] == got["EXACT"]
    if opts == "mat":
        assert torch.equal(got["SAMPLEDpairs"], got["EXACTpairs"])


@pytest.mark.gpu
def test_sampled_shuffle_overflow_falls_back(C, cuda):
    """Rank 0's tuples are laid out against the sample (every 4096-tuple tile
    holds one network digit, so the sampled tiles miss most digits); rank 1's
    are shuffled.  Rank 0's slices overflow; the flag rides in the
    fills all-gather, so BOTH ranks abandon the sampled pass at the same point,
    re-run exactly (one network fallback each) and stay exact afterwards."""
    import torch
    n_ranks, n = 2, 1 << 22
    group = C.InProcessGroup(n_ranks)
    out, errs = [None] * n_ranks, []

    def work(r):
        try:
            i = torch.arange(n, device="cuda")
            g = i + r * n
            keys = g * 512 + (i // 4096) % 512  # unique over ranks; digit = tile index mod 512
            if r == 1:
                keys = keys[torch.randperm(n, device="cuda")]
            R = torch.stack([keys, g], 1).contiguous()
            S = torch.stack([keys.flip(0), g], 1).contiguous()
            ctx = C.ExecContext("device", 0, group.communicator(r))
            cfg = C.JoinConfig()
            cfg.network_histogram = C.HistogramMode.SAMPLED
            cfg.bitmap_join = False
            cfg.key_hashing = C.KeyHashing.OFF
            cfg.network_bits = 9
            cfg.wire_codec = C.WireCodecMode.ON
            cfg.max_partition_blocks = 16  # 64 tiles per workgroup, a few of them sampled
            j = C.HashJoin(C.Relation.from_tensor(R, n * n_ranks), C.Relation.from_tensor(S, n * n_ranks), ctx, cfg)
            assert j.plan.sampled_network, j.plan
            first, second = j.run(), j.run()
            out[r] = (first, second)
        except Exception as e:
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(n_ranks)]
    [t.start() for t in ts]
    [t.join(timeout=600) for t in ts]
    assert not errs, errs
    for first, second in out:
        assert first["network_fallbacks"] == 1 and not first["sampled_network"]
        assert first["global_matches"] == n * n_ranks
        assert second["network_fallbacks"] == 0 and not second["sampled_network"]
        assert second["global_matches"] == n * n_ranks


def _balance(C, n_ranks, loc, G_R, G_S, assignment, split, outer, inner=None, network_bits=0, chunks=1):
    """max / mean of the tuples each rank receives (the work the AssignmentMap spreads)."""
    def cfg_fn(cfg):
        cfg.assignment = getattr(C.AssignmentPolicy, assignment)
        cfg.skew_split = split
        cfg.bitmap_join = False
        cfg.key_hashing = C.KeyHashing.OFF  # hot keys stay in their network partition
        cfg.chunks = chunks
        if network_bits:
            cfg.network_bits = network_bits

    results, exp = run_ranks(C, n_ranks, loc, G_R, G_S, cfg_fn, inner=inner, outer=outer)
    if exp is not None:
        assert all(r[0]["global_matches"] == exp for r in results)
    loads = [r[0]["inner_received"] + r[0]["outer_received"] for r in results]
    return max(loads) / (sum(loads) / len(loads)), sum(r[0]["local_matches"] for r in results)


@pytest.mark.parametrize("dev", devices())
def test_in_process_skew_lpt_balances(C, dev):
    """Zipf(0.9) foreign keys over 16 network partitions on 4 ranks: LPT on the
    global histograms beats the reference's round-robin p % N
    (histograms/AssignmentMap.cpp:41-43) by at least 5 points of max / mean
    load (measured 1.055 vs 1.153) and stays within 10 % of the mean."""
    loc = "device" if dev == "cuda" else "host"
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=4321, domain=200_000, zipf_theta=0.9)
    rr, m_rr = _balance(C, 4, loc, 200_000, 800_000, "ROUND_ROBIN", False, outer, network_bits=4)
    lpt, m_lpt = _balance(C, 4, loc, 200_000, 800_000, "LPT", False, outer, network_bits=4)
    assert m_rr == m_lpt
    assert lpt <= 1.10 and rr >= lpt + 0.05, (rr, lpt)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [4, 8])
def test_skew_split_balances_hot_keys(C, dev, n_ranks):
    """Zipf(0.99) over 5 keys (five partitions hold 43/22/15/11/9 % of the
    outer side): round-robin and plain LPT leave one rank with 1.7-3.4x the
    mean load; LPT + hot-partition split (helper counts that divide the
    (source, chunk) pieces, partitions above half a fair share divided) keeps
    the most loaded rank within 15 % of the mean, with the same count."""
    loc = "device" if dev == "cuda" else "host"
    hot = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=77, domain=5, zipf_theta=0.99)
    inner = C.GenSpec(seed=1234)
    rr, m0 = _balance(C, n_ranks, loc, 20_000, 400_000, "ROUND_ROBIN", False, hot, inner=inner)
    lpt, m1 = _balance(C, n_ranks, loc, 20_000, 400_000, "LPT", False, hot, inner=inner)
    both, m2 = _balance(C, n_ranks, loc, 20_000, 400_000, "LPT", True, hot, inner=inner)
    assert m0 == m1 == m2 == 400_000  # inner keys are unique: every outer tuple meets one
    assert both <= 1.15 and rr >= 1.5 * both and lpt >= 1.4 * both, (rr, lpt, both)


@pytest.mark.parametrize("dev", devices())
def test_in_process_wide_materialize(C, dev):
    loc = "device" if dev == "cuda" else "host"

    def cfg_fn(cfg):
        cfg.format = C.TupleFormat.WIDE
        cfg.materialize = True

    results, exp = run_ranks(C, 2, loc, 100_000, 100_000, cfg_fn)
    assert sum(r[0]["output_pairs"] for r in results) == exp


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,chunks", [(2, 1), (3, 2), (8, 1)])
def test_wire_codec_exchange(C, dev, n_ranks, chunks):
    """Bit-packed exchange (frame-of-reference rids + key fragment): exact
    counts, fewer bytes on the links, and every materialized (rid, rid) pair
    still joins equal keys -- so rids and key fragments decode exactly."""
    import torch
    loc = "device" if dev == "cuda" else "host"
    G_R, G_S = 150_001, 250_003

    def cfg_fn(cfg, mode):
        cfg.wire_codec = mode
        cfg.chunks = chunks
        cfg.materialize = True

    outs = [None] * n_ranks
    results, exp = run_ranks(C, n_ranks, loc, G_R, G_S, lambda c: cfg_fn(c, C.WireCodecMode.ON),
                             outer_dist="UNIFORM", outputs=outs)
    plain, _ = run_ranks(C, n_ranks, loc, G_R, G_S, lambda c: cfg_fn(c, C.WireCodecMode.OFF), outer_dist="UNIFORM")
    for (res, plan), (res0, plan0) in zip(results, plain):
        assert res["global_matches"] == exp
        assert 0 < plan.wire_bits[0] < 64 and 0 < plan.wire_bits[1] < 64
        assert plan0.wire_bits == [0, 0]
        pad = 2 * chunks * n_ranks * 64 * 8  # one partial group per segment
        assert res["wire_bytes"] <= res0["wire_bytes"] * max(plan.wire_bits) / 64 + pad
    pairs = torch.cat(outs)
    assert pairs.shape[0] == exp
    R = C.ops.generate(G_R, 0, G_R, C.GenSpec(seed=1234), "cpu")
    S = C.ops.generate(G_S, 0, G_S, C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=4321, domain=G_R), "cpu")
    assert torch.equal(R[pairs[:, 0], 0], S[pairs[:, 1], 0])
    assert pairs[:, 1].unique().numel() == exp  # every outer row matched once (unique inner keys)


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,chunks,mat", [(2, 1, False), (3, 4, True), (8, 2, False)])
def test_split_histogram_pipeline(C, dev, n_ranks, chunks, mat):
    """N > 1 device joins take the assignment from an outer-side estimate and
    run the outer exact histogram + its all-gather behind the inner exchange
    (JoinPlan.split_histogram).  Skewed outer side, LPT: counts and
    materialized pairs equal the fused-histogram path."""
    import torch
    out = {}
    for split in (True, False):
        pairs = [None] * n_ranks

        def cfg_fn(c, split=split):
            c.bitmap_join = False
            c.split_histogram = split
            c.chunks = chunks
            c.materialize = mat
            c.assignment = C.AssignmentPolicy.LPT

        results, exp = run_ranks(C, n_ranks, "device" if dev == "cuda" else "host", 300_007, 700_001, cfg_fn=cfg_fn,
                                 outer_dist="ZIPF", theta=0.9, outputs=pairs if mat else None)
        for res, plan in results:
            assert plan.split_histogram == split
            assert res["global_matches"] == exp
        if mat:
            p = torch.cat([x.cpu() for x in pairs])
            out[split] = p[torch.argsort(p[:, 1] * (1 << 32) + p[:, 0])]
    if mat:
        assert torch.equal(out[True], out[False])


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,chunks,local", [(2, 2, "EXACT"), (3, 4, "SAMPLED"), (4, 3, "AUTO")])
def test_pipelined_outer_chunks(C, dev, n_ranks, chunks, local):
    """N > 1 counting joins local-partition and probe the outer relation one
    exchange chunk at a time (Window.chunkView); results equal the
    whole-window path, exact and sampled local passes, skewed outer side."""
    got = {}
    for pipe in (True, False):
        def cfg_fn(c, pipe=pipe):
            c.bitmap_join = False
            c.pipeline_outer = pipe
            c.chunks = chunks
            c.local_histogram = getattr(C.HistogramMode, local)
        results, exp = run_ranks(C, n_ranks, "device" if dev == "cuda" else "host", 400_009, 900_007, cfg_fn=cfg_fn,
                                 outer_dist="ZIPF", theta=0.8)
        for res, plan in results:
            assert plan.pipeline_outer == pipe
            assert res["global_matches"] == exp and res["local_fallbacks"] == 0
        got[pipe] = [r[0]["local_matches"] for r in results]
    assert got[True] == got[False]


def _free_port():
    """A free rendezvous port BELOW the kernel's ephemeral range (32768-60999
    here): a port the kernel handed out as ephemeral can be handed out again
    as the local port of any outgoing connection (RCCL's bootstrap sockets of
    the ranks starting up) before rank 0 binds it -- an 8-rank run failed
    that way with EADDRINUSE."""
    import random
    rng = random.Random(os.getpid() ^ int(time.time() * 1e6))
    for _ in range(200):
        port = rng.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_gloo_multiprocess_host_join(world):
    """torchrun-style launch: ProcessGroupCommunicator over gloo, host path."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    script = os.path.join(ROOT, "tests", "dist_worker.py")
    procs = [subprocess.Popen([sys.executable, script], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
    assert "OK" in outs[0], outs[0]


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks", [1, 3])
def test_tpch_late_materialization(C, dev, n_ranks):
    """Config 5 path: sparse TPC-H keys, 4 lineitems per order, 32-byte payloads
    fetched from their owner ranks after the join."""
    import torch
    from hpcjoin.models import workloads as W
    from hpcjoin.models.tpch import TpchJoin, verify_sample
    from hpcjoin.parallel import DistInfo
    wl = W.get("tpch_sf1000").scaled(20_000 / 1_500_000_000)
    loc = "device" if dev == "cuda" else "host"
    group = C.InProcessGroup(n_ranks)
    outs, errs = [None] * n_ranks, []

    def work(r):
        try:
            info = DistInfo(rank=r, world=n_ranks, local_rank=0)
            t = TpchJoin(wl, location=loc, info=info, communicator=group.communicator(r))
            res, out = t.run()
            outs[r] = (res, out.cpu())
        except Exception as e:
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(n_ranks)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    allrows = torch.cat([o[1] for o in outs])
    assert allrows.shape[0] == wl.outer_size == wl.expected_matches()
    assert torch.equal(torch.sort(allrows[:, 1]).values, torch.arange(wl.outer_size))  # every lineitem once
    assert verify_sample(allrows, 200)
    # each order appears exactly 4 times
    counts = torch.bincount(allrows[:, 0], minlength=wl.inner_size)
    assert int(counts.min()) == 4 and int(counts.max()) == 4


@pytest.mark.gpu
@pytest.mark.timeout(200)  # above the deadline below, so a hang reports every rank's stack and last output
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_multiprocess_shared_gpu(world):
    """One process per rank over the real RCCL library, as torchrun launches
    bench.py on an 8-GPU node.  The GPU box has one MI355X, so the ranks share
    it (HPCJOIN_SHARE_GPU=1: each rank claims its own RCCL host id and RCCL
    runs its socket transport instead of xGMI); every engine call -- bootstrap,
    histogram all-gather, chunked all-to-allv, result all-reduce -- is the one
    the multi-GPU run makes."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), HPCJOIN_SHARE_GPU="1")
    script = os.path.join(ROOT, "tests", "rccl_worker.py")
    procs = [subprocess.Popen([sys.executable, "-u", script], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    # RCCL's socket transport between processes sharing one GPU: usually
    # 10-40 s for all cases.  On a timeout the ranks' last output says which
    # case they were in.
    outs = [None] * world
    deadline = time.time() + 150
    gout = os.path.join(ROOT, "gpurun_out")
    try:
        for i, p in enumerate(procs):
            while True:  # a line every 10 s under gpurun_out/: the GPU runner sees the test alive
                try:
                    outs[i] = p.communicate(timeout=max(0.1, min(10.0, deadline - time.time())))[0]
                    break
                except subprocess.TimeoutExpired:
                    if time.time() >= deadline:
                        raise
                    if os.path.isdir(gout):
                        with open(os.path.join(gout, "rccl_progress.log"), "a") as f:
                            f.write(f"world {world}: {time.time() - deadline + 150:.0f} s, waiting for rank {i}\n")
    except subprocess.TimeoutExpired:
        import signal
        for p in procs:  # Python stacks of every rank still running (faulthandler in rccl_worker)
            if p.poll() is None:
                p.send_signal(signal.SIGUSR1)
        time.sleep(3)
        for p in procs:
            if p.poll() is None:
                p.kill()
        full = [(outs[i] if outs[i] is not None else p.communicate()[0]) or "" for i, p in enumerate(procs)]
        # The engine's own lines (case progress, Python tracebacks), without
        # the c10d watchdog noise that follows a peer's exit.
        keep = lambda o: "\n".join(ln for ln in o.splitlines()
                                   if not ln.startswith("frame #") and "c10d" not in ln and "TCPStore" not in ln
                                   and "ProcessGroupNCCL" not in ln)[-4000:]
        report = ("rccl_worker timed out after 150 s; output per rank:\n" +
                  "\n".join(f"----- rank {i}:\n{keep(o)}" for i, o in enumerate(full)))
        if os.path.isdir(os.path.join(ROOT, "gpurun_out")):  # kept by the GPU runner even if pytest is killed
            with open(os.path.join(ROOT, "gpurun_out", f"rccl_hang_world{world}.log"), "w") as f:
                f.write(report)
                for i, o in enumerate(full):
                    f.write(f"\n===== rank {i} full output =====\n{o}")
        pytest.fail(report)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]
    assert "OK" in outs[0], outs[0][-4000:]


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,chunks,opts", [(2, 1, ""), (3, 3, "mat"), (4, 2, "wide"), (8, 1, "")])
def test_one_sided_exchange(C, dev, n_ranks, chunks, opts):
    """The MPI_Put analog (JoinConfig.exchange = ONE_SIDED): every rank writes
    its runs straight into the owners' windows at their exact offsets (device:
    the network scatter stores into the peers' windows, no send buffer; host:
    copies), then a barrier; counts (and materialized pairs) equal the RCCL /
    two-sided path, and on the device the workspace peak is smaller."""
    import torch
    got, peak = {}, {}
    for mode in ("ONE_SIDED", "RCCL"):
        pairs = [None] * n_ranks
        peaks = [0] * n_ranks

        def cfg_fn(c, mode=mode):
            c.exchange = getattr(C.ExchangeMode, mode)
            c.bitmap_join = False
            c.chunks = chunks
            c.materialize = opts == "mat"
            if opts == "wide":
                c.format = C.TupleFormat.WIDE
        results, exp = run_ranks(C, n_ranks, "device" if dev == "cuda" else "host", 300_007, 500_009, cfg_fn=cfg_fn,
                                 outer_dist="ZIPF", theta=0.8, outputs=pairs if opts == "mat" else None,
                                 peaks=peaks)
        peak[mode] = sum(peaks)
        for res, plan in results:
            assert plan.one_sided == (mode == "ONE_SIDED")
            assert res["global_matches"] == exp
        got[mode] = [r[0]["local_matches"] for r in results]
        if opts == "mat":
            p = torch.cat([x.cpu() for x in pairs])
            got[mode + "pairs"] = p[torch.argsort(p[:, 1] * (1 << 32) + p[:, 0])]
    assert got["ONE_SIDED"] == got["RCCL"]
    if dev == "cuda":
        assert peak["ONE_SIDED"] < peak["RCCL"], peak
    if opts == "mat":
        assert torch.equal(got["ONE_SIDEDpairs"], got["RCCLpairs"])


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,chunks,opts", [(4, 1, ""), (8, 2, ""), (4, 1, "mat"), (3, 3, "inner-hot"),
                                                  (4, 2, "one-sided")])
def test_hot_partition_split(C, dev, n_ranks, chunks, opts):
    """Cross-rank splitting of a hot network partition (AssignmentMap,
    skew_split): Zipf(0.99) over 5 keys puts ~43 % of the skewed side in one
    partition, more than a rank's fair share.  Its larger side is divided over
    helper ranks by (source, chunk) and its smaller side replicated, so the
    counts (and materialized pairs) equal the unsplit join and the oracle,
    while the most loaded rank receives fewer tuples."""
    import torch
    G_R, G_S = 20_000, 400_000
    hot = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=77, domain=5, zipf_theta=0.99)
    if opts == "inner-hot":  # duplicates on the build side: the inner side is divided, the outer replicated
        inner, outer, G_R, G_S = hot, C.GenSpec(seed=4321), G_S, G_R
    else:
        inner, outer = C.GenSpec(seed=1234), hot
    got, load = {}, {}
    for split in (True, False):
        pairs = [None] * n_ranks

        def cfg_fn(c, split=split):
            c.skew_split = split
            c.bitmap_join = False
            c.chunks = chunks
            c.materialize = opts == "mat"
            c.key_hashing = C.KeyHashing.OFF  # the hot key stays in one network partition
            if opts == "one-sided":  # replicated inner runs: send buffer; divided outer runs: direct scatter
                c.exchange = C.ExchangeMode.ONE_SIDED

        results, exp = run_ranks(C, n_ranks, "device" if dev == "cuda" else "host", G_R, G_S, cfg_fn=cfg_fn,
                                 outputs=pairs if opts == "mat" else None, inner=inner, outer=outer)
        if exp is None:  # inner-hot: every inner key (0..4) meets exactly one unique outer key
            exp = G_R
        for res, plan in results:
            assert res["global_matches"] == exp
            assert (res["split_partitions"] >= 1) == split
            assert plan.skew_split == split
        got[split] = sum(r[0]["local_matches"] for r in results)
        load[split] = max(r[0]["inner_received"] + r[0]["outer_received"] for r in results)
        if opts == "mat":
            p = torch.cat([x.cpu() for x in pairs])
            got[(split, "pairs")] = p[torch.argsort(p[:, 1] * (1 << 32) + p[:, 0])]
            assert p.shape[0] == exp
    assert got[True] == got[False] == exp
    assert load[True] < load[False], load
    if opts == "mat":
        assert torch.equal(got[(True, "pairs")], got[(False, "pairs")])


@pytest.mark.gpu
def test_one_sided_in_process_distinct_devices(C):
    """In-process one-sided windows on two GPUs: the scatter stores through
    raw peer pointers after Window::enableOneSided enabled peer access between
    the ranks' devices (data/Window.cpp).  Needs two visible devices: skipped
    on the one-GPU test box, run wherever two are visible."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    group = C.InProcessGroup(2)
    G_R, G_S = 300_007, 500_009
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=4321, domain=G_R)
    out, errs = [None, None], []

    def rank_main(r):
        try:
            torch.cuda.set_device(r)
            ctx = C.ExecContext("device", r, group.communicator(r))
            R = C.Relation(C.Relation.local_size_for(G_R, r, 2), G_R, "device", r)
            S = C.Relation(C.Relation.local_size_for(G_S, r, 2), G_S, "device", r)
            R.generate(inner, C.Relation.local_offset_for(G_R, r, 2))
            S.generate(outer, C.Relation.local_offset_for(G_S, r, 2))
            cfg = C.JoinConfig()
            cfg.exchange = C.ExchangeMode.ONE_SIDED
            cfg.bitmap_join = False
            j = C.HashJoin(R, S, ctx, cfg)
            out[r] = (j.run(), j.plan)
        except Exception as e:  # surface in the main thread
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(timeout=600) for t in ts]
    assert not errs, errs
    exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
    for res, plan in out:
        assert plan.one_sided and res["global_matches"] == exp


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,chunks,opts", [(2, 1, "one-sided"), (4, 2, "rccl"), (3, 3, "wide"),
                                                  (4, 2, "mat-one-sided"), (4, 2, "hot-split"), (2, 2, "key-only")])
def test_exchange_verification(C, dev, n_ranks, chunks, opts):
    """verify_exchange: every (source, chunk, partition) run is hashed on the
    sender (from its input) and on the receiver (from its window); runs of a
    split hot partition's replicated side count once per receiving helper.
    Clean exchanges verify on every path (two-sided, one-sided, wide tuples,
    materializing, hot-partition split, key-only words)."""
    hot = opts == "hot-split"
    sparse = opts == "key-only"
    inner = C.GenSpec(seed=1234)
    outer = (C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=77, domain=5, zipf_theta=0.99) if hot
             else C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=4321, domain=200_003, zipf_theta=0.8))
    if sparse:
        inner.sparse64 = True
        outer = C.GenSpec(seed=99)
        outer.sparse64 = True

    def cfg_fn(c):
        c.verify_exchange = C.PlanChoice.ON
        c.bitmap_join = False
        c.chunks = chunks
        c.materialize = opts.startswith("mat")
        if "one-sided" in opts:
            c.exchange = C.ExchangeMode.ONE_SIDED
        if opts == "wide":
            c.format = C.TupleFormat.WIDE
        if hot:
            c.key_hashing = C.KeyHashing.OFF
    results, exp = run_ranks(C, n_ranks, "device" if dev == "cuda" else "host", 200_003, 300_007, cfg_fn=cfg_fn,
                             inner=inner, outer=outer)
    for res, plan in results:
        assert res["global_matches"] == exp
        assert res["exchange_checked"] > 0
        if sparse:
            assert plan.key_only


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("mode", ["ONE_SIDED", "RCCL"])
def test_exchange_verification_catches_corruption(C, dev, mode):
    """A word of one rank's window flipped after it arrived (fault injection
    "corrupt_window") makes the join fail on EVERY rank with the exchange
    verification's message -- instead of returning a wrong count."""
    n_ranks = 3
    group = C.InProcessGroup(n_ranks)
    loc = "device" if dev == "cuda" else "host"
    errors = [None] * n_ranks

    def rank_main(r):
        try:
            ctx = C.ExecContext(loc, 0 if loc == "device" else -1, group.communicator(r))
            G = 100_003
            R = C.Relation(C.Relation.local_size_for(G, r, n_ranks), G, loc, 0)
            S = C.Relation(C.Relation.local_size_for(G, r, n_ranks), G, loc, 0)
            R.generate(C.GenSpec(seed=1234), C.Relation.local_offset_for(G, r, n_ranks))
            S.generate(C.GenSpec(seed=4321), C.Relation.local_offset_for(G, r, n_ranks))
            cfg = C.JoinConfig()
            cfg.verify_exchange = C.PlanChoice.ON
            cfg.bitmap_join = False
            cfg.exchange = getattr(C.ExchangeMode, mode)
            j = C.HashJoin(R, S, ctx, cfg)
            assert j.run()["global_matches"] == G  # clean first
            if r == 1:
                C.fault.arm("corrupt_window", r)
            j.run()
        except Exception as e:  # noqa: BLE001
            errors[r] = str(e)

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(n_ranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    assert all(e is not None and "exchange verification" in e and "did not arrive intact" in e for e in errors), errors


@pytest.mark.parametrize("dev", devices())
@pytest.mark.parametrize("n_ranks,passes,opts", [(2, 3, ""), (4, 2, "shuffle"), (3, 4, "one-sided")])
def test_capacity_spill_multirank(C, dev, n_ranks, passes, opts):
    """Capacity spill across ranks: every rank compacts its slice per key-hash
    pass, the pass joins are distributed joins of their own (global pass sizes
    all-reduced), and the summed counts equal the oracle."""
    def cfg_fn(c):
        c.passes = passes
        if opts:
            c.bitmap_join = False
        if opts == "one-sided":
            c.exchange = C.ExchangeMode.ONE_SIDED
    results, exp = run_ranks(C, n_ranks, "device" if dev == "cuda" else "host", 200_003, 300_007, cfg_fn=cfg_fn,
                             outer_dist="ZIPF", theta=0.8)
    for res, plan in results:
        assert res["global_matches"] == exp and res["passes"] == passes


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_ipc_ordering():
    """Round 4's one-sided failures replayed in a fixed order by two processes
    on one GPU (tests/ipc_order_worker.py): two windows in one allocation,
    the exporter's re-layout while the importer holds mappings, a handle
    opened after its allocation was freed.  The engine's export cache,
    generation checks and coordinated release must give exact contents in
    every case; what raw HIP IPC did in the same orders (round 4's calls) is
    written to gpurun_out/ipc_order.json."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
               HPCJOIN_SHARE_GPU="1")
    script = os.path.join(ROOT, "tests", "ipc_order_worker.py")
    procs = [subprocess.Popen([sys.executable, "-u", script], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    try:
        outs = [p.communicate(timeout=90)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    gout = os.path.join(ROOT, "gpurun_out")
    obs = next((ln[len("IPC_ORDER "):] for ln in outs[1].splitlines() if ln.startswith("IPC_ORDER ")), None)
    if os.path.isdir(gout):
        with open(os.path.join(gout, "ipc_order.json"), "w") as f:
            f.write(obs or "null")
            f.write("\n")
            for i, o in enumerate(outs):
                f.write(f"===== rank {i} =====\n{o}\n")
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]
    assert obs is not None, outs[1][-4000:]


def test_wire_codec_cost_model(C):
    """The wire codec packs only when the link time it saves (per tuple that
    leaves a rank: (64 - w) / 8 bytes at min(N - 1, 7) x the per-peer rate)
    exceeds its extra HBM passes (codec_extra_ps_per_tuple, default 3.5 ps):
    63-bit keys (w = 53) stay raw on 8 fast xGMI peers and pack on slow links
    or few peers; dense keys (w = 20) always pack at the modelled rates."""
    pays = C.HashJoin.codec_pays
    assert not pays(53, 8, 64.0)        # 1.375 B / 448 GB/s = 3.1 ps < 3.5: raw
    assert pays(53, 4, 64.0)            # 3 peers: 7.2 ps
    assert pays(53, 8, 10.0)            # slow links (e.g. the socket-transport rehearsal)
    assert pays(20, 8, 64.0)            # 5.5 B saved: 12.3 ps
    assert not pays(40, 8, 200.0)       # fast links, modest saving
    assert pays(40, 8, 200.0, 1.0)      # ... unless the codec is cheaper than modelled
    assert not pays(64, 2, 1.0) and not pays(20, 1, 64.0)


@pytest.mark.gpu
@pytest.mark.parametrize("link,packed", [(10.0, True), (1000.0, False)])
def test_wire_codec_auto_follows_links(C, cuda, link, packed):
    """Auto codec on the general path (53-bit key words) at N = 2 in-process
    ranks: a slow calibrated link packs, a fast one sends raw words into the
    window; both exact on the sampled shuffle."""
    inner, outer = C.GenSpec(seed=1234), C.GenSpec(seed=99)
    inner.sparse64 = outer.sparse64 = True

    def cfg_fn(c):
        c.link_gbps_per_peer = link
        c.bitmap_join = False
        c.network_histogram = C.HistogramMode.SAMPLED

    results, exp = run_ranks(C, 2, "device", 1_000_003, 1_000_003, cfg_fn, inner=inner, outer=outer)
    for res, plan in results:
        assert plan.key_only and plan.sampled_network
        assert (list(plan.wire_bits) == [plan.key_bits - plan.network_bits] * 2) == packed, plan
        assert res["global_matches"] == exp


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
def test_tpch_every_output_row(C, cuda, fused):
    """BASELINE config 5 at SF 1 (1.5M orders x 6M lineitems, 32-byte payload
    rows): EVERY output row [o_rid, l_rid, orders payload, lineitem payload]
    equals a torch gather oracle -- the join pairs from a sort/searchsorted
    of the orders' keys, the payloads gathered from the same payload tensors.
    fused: rows written by the build/probe (N = 1); else pairs + the
    request/response late materialization (the N > 1 path)."""
    import torch
    from hpcjoin.models import workloads as W
    from hpcjoin.models.tpch import TpchJoin
    wl = W.get("tpch_sf1000").scaled(0.001)
    t = TpchJoin(wl, fused=fused)
    res, rows = t.run()
    assert res["global_matches"] == wl.expected_matches() == rows.shape[0]
    O, L = t.orders.to_tensor(), t.lineitem.to_tensor()
    order = torch.argsort(O[:, 0])
    keys = O[order, 0]
    at = torch.searchsorted(keys, L[:, 0]).clamp(max=keys.numel() - 1)
    assert torch.equal(keys[at], L[:, 0])  # every lineitem has its order
    o_rid, l_rid = O[order, 1][at], L[:, 1]
    exp = torch.cat([o_rid[:, None], l_rid[:, None], t.o_rows[o_rid - t.o_off], t.l_rows[l_rid - t.l_off]], 1)
    got = rows.to(exp.device)
    got = got[torch.argsort(got[:, 1])]
    exp = exp[torch.argsort(exp[:, 1])]
    assert got.shape == exp.shape == (wl.expected_matches(), 10)
    assert torch.equal(got, exp)
