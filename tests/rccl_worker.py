"""Worker for test_rccl_multiprocess_shared_gpu: one rank per process over the
real RCCL library (torchrun environment, ``HPCJOIN_SHARE_GPU=1`` so several
ranks can share the box's one MI355X).  Runs the engine's device path end to
end -- torch.distributed bootstrap, ncclUniqueId broadcast, RCCL all-gather of
histograms, chunked all-to-allv, all-reduce of the result -- on unique, Zipf
and materialising joins, and checks every count against the oracle.
"""
import faulthandler
import os
import signal
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import hpcjoin  # noqa: E402
from hpcjoin.parallel import init_distributed, make_context  # noqa: E402


def main():
    # SIGUSR1 dumps every thread's Python stack (the test sends it to all
    # ranks when a run times out, so a hang says where each rank was).
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    C = hpcjoin.require_native()
    # A rank that fails makes its peers fail too (within the test's deadline)
    # instead of leaving them in a collective: the engine's waits give up
    # after this long.
    C.fault.set_comm_timeout_ms(90_000)
    info = init_distributed()
    ctx, comm = make_context(info, "device")
    assert comm.name() == "rccl", comm.name()
    G_R, G_S = 3_000_017, 5_000_011
    inner = C.GenSpec(seed=1234)
    cases = [
        ("unique", C.GenSpec(seed=99), G_R, {}),
        ("zipf", C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=77, domain=G_R, zipf_theta=0.75), G_S, {}),
        ("uniform-chunks4", C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=5, domain=G_R), G_S,
         {"chunks": 4}),
        ("materialize", C.GenSpec(seed=99), G_R, {"materialize": True}),
        ("wide", C.GenSpec(seed=99), G_R, {"format": C.TupleFormat.WIDE}),
        ("unique-shuffle", C.GenSpec(seed=99), G_R, {"bitmap_join": False}),
        ("zipf-shuffle-chunks3", C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=78, domain=G_R, zipf_theta=0.9),
         G_S, {"bitmap_join": False, "chunks": 3}),
        # one-sided puts into IPC-mapped peer windows (processes on one GPU here)
        ("one-sided", C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=6, domain=G_R), G_S,
         {"bitmap_join": False, "chunks": 2, "exchange": C.ExchangeMode.ONE_SIDED}),
        ("one-sided-materialize", C.GenSpec(seed=99), G_R,
         {"exchange": C.ExchangeMode.ONE_SIDED, "materialize": True}),
        # ~43 % of the outer side on one key: that partition is joined by
        # several ranks (outer divided, inner replicated)
        ("hot-split", C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=79, domain=5, zipf_theta=0.99), G_S,
         {"bitmap_join": False, "chunks": 2, "key_hashing": C.KeyHashing.OFF}),
        ("hot-split-one-sided", C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=79, domain=5, zipf_theta=0.99),
         G_S, {"bitmap_join": False, "key_hashing": C.KeyHashing.OFF, "exchange": C.ExchangeMode.ONE_SIDED}),
        # sampled network pass (no exact pre-read): fills all-gathered per
        # chunk, packed runs on the wire (tasks/SampledShuffle)
        ("sampled-chunks3", C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=7, domain=G_R), G_S,
         {"bitmap_join": False, "chunks": 3, "network_histogram": C.HistogramMode.SAMPLED}),
        ("sampled-materialize", C.GenSpec(seed=99), G_R,
         {"materialize": True, "chunks": 2, "network_histogram": C.HistogramMode.SAMPLED}),
        ("sampled-hot-split", C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=79, domain=5, zipf_theta=0.99),
         G_S, {"bitmap_join": False, "chunks": 2, "key_hashing": C.KeyHashing.OFF,
               "network_histogram": C.HistogramMode.SAMPLED}),
        # raw words (codec off: the cost model's choice on fast links), gathered
        # runs received straight into the windows -- no unpack pass
        ("sampled-raw-chunks2", C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=9, domain=G_R), G_S,
         {"bitmap_join": False, "chunks": 2, "network_histogram": C.HistogramMode.SAMPLED,
          "wire_codec": C.WireCodecMode.OFF}),
    ]
    R = C.Relation(C.Relation.local_size_for(G_R, info.rank, info.world), G_R, "device", info.local_rank)
    R.generate(inner, C.Relation.local_offset_for(G_R, info.rank, info.world))
    # General path: unique random 63-bit keys on both sides -> key-only words,
    # wire codec carrying only the key bits above the network digit.
    sparse_in = C.GenSpec(seed=1234)
    sparse_in.sparse64 = True
    sparse_out = C.GenSpec(seed=99)
    sparse_out.sparse64 = True
    Rs = C.Relation(C.Relation.local_size_for(G_R, info.rank, info.world), G_R, "device", info.local_rank)
    Rs.generate(sparse_in, C.Relation.local_offset_for(G_R, info.rank, info.world))
    Ss = C.Relation(C.Relation.local_size_for(G_R, info.rank, info.world), G_R, "device", info.local_rank)
    Ss.generate(sparse_out, C.Relation.local_offset_for(G_R, info.rank, info.world))
    cfg = C.JoinConfig()
    exp = C.Relation.expected_matches(sparse_in, G_R, sparse_out, G_R)
    for mode, codec in (("EXACT", "ON"), ("SAMPLED", "ON"), ("SAMPLED", "OFF")):
        cfg.network_histogram = getattr(C.HistogramMode, mode)
        cfg.wire_codec = getattr(C.WireCodecMode, codec)
        mode = mode if codec == "ON" else mode + "-raw"
        j = C.HashJoin(Rs, Ss, ctx, cfg)
        want = [j.plan.key_bits - j.plan.network_bits] * 2 if codec == "ON" else [0, 0]
        assert j.plan.key_only and list(j.plan.wire_bits) == want, j.plan
        assert j.plan.sampled_network == mode.startswith("SAMPLED"), j.plan
        for _ in range(2):
            res = j.run()
            assert res["global_matches"] == exp, ("sparse-key-only", mode, res["global_matches"], exp)
            assert res["sampled_network"] == mode.startswith("SAMPLED") and res["network_fallbacks"] == 0, res
        if info.rank == 0:
            print(f"sparse-key-only {mode}: {res['global_matches']} == {exp}, plan {j.plan}", flush=True)
        del j
    del Rs, Ss
    for name, spec, G, opts in cases:
        print(f"[rank {info.rank}] {name}", flush=True)  # progress (shown only when a run times out)
        S = C.Relation(C.Relation.local_size_for(G, info.rank, info.world), G, "device", info.local_rank)
        S.generate(spec, C.Relation.local_offset_for(G, info.rank, info.world))
        cfg = C.JoinConfig()
        for k, v in opts.items():
            setattr(cfg, k, v)
        j = C.HashJoin(R, S, ctx, cfg)
        exp = C.Relation.expected_matches(inner, G_R, spec, G)
        # counting joins of these unique inner keys take the replicated bitmaps
        # (one ncclAllReduce) unless the shuffle is forced
        want_bitmap = not opts.get("materialize") and "format" not in opts and opts.get("bitmap_join", True)
        assert j.plan.bitmap_join == want_bitmap and j.plan.bitmap_replicated == want_bitmap, (name, j.plan)
        assert j.plan.one_sided == ("exchange" in opts), (name, j.plan)
        for _ in range(2):
            res = j.run()
            assert res["global_matches"] == exp, (name, res["global_matches"], exp)
            if "hot-split" in name:  # 43 % of one side: above half a rank's fair share at any world
                assert res["split_partitions"] >= 1, (name, res["split_partitions"])
            if name.startswith("sampled"):
                assert res["sampled_network"] and res["network_fallbacks"] == 0, (name, res)
        if opts.get("materialize"):
            pairs = j.output()
            assert pairs.shape[0] == res["local_matches"], (pairs.shape, res["local_matches"])
        if info.rank == 0:
            print(f"{name}: {res['global_matches']} == {exp}, plan {j.plan}", flush=True)
        del j, S
    # One-sided windows across a workspace growth: the large join grows every
    # rank's arena (a new chunk and generation), so the peers' cached IPC
    # mappings must be re-opened (core/ExecContext::ipcImport); the small join
    # before and after it stays exact.
    cfg1 = C.JoinConfig()
    cfg1.bitmap_join = False
    cfg1.exchange = C.ExchangeMode.ONE_SIDED
    spec = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=8, domain=G_R)
    caps = []
    for G in (G_S, 40 * G_S, G_S):
        S = C.Relation(C.Relation.local_size_for(G, info.rank, info.world), G, "device", info.local_rank)
        S.generate(spec, C.Relation.local_offset_for(G, info.rank, info.world))
        j = C.HashJoin(R, S, ctx, cfg1)
        assert j.plan.one_sided, j.plan
        res = j.run()
        assert res["global_matches"] == C.Relation.expected_matches(inner, G_R, spec, G), ("one-sided-grow", G, res)
        caps.append(ctx.workspace_capacity())
        del j, S
    assert caps[1] > caps[0], ("workspace did not grow", caps)
    if info.rank == 0:
        print(f"one-sided across a workspace growth: exact, workspace {caps}", flush=True)
    # One-sided windows allocated by fallback INSIDE the join: workspace
    # trimmed to nothing and no reservation, so every window is a fallback
    # hipMalloc and the peers import a rank's second window while its first
    # one is in use.  Growth keeps the arena generation, so that first mapping
    # stays open (it used to be closed at the second import).
    step = lambda m: print(f"[rank {info.rank}] fallback case: {m}", flush=True)
    step("trim")
    ctx.trim_workspace(0)
    step("barrier")
    comm.barrier()
    cfg2 = C.JoinConfig()
    cfg2.bitmap_join = False
    cfg2.exchange = C.ExchangeMode.ONE_SIDED
    cfg2.reserve_workspace = False
    G = 4 * G_S
    S = C.Relation(C.Relation.local_size_for(G, info.rank, info.world), G, "device", info.local_rank)
    S.generate(spec, C.Relation.local_offset_for(G, info.rank, info.world))
    step("construct")
    j = C.HashJoin(R, S, ctx, cfg2)
    assert j.plan.one_sided and ctx.workspace_capacity() == 0, (j.plan, ctx.workspace_capacity())
    exp = C.Relation.expected_matches(inner, G_R, spec, G)
    for it in range(2):
        step(f"run {it}")
        res = j.run()
        mine = [it, res["local_matches"], res["inner_received"], res["outer_received"], res["global_matches"]]
        allv = comm.all_gather(mine) if hasattr(comm, "all_gather") else [mine]
        if res["global_matches"] != exp:
            print(f"one-sided-fallback mismatch rank {info.rank}: per-rank [run, local, inner_recv, outer_recv, "
                  f"global] = {allv}, expected {exp}", flush=True)
        assert res["global_matches"] == exp, ("one-sided-fallback", it, allv, exp)
    del j, S
    if info.rank == 0:
        print("one-sided with in-join fallback windows: exact", flush=True)
    # TPC-H-like join + late materialization of 32-byte payload rows across
    # ranks (BASELINE config 5 at SF 0.5): pairs from the build/probe, rows
    # fetched from their owner ranks by the request/response all-to-allv.
    from hpcjoin.models import workloads as W
    from hpcjoin.models.tpch import TpchJoin, verify_sample
    wl = W.get("tpch_sf1000").scaled(0.0005)
    t = TpchJoin(wl, info=info, communicator=comm)
    for _ in range(2):
        res, rows = t.run()
        assert res["global_matches"] == wl.expected_matches(), ("tpch", res["global_matches"])
        assert rows.shape[0] == res["local_matches"] and verify_sample(rows, 64), "tpch rows"
        ph = res.get("materialize_phases")
        assert ph is not None and ph["request_bytes"] > 0 and ph["response_bytes"] > 0, ph
    if info.rank == 0:
        print(f"tpch: {res['global_matches']} pairs, rows verified, phases {ph}", flush=True)
    del t, rows
    torch.cuda.synchronize()
    comm.barrier()
    if info.rank == 0:
        print("OK", flush=True)
    del R, ctx, comm
    hpcjoin.parallel.shutdown()


if __name__ == "__main__":
    main()
