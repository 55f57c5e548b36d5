#!/usr/bin/env python3
"""Headline benchmark: distributed radix hash join throughput on MI355X.

BASELINE metric: billion tuples/s (whole node) for a 1B x 1B join of unique
int64 keys on 1/2/4/8 MI355X (strong scaling: the 1B x 1B total is fixed).
One step = one complete join (histogram -> fused all-gather -> LDS scatter +
RCCL all-to-allv -> local radix pass -> LDS build/probe -> match count), the
reference's JTOTAL span (operators/HashJoin.cpp:51,212).  Data generation is
outside the timed region, as in the reference.  Every step's match count is
checked against the exact oracle (|R| for unique keys).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--inner 1e9] [--outer 1e9]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Host<->device copies of a join are small (plan uploads, cursor and counter
# read-backs): run them as blit kernels on the compute queue, not on the SDMA
# engines.  With SDMA on, about every second process stalled one join (the
# 4th) by 17-45 ms inside the first small copy; with it off 5/5 runs were
# clean (profiles/r1_sdma_outlier.md).  Must be set before HIP initialises.
# Single-process runs only: multi-rank runs keep the runtime default (their
# RCCL rehearsals over the socket transport were measured with SDMA on).
if int(os.environ.get("WORLD_SIZE", "1")) == 1:
    os.environ.setdefault("HSA_ENABLE_SDMA", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import hpcjoin  # noqa: E402
from hpcjoin.parallel import init_distributed, make_context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--inner", type=float, default=1e9)
    ap.add_argument("--outer", type=float, default=1e9)
    ap.add_argument("--dist", default="unique", choices=["unique", "uniform", "zipf", "modulo"])
    ap.add_argument("--theta", type=float, default=0.75)
    ap.add_argument("--chunks", type=int, default=0, help="exchange pipeline slices (0 = auto)")
    ap.add_argument("--input", default="device", choices=["device", "pinned"],
                    help="where the relations live: HBM, or pinned host memory read in place over the host link")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    C = hpcjoin.require_native()
    info = init_distributed()
    assert info.world == args.gpus or args.gpus == 1 and info.world == 1, \
        f"--gpus {args.gpus} but WORLD_SIZE={info.world}"
    on_gpu = torch.cuda.is_available()
    loc = "device" if on_gpu else "host"
    ctx, comm = make_context(info, loc)

    G_R, G_S = int(args.inner), int(args.outer)
    if not on_gpu:  # CPU fallback for plumbing only: keep it small
        G_R, G_S = min(G_R, 1 << 20), min(G_S, 1 << 20)
    inner = C.GenSpec(distribution=C.KeyDistribution.UNIQUE, seed=1234)
    dmap = {"unique": C.KeyDistribution.UNIQUE, "uniform": C.KeyDistribution.UNIFORM,
            "zipf": C.KeyDistribution.ZIPF, "modulo": C.KeyDistribution.MODULO}
    outer = C.GenSpec(distribution=dmap[args.dist], seed=4321, domain=0 if args.dist == "unique" else G_R,
                      zipf_theta=args.theta)
    lr, ls = (C.Relation.local_size_for(G, info.rank, info.world) for G in (G_R, G_S))
    rel_loc = "pinned" if on_gpu and args.input == "pinned" else loc
    R = C.Relation(lr, G_R, rel_loc, info.local_rank)
    S = C.Relation(ls, G_S, rel_loc, info.local_rank)
    R.generate(inner, C.Relation.local_offset_for(G_R, info.rank, info.world))
    S.generate(outer, C.Relation.local_offset_for(G_S, info.rank, info.world))
    expected = C.Relation.expected_matches(inner, G_R, outer, G_S)

    from hpcjoin.utils import config_from_dict  # HPCJOIN_<FIELD> env overrides (sweeps)
    cfg = config_from_dict({})
    if args.chunks > 0:
        cfg.chunks = args.chunks
    elif "HPCJOIN_CHUNKS" not in os.environ:
        cfg.chunks = 1 if info.world == 1 else 4
    join = C.HashJoin(R, S, ctx, cfg)

    def barrier():
        if info.world > 1:
            comm.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    # Grow the engine arena to the first warmup's peak right after it, so the
    # remaining warmups (not the first timed join) are the first to run on the
    # freshly reserved workspace; the first join pays a one-time hipMalloc.
    for i in range(args.warmup):
        join.run()
        if i == 0:
            ctx.reset_scratch()
    ctx.reset_scratch()
    barrier()
    results = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        results.append(join.run())
    barrier()
    elapsed = time.perf_counter() - t0
    # max over ranks
    mine = [int(elapsed * 1e9)]
    elapsed_ns = max(comm.all_gather(mine)) if info.world > 1 else mine[0]
    elapsed = elapsed_ns / 1e9
    ms_per_step = elapsed * 1e3 / args.steps
    value = (G_R + G_S) * args.steps / elapsed / 1e9
    correct = all(r["global_matches"] == expected for r in results) if expected is not None else None
    phases = {k: round(sum(r[k] for r in results) / len(results), 3)
              for k in ("histogram_ms", "network_ms", "local_ms", "dev_histogram_ms", "dev_network_ms",
                        "dev_local_partition_ms", "dev_build_probe_ms")}
    if info.rank == 0:
        line = {
            "metric": "billion tuples/sec (whole node), 1B x 1B uniform int64 keys",
            "value": round(value, 4),
            "unit": "billion tuples/s",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64 keys (8-byte CompressedTuple after the network pass)",
            "data": "synthetic: unique int64 keys 0..G-1 under a keyed Feistel permutation, generated on device",
            "config": {
                "model": f"distributed radix hash join, {args.dist} keys, |R|={G_R}, |S|={G_S}",
                "global_batch": G_R + G_S,
                "seq_len": 1,
                "parallelism": f"hash-partition x{info.world} (RCCL all-to-allv over xGMI)" if info.world > 1
                else "single MI355X",
                "plan": repr(join.plan),
                "chunks": cfg.chunks,
                "input": rel_loc,
            },
            "matches": results[-1]["global_matches"],
            "expected_matches": expected,
            "correct": correct,
            "phases_ms": phases,
            "engine": {"reruns": results[-1]["reruns"], "build_probe_items": results[-1]["build_probe_items"],
                       "network_fallbacks": sum(r["network_fallbacks"] for r in results),
                       "local_fallbacks": sum(r["local_fallbacks"] for r in results),
                       "wire_bytes": results[-1]["wire_bytes"],
                       "local_items": results[-1]["local_items"], "workspace_GB": round(ctx.workspace_capacity() / 1e9, 2),
                       "workspace_peak_GB": round(ctx.workspace_peak() / 1e9, 2),
                       "step_ms": [round(r["join_ms"], 2) for r in results],
                       "step_phases_ms": [[round(r[k], 2) for k in ("histogram_ms", "network_ms", "local_ms",
                                                                      "dev_histogram_ms", "dev_network_ms",
                                                                      "dev_local_partition_ms", "dev_build_probe_ms")]
                                          for r in results],
                       "setup_ms": [round(r["setup_ms"], 2) for r in results],
                       "teardown_ms": [round(r["teardown_ms"], 2) for r in results]},
            "device": torch.cuda.get_device_name(0) if on_gpu else "cpu",
        }
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(line, f, indent=1)
    # Deterministic teardown: engine objects (HIP streams, arenas, the RCCL
    # communicator) go before torch.distributed and before interpreter exit.
    del join, R, S, ctx
    if on_gpu:
        torch.cuda.synchronize()
    if info.world > 1:
        comm.barrier()
    del comm
    if info.world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if correct is False:
        sys.exit(3)


if __name__ == "__main__":
    main()
