#!/usr/bin/env python3
"""Skewed-join configurations (BASELINE config 4: Zipf theta = 0.75, the
skew-aware AssignmentMap path) with an exact oracle.

Configs (one JSON line each, rank 0):
  zipf_both_sparse  zipf_both through the sparse 63-bit key bijection: the
                general path (key-only words, quotient table) with duplicate
                inner keys
  zipf_both     inner AND outer Zipf(theta) over the same dense domain: the
                inner side has duplicates, so the bitmap plan cannot apply and
                the two-level plan (+ LPT / hot-partition split at N > 1) runs
  uniform_two   inner unique, outer uniform foreign keys, bitmap plan off: the
                two-level reference time the Zipf run is compared with
  uniform_sparse  uniform_two through the sparse 63-bit key bijection: the
                general path at this size (1B x 4B: outer slots past 2^31)
  zipf_outer    inner unique, outer Zipf(theta) (default plan)
Assignment variants at N > 1: --assign lpt,round_robin and --split on,off.

Oracle: sum_k cntR(k) * cntS(k) from per-key counts on the device
(Relation.count_keys, all-reduced over ranks), independent of the join.

    python tools/bench_skew.py [--gpus N] [--inner 1e9] [--outer 4e9] [--configs zipf_both,uniform_two]
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def spawn_if_needed():
    """Without a launcher and with --gpus N > 1: N rank processes of the
    running script (torchrun env); exits with their status."""
    if "WORLD_SIZE" in os.environ:
        return
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args()[0].gpus
    if n <= 1:
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(sys.argv[0]), *sys.argv[1:]],
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r)), start_new_session=True) for r in range(n)]
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code and not rc:
                rc = code if code > 0 else 1
                for q in procs:
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.05)
    sys.exit(rc)


if __name__ == "__main__":
    spawn_if_needed()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import hpcjoin  # noqa: E402
from hpcjoin.parallel import init_distributed, make_context  # noqa: E402
from hpcjoin.utils import config_from_dict  # noqa: E402


def oracle(C, info, R, S, domain):
    """Exact count of a join of dense keys in [0, domain) from per-key counts."""
    cr = torch.zeros(domain, dtype=torch.int32, device="cuda")
    cs = torch.zeros(domain, dtype=torch.int32, device="cuda")
    out = R.count_keys(cr, 0) + S.count_keys(cs, 0)
    if info.world > 1:
        dist.all_reduce(cr)
        dist.all_reduce(cs)
    # int32 counts fit (a key repeats < 2^31 times); the products need int64.
    total = 0
    step = 1 << 26
    for b in range(0, domain, step):
        total += int((cr[b:b + step].to(torch.int64) * cs[b:b + step].to(torch.int64)).sum().item())
    del cr, cs
    torch.cuda.empty_cache()
    return total if out == 0 else None


def run_config(C, info, ctx, comm, name, G_R, G_S, theta, cfg, steps, warmup, domain=0):
    domain = domain or G_R
    if name in ("zipf_both", "zipf_both_sparse"):
        inner = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=1234, domain=domain, zipf_theta=theta)
        outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=4321, domain=domain, zipf_theta=theta)
    elif name == "zipf_outer":
        inner = C.GenSpec(distribution=C.KeyDistribution.UNIQUE, seed=1234)
        outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=4321, domain=domain, zipf_theta=theta)
    else:  # uniform_two, uniform_sparse
        inner = C.GenSpec(distribution=C.KeyDistribution.UNIQUE, seed=1234)
        outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=4321, domain=domain)
        inner.sparse64 = outer.sparse64 = name == "uniform_sparse"
    lr, ls = (C.Relation.local_size_for(G, info.rank, info.world) for G in (G_R, G_S))

    def relations():
        R = C.Relation(lr, G_R, "device", info.local_rank)
        S = C.Relation(ls, G_S, "device", info.local_rank)
        R.generate(inner, C.Relation.local_offset_for(G_R, info.rank, info.world))
        S.generate(outer, C.Relation.local_offset_for(G_S, info.rank, info.world))
        return R, S

    R, S = relations()
    expected = C.Relation.expected_matches(inner, G_R, outer, G_S)
    oracle_source = "closed form"
    # The per-key oracle allocates and frees two domain-sized count arrays;
    # run it after the timed joins unless the relations are replaced below,
    # so the first join is not measured behind the oracle's frees.
    deferred_oracle = expected is None and name != "zipf_both_sparse"
    if expected is None and not deferred_oracle:
        expected = oracle(C, info, R, S, domain)
        oracle_source = "per-key device counts"
    if name == "zipf_both_sparse":
        # The same Zipf relations through the sparse 63-bit key bijection
        # (general path: key-only words, duplicate inner keys); the count is
        # that of the dense relations the oracle just read.
        del R, S
        torch.cuda.empty_cache()
        inner.sparse64 = outer.sparse64 = True
        R, S = relations()
        oracle_source += " of the dense pre-image"

    def barrier():
        if info.world > 1:
            comm.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    join = C.HashJoin(R, S, ctx, cfg)
    barrier()
    setup_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    first = join.run()
    barrier()
    first_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(max(0, warmup - 1)):
        join.run()
    ctx.reset_scratch()
    barrier()
    res = []
    t0 = time.perf_counter()
    for _ in range(steps):
        res.append(join.run())
    barrier()
    mine_ms = (time.perf_counter() - t0) * 1e3 / steps
    if deferred_oracle:
        expected = oracle(C, info, R, S, domain)
        oracle_source = "per-key device counts (after the timed joins)"
    per = [res[-1]["inner_received"], res[-1]["outer_received"], int(mine_ms * 1e3),
           int(sum(r["join_ms"] for r in res) / len(res) * 1e3), int(first_ms * 1e3), int(setup_ms * 1e3),
           int(join.plan_ms * 1e3)]
    K = len(per)
    allv = comm.all_gather(per) if info.world > 1 else per
    recv = [allv[i] + allv[i + 1] for i in range(0, len(allv), K)]
    ms = max(allv[2::K]) / 1e3
    mean = sum(recv) / len(recv)
    out = {
        "config": name, "n_gpus": info.world, "inner": G_R, "outer": G_S, "theta": theta,
        "ms_per_step": round(ms, 3), "value": round((G_R + G_S) / ms / 1e6, 3), "unit": "billion tuples/s",
        "first_join_ms": max(allv[4::K]) / 1e3, "setup_ms": max(allv[5::K]) / 1e3, "plan_ms": max(allv[6::K]) / 1e3,
        "first_over_steady": round(max(allv[4::K]) / 1e3 / ms, 3) if ms else None,
        "matches": res[-1]["global_matches"], "expected_matches": expected, "oracle": oracle_source,
        "correct": expected is not None and all(r["global_matches"] == expected for r in [first] + res),
        "plan": repr(join.plan), "assignment": str(cfg.assignment).split(".")[-1], "skew_split": cfg.skew_split,
        "split_partitions": res[-1]["split_partitions"],
        "received_per_rank": recv, "max_over_mean_received": round(max(recv) / mean, 4) if mean else None,
        "join_ms_per_rank": [v / 1e3 for v in allv[3::K]],
        "first_reruns": first["reruns"], "first_local_fallbacks": first["local_fallbacks"],
        "local_fallbacks": sum(r["local_fallbacks"] for r in res), "network_fallbacks": sum(r["network_fallbacks"] for r in res),
        "reruns": res[-1]["reruns"],
        "phases_ms": {k: round(res[-1][k], 3) for k in ("dev_network_ms", "dev_local_partition_ms", "dev_build_probe_ms")},
        "first_phases_ms": {k: round(first[k], 3) for k in ("histogram_ms", "network_ms", "local_ms", "join_ms",
                                                             "dev_network_ms", "dev_local_partition_ms",
                                                             "dev_build_probe_ms") if k in first},
        "steady_phases_ms": {k: round(res[-1][k], 3) for k in ("histogram_ms", "network_ms", "local_ms", "join_ms")
                             if k in res[-1]},
    }
    del join, R, S
    ctx.reset_scratch()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--inner", type=float, default=1e9)
    ap.add_argument("--outer", type=float, default=4e9)
    ap.add_argument("--theta", type=float, default=0.75)
    ap.add_argument("--domain", type=float, default=0, help="Zipf / uniform key domain (0 = |R|); a small domain "
                    "puts more than a rank's fair share on one network partition")
    ap.add_argument("--configs", default="zipf_both,uniform_two,zipf_outer")
    ap.add_argument("--assign", default="lpt", help="comma list of lpt,round_robin (N > 1)")
    ap.add_argument("--split", default="on", help="comma list of on,off: hot-partition split (N > 1, LPT)")
    ap.add_argument("--shuffle", action="store_true",
                    help="N > 1: force the hash-partition shuffle (no replicated bitmaps), so the assignment decides "
                         "what every rank receives")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    C = hpcjoin.require_native()
    info = init_distributed()
    ctx, comm = make_context(info, "device")
    G_R, G_S = int(args.inner), int(args.outer)
    for name in args.configs.replace("+", ",").split(","):
        for assign in args.assign.replace("+", ",").split(","):
            for split in args.split.replace("+", ",").split(","):
                if assign != "lpt" and split == "on" and len(args.split.replace("+", ",").split(",")) > 1:
                    continue  # the split only exists under LPT
                cfg = config_from_dict({"assignment": assign.upper(), "skew_split": split == "on", "chunks": 1 if info.world == 1 else 4})
                if name == "uniform_two" or args.shuffle:
                    if name == "uniform_two":
                        cfg.bitmap_join = False
                    cfg.replicate_bitmap = C.PlanChoice.OFF
                out = run_config(C, info, ctx, comm, name, G_R, G_S, args.theta, cfg, args.steps, args.warmup,
                                 int(args.domain))
                out["domain"] = int(args.domain) or G_R
                if info.rank == 0:
                    print(json.dumps(out), flush=True)
    del ctx
    torch.cuda.synchronize()
    if info.world > 1:
        comm.barrier()
    del comm
    if info.world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
