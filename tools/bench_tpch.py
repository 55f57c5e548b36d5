#!/usr/bin/env python3
"""TPC-H-like orders x lineitem join with late materialization of 32-byte
payloads (BASELINE config 5; SF1000 = 1.5B orders x 6B lineitems on 8 GPUs).

One step = join (sparse o_orderkey layout, 4 lineitems per order) + fetching
both payload rows of every result pair from their owner ranks.  Default size
is SF100 per GPU (150M x 600M), which fits one MI355X with room for the
60 GB output.  Prints one JSON line (rank 0).

    python tools/bench_tpch.py [--gpus N] [--sf-per-gpu 100] [--steps 5] [--warmup 1]
    python -m torch.distributed.run --nproc-per-node N ... tools/bench_tpch.py

At N > 1 the JSON also carries the request/response phases of the late
materialization (bucket, request all-to-allv, gather, response all-to-allv,
place; link bytes per rank), the measured link bandwidth, and a link-byte
and link-time prediction for SF1000 on 8 GPUs from the plan's wire format.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    from bench_skew import spawn_if_needed  # torch-free helper: N rank processes without a launcher
    spawn_if_needed()

import torch  # noqa: E402

import hpcjoin  # noqa: E402
from hpcjoin.models import workloads as W  # noqa: E402
from hpcjoin.models.tpch import TpchJoin, verify_sample  # noqa: E402
from hpcjoin.parallel import init_distributed, shutdown  # noqa: E402


def sf1000_prediction(wl, plan, calib, info):
    """Link bytes and time one rank of an 8-GPU SF1000 join would move: the
    shuffle of both relations in this plan's wire format, plus the
    late materialization (per remote pair side: an 8-byte rid out, a 32-byte
    row back), at the calibrated per-rank all-to-all bandwidth."""
    N, O, L = 8, 1_500_000_000, 6_000_000_000
    wire = [b if b else 64 for b in plan.wire_bits]
    shuffle = (N - 1) / N * (O * wire[0] + L * wire[1]) / 8 / N
    pairs = L / N  # 4 lineitems per order: one pair per lineitem, spread over the ranks
    mat = pairs * 2 * (N - 1) / N * (8 + 32)
    gbps = calib["all_to_all_GBps_per_rank"] * 7 / max(info.world - 1, 1) if calib else None
    return {"wire_bits": wire, "shuffle_bytes_per_rank": int(shuffle), "materialize_bytes_per_rank": int(mat),
            "link_GBps_per_rank": round(gbps, 2) if gbps else None,
            "bandwidth_source": ("measured per-peer all-to-all bandwidth x 7 peers" if calib else None),
            "predicted_shuffle_ms": round(shuffle / gbps / 1e6, 1) if gbps else None,
            "predicted_materialize_ms": round(mat / gbps / 1e6, 1) if gbps else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--sf-per-gpu", type=float, default=100.0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--unfused", action="store_true",
                    help="join, then a separate late-materialization pass (the N>1 path) even at N=1")
    args = ap.parse_args()
    hpcjoin.require_native()
    info = init_distributed()
    sf = args.sf_per_gpu * info.world
    if not torch.cuda.is_available():
        sf = min(sf, 0.01)
    wl = W.get("tpch_sf1000").scaled(sf / 1000.0)
    t = TpchJoin(wl, info=info, fused=not args.unfused)
    for _ in range(args.warmup):
        t.run()
    t.ctx.reset_scratch()  # arena grown to the warmup peak before timing
    calib = None
    if info.world > 1 and torch.cuda.is_available():
        import bench as B  # link calibration on the engine communicator (RCCL all-to-allv)
        calib = B.calibrate_links(t.comm, info, True)
    join_ms, mat_ms, tot_ms, ok = [], [], [], True
    phases = []
    out = None
    for _ in range(args.steps):
        out = None  # release the previous output rows before the next step allocates
        t.comm.barrier()
        res, out = t.run()
        join_ms.append(res["join_ms"])
        mat_ms.append(res["materialize_ms"])
        tot_ms.append(res["total_ms"])
        if "materialize_phases" in res:
            phases.append(res["materialize_phases"])
        ok &= res["global_matches"] == wl.expected_matches()
    ok &= verify_sample(out, 256)
    tot = sorted(tot_ms)[len(tot_ms) // 2]
    if info.world > 1:  # slowest rank defines the step
        import torch.distributed as dist
        v = torch.tensor([tot], device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        tot = float(v.item())
    mat = None
    if phases:
        mat = {k: round(sorted(p[k] for p in phases)[len(phases) // 2], 3) for k in phases[0]}
    prediction = sf1000_prediction(wl, t.engine.plan, calib, info)
    if info.rank == 0:
        print(json.dumps({
            "metric": "TPC-H-like join + 32 B payload late materialization",
            "value": (wl.inner_size + wl.outer_size) / tot / 1e6, "unit": "G input tuples/s",
            "n_gpus": info.world, "scale_factor": sf, "orders": wl.inner_size, "lineitem": wl.outer_size,
            "output_rows_local": int(out.shape[0]), "output_bytes_per_row": int(out.shape[1]) * 8,
            "median_total_ms": tot, "median_join_ms": sorted(join_ms)[len(join_ms) // 2],
            "median_materialize_ms": sorted(mat_ms)[len(mat_ms) // 2],
            "matches": int(res["global_matches"]), "correct": bool(ok), "rows_fused": bool(res["rows_fused"]),
            "phases_ms": {k: round(res[k], 3) for k in ("histogram_ms", "network_ms", "local_ms", "dev_histogram_ms",
                                                         "dev_network_ms", "dev_local_partition_ms",
                                                         "dev_build_probe_ms", "setup_ms")},
            "engine": {k: res[k] for k in ("reruns", "build_probe_items", "local_items", "output_overflow",
                                           "sampled_network", "sampled_local", "network_fallbacks",
                                           "local_fallbacks")},
            "step_join_ms": [round(x, 3) for x in join_ms],
            "materialize_phases_ms_rank0": mat,
            "links": calib, "sf1000_8gpu_prediction": prediction,
            "plan": repr(t.engine.plan)}), flush=True)
    del out, t
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    shutdown()
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
