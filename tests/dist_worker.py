"""Worker for test_gloo_multiprocess_host_join (one rank per process, gloo)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import hpcjoin  # noqa: E402
from hpcjoin.parallel import init_distributed, make_context  # noqa: E402


def main():
    C = hpcjoin.require_native()
    info = init_distributed(backend="gloo", device=False)
    ctx, comm = make_context(info, "host")
    G_R, G_S = 300_000, 400_000
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(distribution=C.KeyDistribution.ZIPF, seed=77, domain=G_R)
    R = C.Relation(C.Relation.local_size_for(G_R, info.rank, info.world), G_R, "host", 0)
    S = C.Relation(C.Relation.local_size_for(G_S, info.rank, info.world), G_S, "host", 0)
    R.generate(inner, C.Relation.local_offset_for(G_R, info.rank, info.world))
    S.generate(outer, C.Relation.local_offset_for(G_S, info.rank, info.world))
    for chunks in (1, 2):
        cfg = C.JoinConfig()
        cfg.chunks = chunks
        cfg.max_partition_blocks = 8
        res = C.HashJoin(R, S, ctx, cfg).run()
        exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
        assert res["global_matches"] == exp, (res, exp)
    # reference-style distribute() through the process group
    R.distribute(info.rank, info.world, comm)
    res = C.HashJoin(R, S, ctx, C.JoinConfig()).run()
    assert res["global_matches"] == exp
    if info.rank == 0:
        print("OK", res["global_matches"])
    hpcjoin.parallel.shutdown()


if __name__ == "__main__":
    main()
