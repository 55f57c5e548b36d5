"""Worker for test_stalled_rank_ends_every_rank (one gloo rank per process).

HPCJOIN_STALL=<phase>:<rank> makes that rank stop making progress at the
phase; HPCJOIN_COMM_TIMEOUT_S bounds every wait.  Every rank must then exit
non-zero within the timeout, its message naming rank, phase, wait site and
last completed collective (what bench.py prints on a real multi-GPU run).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import hpcjoin  # noqa: E402
from hpcjoin.parallel import init_distributed, make_context  # noqa: E402


def main():
    C = hpcjoin.require_native()
    info = init_distributed(backend="gloo", device=False)
    ctx, comm = make_context(info, "host")
    G = 200_000
    R = C.Relation(C.Relation.local_size_for(G, info.rank, info.world), G, "host", 0)
    S = C.Relation(C.Relation.local_size_for(G, info.rank, info.world), G, "host", 0)
    R.generate(C.GenSpec(seed=1), C.Relation.local_offset_for(G, info.rank, info.world))
    S.generate(C.GenSpec(seed=2), C.Relation.local_offset_for(G, info.rank, info.world))
    t0 = time.time()
    try:
        C.HashJoin(R, S, ctx, C.JoinConfig()).run()
    except Exception as e:  # noqa: BLE001
        print(f"RANK_FAILED rank={info.rank} after={time.time() - t0:.1f}s msg={e}", file=sys.stderr, flush=True)
        os._exit(4)  # no teardown: peers may still sit in a collective
    print(f"RANK_DONE rank={info.rank}", flush=True)
    hpcjoin.parallel.shutdown()


if __name__ == "__main__":
    main()
