"""General path (sparse 63-bit keys, key-only words) at one outer size:
inner GR (env, default 1e9) unique sparse keys, outer argv[1] uniform
foreign keys over the inner domain (DENSE=1: the same keys without the
sparse bijection); two joins, JoinConfig from HPCJOIN_<FIELD> variables.
Used to bisect the >2^31-slot span-offset bug (profiles/r3cnt/README.md).

    GR=1e9 python tools/general_path_sizes.py 1.6e9
"""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, hpcjoin
from hpcjoin.parallel import init_distributed, make_context
from hpcjoin.utils import config_from_dict
C = hpcjoin.require_native()
info = init_distributed()
ctx, comm = make_context(info, "device")
G_R = int(float(os.environ.get("GR", "1e9")))
G_S = int(float(sys.argv[1]))
sp = os.environ.get("DENSE") != "1"
inner = C.GenSpec(seed=1234); inner.sparse64 = sp
outer = C.GenSpec(distribution=C.KeyDistribution.UNIFORM, seed=4321, domain=G_R); outer.sparse64 = sp
exp = C.Relation.expected_matches(inner, G_R, outer, G_S)
R = C.Relation(G_R, G_R, "device", 0); R.generate(inner, 0)
S = C.Relation(G_S, G_S, "device", 0); S.generate(outer, 0)
j = C.HashJoin(R, S, ctx, config_from_dict())
out = [j.run() for _ in range(2)]
keys = ("global_matches", "inner_received", "outer_received", "local_fallbacks", "network_fallbacks", "reruns")
print(os.environ.get("TAG"), G_S, repr(j.plan), exp, [{k: out_i.get(k) for k in keys} for out_i in out],
      {k: round(out[-1][k], 2) for k in ("dev_network_ms", "dev_local_partition_ms", "dev_build_probe_ms")}, flush=True)
