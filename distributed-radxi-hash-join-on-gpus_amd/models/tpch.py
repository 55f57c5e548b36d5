"""TPC-H-like orders x lineitem join with 32-byte payloads (BASELINE config 5).

orders(o_orderkey, 32 B payload) x lineitem(l_orderkey, 32 B payload):
* o_orderkey uses the TPC-H sparse layout ((k / 8) * 32 + k % 8 + 1), every
  order has 4 lineitems (lineitem key = orderkey of a random order, each
  exactly 4 times: the MODULO generator);
* payload rows stay on the rank that generated them (32 B per row, a pure
  function of (seed, rid), so results are verifiable anywhere);
* the join moves only 8-byte CompressedTuples (keys reach 2^33 and rids 2^33
  at SF1000, so keyShift = 33), materializes (o_rid, l_rid) pairs, then
  fetches both payload rows per pair with a request/response all-to-all
  (operators/LateMaterialization).
Output rows: [o_rid, l_rid, orders payload (4 x u64), lineitem payload (4 x u64)].
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from .._native import require_native
from ..parallel import DistInfo, init_distributed, make_context
from . import workloads as W

ORDERS_SEED, LINEITEM_SEED = 0x0DE45, 0x11AE17E


@dataclass
class TpchJoin:
    workload: W.Workload
    location: str = "auto"
    info: DistInfo = None
    communicator: object = None
    fused: bool = True

    def __post_init__(self):
        C = require_native()
        if self.location == "auto":
            self.location = "device" if torch.cuda.is_available() else "host"
        self.info = self.info or init_distributed(device=self.location == "device")
        self.ctx, self.comm = make_context(self.info, self.location, self.communicator)
        w, r, n = self.workload, self.info.rank, self.info.world
        self.orders, self.lineitem = w.relations(self.info, self.location)
        dev = f"cuda:{self.info.local_rank}" if self.location == "device" else "cpu"
        self.o_off = C.Relation.local_offset_for(w.inner_size, r, n)
        self.l_off = C.Relation.local_offset_for(w.outer_size, r, n)
        self.o_rows = C.ops.generate_payload(self.orders.local_size(), self.o_off, ORDERS_SEED, dev)
        self.l_rows = C.ops.generate_payload(self.lineitem.local_size(), self.l_off, LINEITEM_SEED, dev)
        self.engine = C.HashJoin(self.orders, self.lineitem, self.ctx, w.join_config())

    def run(self):
        """One join + late materialization; returns (result dict, output rows tensor).

        With ``fused`` (default) a device join at N = 1 writes the output rows
        from its build/probe directly (HashJoin.join_materialized: no pair
        array, inner rows re-read while their work item is hot); elsewhere the
        pairs are materialized by a separate request/response pass."""
        if self.fused and self.engine.can_fuse_rows:
            t0 = time.perf_counter()
            res, out = self.engine.join_materialized(self.ctx, self.o_rows, self.o_off, self.workload.inner_size,
                                                     self.l_rows, self.l_off, self.workload.outer_size)
            if self.location == "device":
                torch.cuda.synchronize()
            t2 = time.perf_counter()
            res = dict(res, join_wall_ms=(t2 - t0) * 1e3, materialize_ms=0.0, total_ms=(t2 - t0) * 1e3)
            return res, out
        t0 = time.perf_counter()
        res = self.engine.run()
        t1 = time.perf_counter()
        out, phases = self.engine.materialize_payloads(self.ctx, self.o_rows, self.o_off, self.workload.inner_size,
                                                       self.l_rows, self.l_off, self.workload.outer_size,
                                                       return_stats=True)
        if self.location == "device":
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = dict(res, join_wall_ms=(t1 - t0) * 1e3, materialize_ms=(t2 - t1) * 1e3, total_ms=(t2 - t0) * 1e3,
                   materialize_phases=phases)
        return res, out


def payload_reference(rids: torch.Tensor, seed: int) -> torch.Tensor:
    """Expected payload rows for the given rids (computed by the host formula)."""
    C = require_native()
    rows = [C.ops.generate_payload(1, int(r), seed, "cpu")[0] for r in rids.tolist()]
    return torch.stack(rows) if rows else torch.empty(0, 4, dtype=torch.int64)


def verify_sample(out: torch.Tensor, k: int = 64) -> bool:
    """Spot-check k output rows: payloads must be those of the rids they carry."""
    if out.shape[0] == 0:
        return True
    n = out.shape[0]
    k = min(k, n)
    # integer sample positions (a float linspace rounds past the last row at 6e8 rows)
    pos = torch.arange(k, dtype=torch.int64) * (n - 1) // max(k - 1, 1)
    assert int(pos.max()) < n
    sel = out[pos.to(out.device)].cpu()
    return bool(torch.equal(sel[:, 2:6], payload_reference(sel[:, 0], ORDERS_SEED)) and
                torch.equal(sel[:, 6:10], payload_reference(sel[:, 1], LINEITEM_SEED)))
