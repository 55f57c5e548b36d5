"""Worker for test_ipc_ordering: two processes on one GPU drive the one-sided
windows' IPC calls (core/ExecContext ipcExport / ipcImport) in the orders
behind round 4's failures (profiles/r4final4/rccl_repeat4.log: an inexact
one-sided join after a workspace re-layout; rccl_repeat10.log:
hipIpcOpenMemHandle -> invalid device pointer).  Rank 0 exports, rank 1
imports; every step is a fixed sequence separated by collectives.

  1. two windows in one allocation (a join's inner and outer windows)
  2. the exporter re-lays its workspace out (free + allocate, same address)
     while the importer still holds its mapping -- the engine closes the
     stale mapping (generation moved) and re-opens: exact
  3. the same, but with a second, unbalanced raw open of the old handle in
     the importer (round 4's engine opened per window): the runtime hands the
     new handle's open the OLD mapping and a put through it is lost -- the
     engine's tag check must refuse that import instead
  4. a handle opened only after the exporter freed its allocation (raw), and
     the engine's coordinated order (release, barrier, free, export, import)

Raw steps only observe (handle equality, what a read sees, where a put lands)
through mappings the runtime still reports as device memory.  Engine steps
are checked; rank 1 prints one JSON line of observations (IPC_ORDER), rank 0
its IPC event log.  Reference semantics: passive-target MPI_Put into
exactly-sized windows (/root/reference/data/Window.cpp:86-144,180-191).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import hpcjoin  # noqa: E402
from hpcjoin.parallel import init_distributed  # noqa: E402

MiB = 1 << 20
TAGS = list(range(1, 32))


def pat(tag, n=4096):
    """n bytes that name `tag` (so a read says which write it saw)."""
    return bytes((tag * 37 + i) & 0xFF for i in range(n))


def which(buf):
    for t in TAGS:
        if buf == pat(t, len(buf)):
            return t
    return None


def main():
    C = hpcjoin.require_native()
    info = init_distributed(backend="gloo", device=True)
    assert info.world == 2, "two ranks: 0 exports, 1 imports"
    ctx = C.ExecContext("device", info.local_rank, C.LocalCommunicator())
    exporter = info.rank == 0
    obs, failed = {}, []

    def check(name, got, want):
        """An engine-path observation; the run fails at the end (after the
        observations are printed) unless it is `want`."""
        obs[name] = got
        if got != want:
            failed.append(f"{name}: got {got!r}, want {want!r}")

    def share(obj):
        out = [None, None]
        dist.all_gather_object(out, obj)
        return out[0]  # what the exporter sent

    def rd(addr):
        return which(C.ipc.read(addr, 4096))

    def imp(e):
        return ctx.ipc_import(0, e[0], e[2], e[3], e[4])

    def relayout(tag):
        """Exporter: free the workspace and allocate it again (the same
        address, in practice), write `tag` into a new window, export it."""
        ctx.reserve_workspace(64 * MiB)
        q = ctx.workspace_scratch(MiB)
        C.ipc.write(q, pat(tag))
        e = ctx.ipc_export(q)
        torch.cuda.synchronize()
        return q, e

    ctx.reserve_workspace(64 * MiB)

    # 1. Two windows in one allocation.
    if exporter:
        p1, p2 = ctx.workspace_scratch(MiB), ctx.workspace_scratch(MiB)
        C.ipc.write(p1, pat(1))
        C.ipc.write(p2, pat(2))
        e1, e2 = ctx.ipc_export(p1), ctx.ipc_export(p2)
        base = p1 - e1[1]
        raw = [C.ipc.get_handle(base), C.ipc.get_handle(base)]
        torch.cuda.synchronize()
        m = share({"e1": e1, "e2": e2, "raw": raw})
    else:
        m = share(None)
        obs["1_raw_handles_of_one_allocation_equal"] = m["raw"][0] == m["raw"][1]
        check("1_engine_one_export_per_allocation", m["e1"][0] == m["e2"][0] and m["e1"][4] == m["e2"][4], True)
        b1, b2 = imp(m["e1"]), imp(m["e2"])
        check("1_engine_one_mapping", [b1 == b2, ctx.ipc_mappings()], [True, 1])
        check("1_engine_reads", [rd(b1 + m["e1"][1]), rd(b2 + m["e2"][1])], [1, 2])
        C.ipc.write(b1 + m["e1"][1] + 4096, pat(3))  # a put
        torch.cuda.synchronize()
    e_first = m["e1"]
    dist.barrier()
    got = share(rd(p1 + 4096) if exporter else None)
    if not exporter:
        check("1_engine_put_lands", got, 3)

    # 2. Re-layout while the importer still holds the mapping.
    if exporter:
        q, e3 = relayout(4)
        m = share({"e3": e3, "same_va": q == p1})
    else:
        m = share(None)
        obs["2_relayout_same_address"] = m["same_va"]
        obs["2_relayout_raw_handle_equal"] = m["e3"][0] == e_first[0]
        b3 = imp(m["e3"])
        check("2_engine_reads_after_relayout", rd(b3 + m["e3"][1]), 4)
        C.ipc.write(b3 + m["e3"][1] + 4096, pat(5))
        torch.cuda.synchronize()
    dist.barrier()
    got = share(rd(q + 4096) if exporter else None)
    if not exporter:
        check("2_engine_put_lands", got, 5)

    # 3. Round 4's state: an extra open of the current handle that is never
    #    closed, then another re-layout at the same address.
    if not exporter:
        e_cur = m["e3"]
        leak = C.ipc.open(e_cur[0])  # the runtime's open count of this handle: 2
        obs["3_extra_open_same_mapping"] = leak == b3
    dist.barrier()
    if exporter:
        q, e4 = relayout(6)
        m = share({"e4": e4})
    else:
        m = share(None)
        obs["3_handle_equal"] = m["e4"][0] == e_cur[0]
        # raw (round 4's import: close the stale mapping once, open the new handle)
        ctx.release_imports()  # closes the engine's mapping; `leak` keeps the old one open
        r = C.ipc.open(m["e4"][0])
        obs["3_raw_reopen_is_old_mapping"] = r == leak
        if C.ipc.is_device_pointer(r):
            obs["3_raw_reopen_reads"] = rd(r + m["e4"][1])  # 4 = the FREED allocation's window
            C.ipc.write(r + m["e4"][1] + 4096, pat(7))  # a put through it
            torch.cuda.synchronize()
        C.ipc.close(r)
        # engine: the tag read back through the fresh open is the freed
        # allocation's, so the import must throw
        try:
            imp(m["e4"])
            check("3_engine_refuses_stale_mapping", "imported", "refused")
        except RuntimeError as e:
            check("3_engine_refuses_stale_mapping", "refused", "refused")
            obs["3_engine_error"] = str(e).split("\n")[0][:200]
    dist.barrier()
    got = share(rd(q + 4096) if exporter else None)
    if not exporter:
        obs["3_raw_put_landed_in_new_window"] = got == 7  # False = lost put (round 4's wrong count)
        C.ipc.close(leak)  # balance the extra open: the old mapping goes away
        b4 = imp(m["e4"])
        check("3_engine_reads_once_balanced", rd(b4 + m["e4"][1]), 6)
        ctx.release_imports()

    # 4. Open after free (raw), then the engine's coordinated order.
    dist.barrier()
    if exporter:
        stale = ctx.ipc_export(q)
        q, e5 = relayout(8)  # frees the allocation `stale` names
        m = share({"stale": stale, "e5": e5})
    else:
        m = share(None)
        try:
            r = C.ipc.open(m["stale"][0])
            obs["4_raw_open_after_free"] = "opened"
            if C.ipc.is_device_pointer(r):
                obs["4_raw_open_after_free_reads"] = rd(r + m["e5"][1])
            C.ipc.close(r)
        except RuntimeError as e:
            obs["4_raw_open_after_free"] = "failed: " + str(e).split("\n")[0][:160]
        try:
            imp(m["stale"])
            obs["4_engine_open_after_free"] = "imported"
        except RuntimeError as e:
            obs["4_engine_open_after_free"] = "refused: " + str(e).split("\n")[0][:160]
        ctx.release_imports()
    dist.barrier()  # engine order: every import closed before the exporter frees
    if exporter:
        q, e6 = relayout(9)
        m = share({"e6": e6})
    else:
        m = share(None)
        b6 = imp(m["e6"])
        check("4_engine_coordinated_reads", rd(b6 + m["e6"][1]), 9)
        C.ipc.write(b6 + m["e6"][1] + 4096, pat(10))
        torch.cuda.synchronize()
        ctx.release_imports()
    dist.barrier()
    got = share(rd(q + 4096) if exporter else None)
    if not exporter:
        check("4_engine_coordinated_put_lands", got, 10)
        obs["importer_log"] = [list(e[:5]) for e in ctx.ipc_log()]
        obs["failed"] = failed
        print("IPC_ORDER " + json.dumps(obs), flush=True)
    else:
        print("EXPORTER_LOG " + json.dumps([list(e[:5]) for e in ctx.ipc_log()]), flush=True)
    dist.barrier()
    assert not failed, failed
    del ctx
    dist.destroy_process_group()
    print(f"[rank {info.rank}] OK", flush=True)


if __name__ == "__main__":
    main()
