from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .._native import require_native


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


def init_distributed(backend: str | None = None, device: bool | None = None) -> DistInfo:
    """Initialise torch.distributed from the launcher environment (idempotent)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("HPCJOIN_SHARE_GPU") == "1" and world > 1:
        # Rehearsal of the multi-GPU path on a box with fewer GPUs than ranks:
        # ranks share devices round-robin, and each rank claims its own RCCL
        # host id so RCCL's duplicate-GPU check passes and it falls back to its
        # socket transport.  Every engine code path (RCCL all-gather,
        # all-to-allv, all-reduce, torch.distributed bootstrap) still runs.
        # Must happen before anything initialises RCCL.
        os.environ["NCCL_HOSTID"] = f"hpcjoin-rehearsal-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        local_rank = local_rank % max(1, torch.cuda.device_count())
    if device is None:
        device = torch.cuda.is_available()
    if device:
        torch.cuda.set_device(local_rank)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        be = backend or ("nccl" if device else "gloo")
        kwargs = {"backend": be, "init_method": "env://", "rank": rank, "world_size": world}
        if be == "nccl":
            kwargs["device_id"] = torch.device("cuda", local_rank)
        dist.init_process_group(**kwargs)
    return DistInfo(rank=rank, world=world, local_rank=local_rank)


def make_communicator(info: DistInfo, location: str = "device"):
    """Native communicator for ``location`` ("device" -> RCCL, "host" -> gloo PG)."""
    C = require_native()
    if info.world == 1:
        return C.LocalCommunicator()
    if location == "device":
        obj = [C.rccl_unique_id() if info.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return C.RcclCommunicator(obj[0], info.rank, info.world, info.local_rank)
    pg = dist.distributed_c10d._get_default_group()
    return C.ProcessGroupCommunicator(pg)


def make_context(info: DistInfo, location: str = "device", communicator=None):
    C = require_native()
    comm = communicator if communicator is not None else make_communicator(info, location)
    return C.ExecContext(location, info.local_rank if location == "device" else -1, comm), comm


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
