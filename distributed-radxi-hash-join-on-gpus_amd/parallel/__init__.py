"""Process bootstrap and communicators: one process per MI355X.

* ``init_distributed()`` reads RANK / WORLD_SIZE / LOCAL_RANK (torchrun) and
  initialises torch.distributed (``nccl`` = RCCL on ROCm, ``gloo`` on CPU).
* ``make_communicator()`` returns the native communicator the engine uses:
  ``RcclCommunicator`` (device, direct xGMI peer links; its ncclUniqueId is
  broadcast over torch.distributed), ``ProcessGroupCommunicator`` (host
  reference path over gloo), or ``LocalCommunicator`` (world of one).
"""
from .bootstrap import DistInfo, init_distributed, make_communicator, make_context, shutdown  # noqa: F401
