"""Native RCCL communicator bootstrap (one communicator per process/GPU, over xGMI).

The 128-byte ncclUniqueId made by rank 0 travels through the torch.distributed TCP store;
every rank then calls ncclCommInitRank inside the extension.  Collectives run on the caller's
HIP stream on device buffers -- the MI355X replacement for the reference's host-buffer
MPI_Scatter / MPI_Gather (/root/reference/namegensf.cu:636,889) and for the gradient
all-reduce the north star adds.
"""
from __future__ import annotations

import itertools

from .dist import DistCtx, store_exchange

_counter = itertools.count()


def make_comm(ctx: DistCtx):
    if ctx.world <= 1:
        return None
    from ..ops import load_ext
    C = load_ext()
    C.set_rank(ctx.rank)
    key = f"gk_rccl_uid_{next(_counter)}"
    uid = C.RcclComm.unique_id() if ctx.rank == 0 else None
    uid = store_exchange(key, uid)
    return C.RcclComm(uid, ctx.rank, ctx.world)
