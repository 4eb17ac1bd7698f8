"""Process-group plumbing for tensor parallelism.

One process drives one GPU (``torch.distributed.run`` / one pod container per
rank). Rank discovery and the RCCL bootstrap go through ``torch.distributed``;
the per-token collectives themselves run inside the C++ engine on its own
RCCL communicator (``ncclCommInitRank`` with a unique id broadcast here), so
they are enqueued on the engine's HIP stream and captured in its hipGraph.

The CPU backend's tensor-parallel mode (used to validate the shard plan
without GPUs) gets host collectives over a gloo group.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence, Tuple

import numpy as np

_GLOO = None


def dist_ready() -> bool:
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except Exception:
        return False


def check_tensor_split(tensor_split: Optional[Sequence[float]], world: int) -> list:
    """Per-rank weights for the row-split shard plan (runtime/shard.h): heads are
    apportioned in whole kv heads, FFN features in 256-wide superblocks, by these
    ratios (llama.cpp's ``tensor_split`` semantics: proportions, not sizes).
    Trailing zeros (GPUs a node has but the group does not use) are dropped;
    returns [] for an even split."""
    if not tensor_split:
        return []
    ts = [float(v) for v in tensor_split]
    while ts and ts[-1] == 0:
        ts.pop()
    if len(ts) != world or any(v <= 0 for v in ts):
        raise ValueError(f"tensor_split {list(tensor_split)} must give a positive weight to each of the {world} "
                         "ranks")
    return ts


def tp_group_info(tensor_split: Optional[Sequence[float]] = None) -> Tuple[int, int]:
    """(rank, world) of the tensor-parallel group = the default process group."""
    if not dist_ready():
        return 0, 1
    import torch.distributed as dist
    world = dist.get_world_size()
    check_tensor_split(tensor_split, world)
    return dist.get_rank(), world


def broadcast_nccl_id(make_id: Callable[[], bytes]) -> bytes:
    """Rank 0 creates the RCCL unique id, every rank receives it."""
    import torch.distributed as dist
    obj = [make_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def broadcast_object(obj, src: int = 0, group=None):
    """Rank `src`'s object on every rank."""
    import torch.distributed as dist
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=group)
    return box[0]


def allgather_bytes(b: bytes, group=None) -> list:
    """Every rank's bytes object, in rank order (IPC handle exchange)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, b, group=group)
    return out


def _gloo_group():
    global _GLOO
    import torch.distributed as dist
    if dist.get_backend() == "gloo":
        return None
    if _GLOO is None:
        _GLOO = dist.new_group(backend="gloo")
    return _GLOO


def host_collectives():
    """(allreduce, allgather) over host float32 numpy buffers for the C++ CPU engine."""
    import torch
    import torch.distributed as dist
    group = _gloo_group()
    world = dist.get_world_size()

    def allreduce(buf: np.ndarray) -> None:
        dist.all_reduce(torch.from_numpy(buf), group=group)   # in place on the engine's buffer

    def allgather(local: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(local))
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return torch.cat(out).numpy()

    return allreduce, allgather


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))
