"""Serving one tensor-parallel model from N processes (one per GPU).

The reference serves one model per pod from one process (gunicorn -w 1,
reference docker/Dockerfile.app:12). With ``split_mode=row`` over N GPUs every
rank holds a shard and must run every generation in lock-step (its all-reduces
pair with the other ranks'). Rank 0 owns the HTTP server and the admission
queue unchanged.

  * MI355X engine: the engine itself mirrors every command rank 0 runs to the
    followers over a native shared-memory channel (csrc/runtime/tp_channel.h);
    followers call ``Llama.follow()``. Continuous batching and cooperative
    cancel work as on one GPU (a cancelled row simply gets no further steps).
  * CPU backend (shard-plan validation): ``TPLeader`` broadcasts each
    facade call over a gloo control group and ``follower_loop`` replays it.
    Generation is deterministic across ranks, so every rank stops at the same
    token; cooperative cancel is off there (a leader that stopped early would
    leave followers blocked in a collective), and one lock keeps the broadcast
    order equal to the execution order.
"""
from __future__ import annotations

import datetime
import logging
import os
from typing import Any, Dict, Optional

logger = logging.getLogger(__name__)

_LONG = datetime.timedelta(days=365)   # followers may idle between requests


class TPLeader:
    """Engine wrapper for rank 0 (CPU backend): mirrors each call to the follower ranks."""
    supports_cancel = False
    batch_width = 1

    def __init__(self, llm, group=None):
        import threading
        self.llm = llm
        self.group = group
        # broadcast + generate as one critical section: the followers replay calls in
        # broadcast order, which must be the order rank 0 runs them
        self._lock = threading.Lock()

    def _send(self, op: str, kw: Optional[Dict[str, Any]]):
        import torch.distributed as dist
        dist.broadcast_object_list([(op, kw)], src=0, group=self.group)

    def create_chat_completion(self, **kw):
        kw.pop("cancel_event", None)
        with self._lock:
            self._send("chat", kw)
            return self.llm.create_chat_completion(**kw)

    def create_completion(self, prompt, **kw):
        kw.pop("cancel_event", None)
        with self._lock:
            self._send("completion", dict(kw, prompt=prompt))
            return self.llm.create_completion(prompt, **kw)

    def health(self):
        return self.llm.health()

    def device_memory(self):
        return self.llm.device_memory()

    def close(self):
        with self._lock:
            self._send("stop", None)
        self.llm.close()


def follower_loop(llm, group=None) -> None:
    import torch.distributed as dist
    while True:
        obj = [None]
        dist.broadcast_object_list(obj, src=0, group=group)
        op, kw = obj[0]
        if op == "stop":
            return
        try:
            if op == "chat":
                r = llm.create_chat_completion(**kw)
            elif op == "completion":
                r = llm.create_completion(kw.pop("prompt"), **kw)
            else:
                r = None
            if r is not None and not isinstance(r, dict):   # a stream: drive it like the leader does
                for _ in r:
                    pass
        except Exception as e:  # the leader raises the same error and reports it
            logger.warning("follower: %s failed: %s", op, e)


def init_tp(settings) -> tuple:
    """Initialise torch.distributed from the torchrun env; returns (rank, world, control group).

    One bootstrap for the container, the bench and the tests alike: a gloo process group
    carries the control traffic only (the seed, the RCCL unique id, the P2P IPC handles, the
    CPU backend's call mirroring). The MI355X engine creates and owns the only RCCL
    communicator (ncclCommInitRank inside the engine, its collectives on the engine stream and
    in its hipGraphs) - a torch NCCL process group would be a second communicator on the same
    GPUs that nothing uses."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return 0, 1, None
    dist.init_process_group("gloo", timeout=_LONG)
    ctrl = None   # the default group is the gloo control group
    rank = dist.get_rank()
    if settings.seed is None:   # every rank must sample with the same seed
        obj = [int.from_bytes(os.urandom(4), "little") if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=ctrl)
        settings.seed = obj[0]
    settings.split_mode = "row"
    return rank, world, ctrl
