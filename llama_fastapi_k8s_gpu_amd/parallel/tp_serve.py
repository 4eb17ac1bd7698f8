"""Serving one tensor-parallel model from N processes (one per GPU).

The reference serves one model per pod from one process (gunicorn -w 1,
reference docker/Dockerfile.app:12). With ``split_mode=row`` over N GPUs every
rank holds a shard and must run every generation in lock-step (its RCCL
all-reduces pair with the other ranks'). Rank 0 owns the HTTP server and the
admission queue unchanged; before each engine call it broadcasts the call's
arguments over a CPU (gloo) control group and the follower ranks replay it.

Generation is deterministic across ranks (identical all-reduced activations,
identical gathered logits, shared seed), so every rank stops at the same token
without further coordination. Cooperative cancel is disabled in this mode: a
leader that stopped early would leave followers blocked in a collective.
"""
from __future__ import annotations

import datetime
import logging
import os
from typing import Any, Dict, Optional

logger = logging.getLogger(__name__)

_LONG = datetime.timedelta(days=365)   # followers may idle between requests


class TPLeader:
    """Engine wrapper for rank 0: mirrors each call to the follower ranks."""
    supports_cancel = False

    def __init__(self, llm, group=None):
        self.llm = llm
        self.group = group

    def _send(self, op: str, kw: Optional[Dict[str, Any]]):
        import torch.distributed as dist
        dist.broadcast_object_list([(op, kw)], src=0, group=self.group)

    def create_chat_completion(self, **kw):
        kw.pop("cancel_event", None)
        self._send("chat", kw)
        return self.llm.create_chat_completion(**kw)

    def create_completion(self, prompt, **kw):
        kw.pop("cancel_event", None)
        self._send("completion", dict(kw, prompt=prompt))
        return self.llm.create_completion(prompt, **kw)

    def health(self):
        return self.llm.health()

    def device_memory(self):
        return self.llm.device_memory()

    def close(self):
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
    """Initialise torch.distributed from the torchrun env; returns (rank, world, control group)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return 0, 1, None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", timeout=_LONG, device_id=torch.device("cuda", local))
        ctrl = dist.new_group(backend="gloo", timeout=_LONG)
    else:
        dist.init_process_group("gloo", timeout=_LONG)
        ctrl = None
    rank = dist.get_rank()
    if settings.seed is None:   # every rank must sample with the same seed
        obj = [int.from_bytes(os.urandom(4), "little") if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=ctrl)
        settings.seed = obj[0]
    settings.split_mode = "row"
    return rank, world, ctrl
