"""HipBackend: the MI355X engine behind the ``Llama`` facade.

Placement semantics of the reference's ``Llama(...)`` arguments (reference
api.py:24-28) mapped onto one process per GPU:

  * ``n_gpu_layers=-1`` (or >= n_layer): every layer, the embedding and the
    output head live on the GPU (upstream keeps the embedding on the CPU; we
    gather it on the GPU - SURVEY K1).
  * ``split_mode="row"`` + ``torch.distributed`` initialised with world size N:
    tensor parallelism over N ranks (one per GPU) - heads and FFN features are
    sharded, two all-reduces per layer over xGMI (decode: one-shot P2P kernel;
    prefill: RCCL). ``tensor_split`` weights apportion kv heads / FFN superblocks
    per rank (llama.cpp proportions; csrc/runtime/shard.h), the vocabulary
    split stays even (the logit all-gather moves equal counts).
  * ``split_mode="none"/"layer"`` in one process: the model runs on
    ``main_gpu`` (one GPU holds any BASELINE model: 288 GB HBM).
"""
from __future__ import annotations

import logging
import os
from typing import Callable, Optional, Sequence

from ..engine.backends import GenerationResult
from ..engine.sampling import SamplingParams, sample_token
from . import load_hip

logger = logging.getLogger(__name__)


def _tp_setup(split_mode: str, tensor_split):
    """(tp_rank, tp_size, device, nccl_id, shard weights) from torch.distributed (if initialised)."""
    from ..parallel.comm import broadcast_nccl_id, check_tensor_split, local_rank, tp_group_info
    local = local_rank()
    if split_mode != "row":
        return 0, 1, local, b"", []
    rank, ws = tp_group_info(tensor_split)
    if ws == 1:
        return 0, 1, local, b"", []
    return (rank, ws, local, broadcast_nccl_id(lambda: load_hip().nccl_unique_id()),
            check_tensor_split(tensor_split, ws))


class HipBackend:
    name = "hip"

    def __init__(self, model_path: str, hparams, n_ctx: int = 1024, n_gpu_layers: int = -1,
                 tensor_split: Optional[Sequence[float]] = None, split_mode: str = "layer", main_gpu: int = 0,
                 n_batch: int = 512, use_graphs: bool = True, **_):
        hip = load_hip()
        if 0 <= n_gpu_layers < hparams.n_layer:
            raise ValueError(f"n_gpu_layers={n_gpu_layers} < n_layer={hparams.n_layer}: partial offload runs on "
                             "the hybrid backend (backend='hybrid')")
        rank, size, local, nccl_id, ts = _tp_setup(split_mode, tensor_split)
        device = local if size > 1 else (main_gpu if split_mode in ("none", "layer") and main_gpu else local)
        self.tp_rank, self.tp_size = rank, size
        self.engine = hip.Engine(model_path, n_ctx=n_ctx, n_batch=min(n_batch, n_ctx), device=device,
                                 use_graph=use_graphs, tp_rank=rank, tp_size=size, nccl_id=nccl_id,
                                 tensor_split=ts)
        self.n_ctx = n_ctx
        self.n_batch = min(n_batch, n_ctx)  # the engine's prefill chunk bound (eval_logits rejects T > n_batch)
        self.device = device
        if size > 1:
            self._open_p2p()

    def _open_p2p(self):
        """Exchange the ranks' IPC handles so decode all-reduces take the one-shot
        P2P kernel over xGMI (prefill-sized ones stay on RCCL). Any failure leaves
        the engine on RCCL for everything."""
        import os
        if os.environ.get("LFK_P2P_ALLREDUCE", "1") == "0":
            return
        from ..parallel.comm import allgather_bytes
        try:
            handles = allgather_bytes(self.engine.p2p_handle())
            self.engine.p2p_open(handles)
        except Exception as e:  # pragma: no cover - depends on the node's IPC support
            logger.warning("P2P all-reduce unavailable, using RCCL only: %s", e)

    def health(self):
        return {"ok": bool(self.engine.healthy), "backend": self.name, "tp": self.tp_size,
                "error": self.engine.last_error or None}

    def device_memory(self):
        return {f"hip:{self.device}": int(self.engine.device_bytes)}

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        if not (0 <= params.top_k <= 64) or params.tfs_z != 1.0 or params.typical_p != 1.0:
            return self._generate_host_sampler(prompt, n_keep, max_new, params, stop_ids, poll, on_token)
        sp = {"top_k": params.top_k, "top_p": params.top_p, "min_p": params.min_p,
              "temperature": params.temperature, "repeat_penalty": params.repeat_penalty,
              "frequency_penalty": params.frequency_penalty, "presence_penalty": params.presence_penalty,
              "last_n": params.last_n, "seed": params.seed & 0xFFFFFFFFFFFFFFFF}
        r = self.engine.generate(list(prompt), int(n_keep), int(max_new), sp, list(stop_ids), poll, on_token)
        return GenerationResult(list(r["tokens"]), r["finish"], int(r["n_evaluated"]), r["prefill_s"],
                                r["decode_s"], int(r["n_prefilled"]))

    def _generate_host_sampler(self, prompt, n_keep, max_new, params, stop_ids, poll, on_token):
        """Slow path for sampler settings the GPU kernel does not implement
        (top_k outside [0, 64], tail-free, typical): logits come back to the host."""
        import time
        t0 = time.perf_counter()
        hist = list(prompt)
        e = self.engine
        logits = None
        pos = n_keep
        while pos < len(hist):
            T = min(len(hist) - pos, self.n_batch)
            logits = e.eval_logits(hist[pos:pos + T], pos)
            pos += T
        t1 = time.perf_counter()
        out, reason = [], "length"
        for step in range(max_new):
            if poll is not None and poll():
                reason = "cancelled"
                break
            tok = sample_token(logits, hist[-params.last_n:] if params.last_n else [], params, step)
            out.append(tok)
            hist.append(tok)
            if on_token:
                on_token(tok)
            if tok in set(stop_ids):
                reason = "stop"
                break
            if step + 1 == max_new or len(hist) > self.n_ctx - 1:
                break
            logits = e.decode_logits(tok, len(hist) - 1)
        return GenerationResult(out, reason, len(prompt) + max(0, len(out) - 1), t1 - t0,
                                time.perf_counter() - t1, len(prompt) - n_keep)
