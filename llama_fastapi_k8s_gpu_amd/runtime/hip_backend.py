"""HipBackend: the MI355X engine behind the ``Llama`` facade.

Placement semantics of the reference's ``Llama(...)`` arguments (reference
api.py:24-28) mapped onto one process per GPU:

  * ``n_gpu_layers=-1`` (or >= n_layer): every layer, the embedding and the
    output head live on the GPU (upstream keeps the embedding on the CPU; we
    gather it on the GPU - SURVEY K1).
  * ``split_mode="row"`` + ``torch.distributed`` initialised with world size N:
    tensor parallelism over N ranks (one per GPU) - heads and FFN features are
    sharded, two all-reduces per layer over xGMI (decode: one-shot P2P kernel;
    prefill: RCCL; ``comm="ipc"``: the P2P kernel for everything, no RCCL - ranks
    may then share a GPU, which is how the one-GPU test box runs TP). The
    vocabulary is split evenly and sampled vocabulary-parallel (each rank's
    top-k candidates are all-gathered, csrc/kernels/sampler.hip). ``tensor_split``
    weights apportion kv heads / FFN superblocks per rank (llama.cpp proportions;
    csrc/runtime/shard.h). Rank 0 drives; ranks 1..N-1 run ``follow()``, which
    replays rank 0's engine commands natively (csrc/runtime/tp_channel.h), so
    continuous batching and cooperative cancel work unchanged under TP.
  * ``split_mode="none"``, or ``"layer"`` without a multi-GPU ``tensor_split``: the model
    runs on ``main_gpu`` (one GPU holds any BASELINE model: 288 GB HBM). A layer split
    over several GPUs is runtime/layer_split_backend.py (contiguous layer ranges per GPU).
  * ``max_batch=M > 1``: continuous batching (under TP the scheduler runs on rank 0). The engine gets M + 1 KV
    slots; a native scheduler thread (csrc/runtime/scheduler.cpp) decodes every
    admitted request as one row of a batched step (one weight stream per step
    instead of one per request) and admits new requests into free slots between
    steps. Requests whose sampler settings the GPU chain does not cover take the
    single-sequence path on slot 0 (serialised with the scheduler by the engine).
"""
from __future__ import annotations

import logging
import os
from typing import Callable, Optional, Sequence

from ..engine.backends import GenerationResult, host_generate
from ..engine.sampling import SamplingParams
from . import load_hip

logger = logging.getLogger(__name__)


def _tp_setup(split_mode: str, tensor_split, comm: str):
    """(tp_rank, tp_size, device, nccl_id, shard weights) from torch.distributed (if initialised)."""
    from ..parallel.comm import broadcast_nccl_id, check_tensor_split, local_rank, tp_group_info
    local = local_rank()
    if split_mode != "row":
        return 0, 1, local, b"", []
    rank, ws = tp_group_info(tensor_split)
    if ws == 1:
        return 0, 1, local, b"", []
    nccl_id = b"" if comm == "ipc" else broadcast_nccl_id(lambda: load_hip().nccl_unique_id())
    return rank, ws, local, nccl_id, check_tensor_split(tensor_split, ws)


def _test_fault() -> str:
    """The fault-injection test hook (EngineOptions::test_fault): ``LFK_TP_FAULT`` is honoured only
    with the explicit opt-in ``LFK_TEST_HOOKS=1`` (the fault tests set both); a stray
    ``LFK_TP_FAULT`` in a pod is ignored, loudly."""
    spec = os.environ.get("LFK_TP_FAULT", "")
    if not spec:
        return ""
    if os.environ.get("LFK_TEST_HOOKS") != "1":
        logger.warning("LFK_TP_FAULT=%s ignored: fault injection needs LFK_TEST_HOOKS=1", spec)
        return ""
    logger.warning("fault-injection test hook active: LFK_TP_FAULT=%s", spec)
    return spec



def gpu_sampling_dict(params: SamplingParams, n_vocab: int) -> dict:
    """The device sampler's options (the engines' ``sampling`` dict)."""
    return {"top_k": params.top_k, "top_p": params.top_p, "min_p": params.min_p,
            "temperature": params.temperature, "repeat_penalty": params.repeat_penalty,
            "frequency_penalty": params.frequency_penalty, "presence_penalty": params.presence_penalty,
            "last_n": params.last_n, "seed": params.seed & 0xFFFFFFFFFFFFFFFF, "tfs_z": params.tfs_z,
            "typical_p": params.typical_p,
            "logit_bias": {int(t): float(b) for t, b in params.logit_bias.items() if 0 <= int(t) < n_vocab}}

class HipBackend:
    name = "hip"

    def __init__(self, model_path: str, hparams, n_ctx: int = 1024, n_gpu_layers: int = -1,
                 tensor_split: Optional[Sequence[float]] = None, split_mode: str = "layer", main_gpu: int = 0,
                 n_batch: int = 512, use_graphs: bool = True, max_batch: int = 1, tp_comm: Optional[str] = None,
                 device: Optional[int] = None, **_):
        hip = load_hip()
        if 0 <= n_gpu_layers < hparams.n_layer:
            raise ValueError(f"n_gpu_layers={n_gpu_layers} < n_layer={hparams.n_layer}: partial offload runs on "
                             "the hybrid backend (backend='hybrid')")
        if split_mode == "layer" and tensor_split and sum(1 for v in tensor_split if float(v) > 0) > 1:
            # upstream's layer split (contiguous layer ranges by tensor_split) is its own backend:
            # the Llama facade routes it to runtime/layer_split_backend.py
            raise ValueError("split_mode='layer' with a multi-GPU tensor_split runs on the layer-split backend "
                             "(backend='layer')")
        comm = tp_comm or "auto"
        rank, size, local, nccl_id, ts = _tp_setup(split_mode, tensor_split, comm)
        if device is None:
            device = local if size > 1 else (main_gpu if split_mode in ("none", "layer") and main_gpu else local)
        self.tp_rank, self.tp_size = rank, size
        max_batch = max(1, int(max_batch or 1))
        self.max_batch = max_batch
        self.engine = hip.Engine(model_path, n_ctx=n_ctx, n_batch=min(n_batch, n_ctx), device=device,
                                 use_graph=use_graphs, tp_rank=rank, tp_size=size, nccl_id=nccl_id,
                                 tensor_split=ts, n_slots=max_batch + 1 if max_batch > 1 else 1, comm=comm,
                                 test_fault=_test_fault() if size > 1 else "")
        self.n_ctx = n_ctx
        self.n_vocab = int(hparams.n_vocab)
        self.n_batch = min(n_batch, n_ctx)  # the engine's prefill chunk bound (eval_logits rejects T > n_batch)
        self.device = device
        if size > 1:
            self._tp_connect(comm)
        # the continuous-batching scheduler drives the engine from rank 0 only
        self.sched = hip.BatchScheduler(self.engine) if max_batch > 1 and rank == 0 else None

    def _tp_connect(self, comm: str):
        """Join the TP group: exchange the ranks' IPC handles (one-shot P2P collectives over
        xGMI) and open the native control channel rank 0 publishes its commands on."""
        import torch.distributed as dist

        from ..parallel.comm import allgather_bytes, broadcast_object
        if comm != "rccl":
            try:
                handles = allgather_bytes(self.engine.p2p_handle())
                self.engine.p2p_open(handles)
            except Exception as e:  # pragma: no cover - depends on the node's IPC support
                if comm == "ipc":
                    raise
                logger.warning("P2P collectives unavailable, using RCCL only: %s", e)
        name = broadcast_object(f"lfk_tp_{os.getpid()}_{os.urandom(6).hex()}" if self.tp_rank == 0 else None)
        if self.tp_rank == 0:
            self.engine.tp_ctl_create(name)
        dist.barrier()
        if self.tp_rank > 0:
            self.engine.tp_ctl_attach(name)
        dist.barrier()

    @property
    def follows(self) -> bool:
        """A follower rank of a TP group: call follow() instead of generating."""
        return self.tp_size > 1 and self.tp_rank > 0

    def follow(self):
        """Follower ranks: replay rank 0's engine commands until rank 0 closes the group."""
        self.engine.follow()

    def health(self):
        h = {"ok": bool(self.engine.healthy), "backend": self.name, "tp": self.tp_size,
             "error": self.engine.last_error or None}
        if self.sched is not None:
            h["batching"] = dict(self.sched.stats(), max_batch=self.max_batch)
        return h

    def batches(self, params: SamplingParams) -> bool:
        """Whether this request runs as a row of the continuous batch (the facade then
        skips its single-sequence lock and KV prefix bookkeeping: the scheduler reuses
        prefixes per slot)."""
        return self.sched is not None and params.gpu_compatible(self.n_vocab)

    def close(self):
        if self.sched is not None:
            self.sched.shutdown()
        if self.tp_size > 1 and self.tp_rank == 0:
            self.engine.tp_stop()

    def device_memory(self):
        return {f"hip:{self.device}": int(self.engine.device_bytes)}

    def _sp(self, params: SamplingParams) -> dict:
        return gpu_sampling_dict(params, self.n_vocab)

    def _generate_batched(self, prompt: Sequence[int], max_new: int, params: SamplingParams,
                          stop_ids: Sequence[int], poll: Optional[Callable[[], bool]],
                          on_token: Optional[Callable[[int], None]]) -> GenerationResult:
        rid = self.sched.submit(list(prompt), int(max_new), self._sp(params), list(stop_ids))
        toks = []
        try:
            while True:
                r = self.sched.wait(rid, len(toks), 20)
                for t in r["tokens"]:
                    toks.append(t)
                    if on_token:
                        on_token(t)
                if r["done"]:
                    break
                if poll is not None and poll():
                    self.sched.cancel(rid)
        finally:
            self.sched.release(rid)
        if r["finish"] == "error":
            raise RuntimeError(r["error"] or "batched generation failed")
        return GenerationResult(toks, r["finish"], len(prompt) + max(0, len(toks) - 1), r["prefill_s"],
                                r["decode_s"], int(r["n_prefilled"]))

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        if not params.gpu_compatible(self.n_vocab):
            return host_generate(self._forward, prompt, n_keep, max_new, params, stop_ids, self.n_ctx, poll,
                                 on_token)
        if self.sched is not None:
            return self._generate_batched(prompt, max_new, params, stop_ids, poll, on_token)
        sp = self._sp(params)
        r = self.engine.generate(list(prompt), int(n_keep), int(max_new), sp, list(stop_ids), poll, on_token)
        return GenerationResult(list(r["tokens"]), r["finish"], int(r["n_evaluated"]), r["prefill_s"],
                                r["decode_s"], int(r["n_prefilled"]))

    def save_kv(self, n: int, on_device: bool = False):
        """KV snapshot of positions [0, n): host bytes, or (``on_device``) an HBM buffer
        filled by a device-to-device strided copy - 288 GB of HBM holds thousands of
        1K-token conversation states, and restoring one costs tens of microseconds."""
        if not on_device:
            return self.engine.kv_save(int(n))
        import torch
        buf = torch.empty(max(1, self.engine.kv_state_bytes(int(n))), dtype=torch.uint8, device=f"cuda:{self.device}")
        self.engine.kv_transfer_ptr(buf.data_ptr(), int(n), False)
        return buf

    def load_kv(self, kv, n: int):
        if hasattr(kv, "data_ptr"):
            if kv.numel() < self.engine.kv_state_bytes(int(n)):
                raise ValueError("load_kv: device snapshot too small")
            self.engine.kv_transfer_ptr(kv.data_ptr(), int(n), True)
        else:
            self.engine.kv_load(kv, int(n))

    def _forward(self, tokens: Sequence[int], pos0: int):
        """Evaluate tokens into the KV cache (prefill chunks of at most n_batch, the
        engine's bound; the eager decode path for single tokens) -> last raw logits."""
        tokens = list(tokens)
        if len(tokens) == 1:
            return self.engine.decode_logits(int(tokens[0]), int(pos0))
        logits = None
        for p in range(0, len(tokens), self.n_batch):
            logits = self.engine.eval_logits(tokens[p:p + self.n_batch], int(pos0 + p))
        return logits
