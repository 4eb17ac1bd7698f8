"""CpuBackend: the C++ CPU engine (``csrc/cpu/cpu_backend.cpp``) behind the
``Llama`` facade for ``n_gpu_layers=0`` (BASELINE config #1: TinyLlama Q8_0 on
the CPU, reference api.py:24-28 with ``N_GPU_LAYERS=0``).

The CPU engine uses the same planar weight layout and the same q8-activation
integer dot products as the gfx950 GEMV, the same f16 KV cache and the same
SplitMix64 draw, so CPU and GPU runs of one seed agree up to float rounding.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence

from ..engine.backends import GenerationResult, host_generate
from ..engine.sampling import SamplingParams
from . import load_cpu


def native_sampling(p: SamplingParams) -> bool:
    """Whether the C++ CPU sampler (csrc/cpu/cpu_backend.cpp:cpu_sample) implements
    this chain: penalties, top-k, top-p, min-p, temperature - no tail-free, typical,
    logit bias, mirostat or log-probabilities (those take the host loop)."""
    return (p.tfs_z >= 1.0 and p.typical_p >= 1.0 and not p.logit_bias and p.n_probs <= 0
            and p.logits_processor is None and p.grammar is None
            and (p.mirostat_mode == 0 or p.greedy()))


def sampling_dict(p: SamplingParams) -> dict:
    return {"top_k": p.top_k, "top_p": p.top_p, "min_p": p.min_p, "temperature": p.temperature,
            "repeat_penalty": p.repeat_penalty, "frequency_penalty": p.frequency_penalty,
            "presence_penalty": p.presence_penalty, "last_n": p.last_n, "seed": p.seed & 0xFFFFFFFFFFFFFFFF}


class CpuBackend:
    name = "cpu"

    def __init__(self, model_path: str, n_ctx: int = 512, n_threads: Optional[int] = None, n_batch: int = 64,
                 split_mode: str = "none", tensor_split=None, **_):
        cpu = load_cpu()
        threads = int(n_threads or os.environ.get("N_THREADS", 0) or 0)
        rank, size, ts = 0, 1, []
        if split_mode == "row":
            from ..parallel.comm import check_tensor_split, tp_group_info
            rank, size = tp_group_info(tensor_split)
            ts = check_tensor_split(tensor_split, size) if size > 1 else []
        if size > 1 and threads == 0:
            # TP ranks on one host share its cores: an OpenMP team per rank as wide as the
            # machine oversubscribes it, and the per-layer all-reduces then wait on
            # descheduled threads (a 2-rank tiny-model request ran past the 25 s timeout)
            local = int(os.environ.get("LOCAL_WORLD_SIZE", size) or size)
            threads = max(1, len(os.sched_getaffinity(0)) // max(1, local))
        self.engine = cpu.CpuEngine(model_path, n_ctx=n_ctx, n_threads=threads, n_batch=min(n_batch, 128),
                                    tp_rank=rank, tp_size=size, tensor_split=ts)
        if size > 1:
            from ..parallel.comm import host_collectives
            self.engine.set_comm(*host_collectives())
        self.tp_rank, self.tp_size = rank, size
        self.n_ctx = n_ctx

    def health(self):
        return {"ok": True, "backend": self.name, "tp": self.tp_size}

    def device_memory(self):
        return {}

    def save_kv(self, n: int, on_device: bool = False):
        return self.engine.kv_save(int(n))

    def load_kv(self, kv, n: int):
        self.engine.kv_load(kv, int(n))

    def eval_logits(self, tokens: Sequence[int], pos0: int = 0):
        return self.engine.eval_logits(list(tokens), int(pos0))

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        if not native_sampling(params):
            return host_generate(lambda toks, pos0: self.engine.eval_logits(list(toks), int(pos0)), prompt, n_keep,
                                 max_new, params, stop_ids, self.n_ctx, poll, on_token)
        r = self.engine.generate(list(prompt), int(n_keep), int(max_new), sampling_dict(params), list(stop_ids),
                                 poll, on_token)
        return GenerationResult(list(r["tokens"]), r["finish"], int(r["n_evaluated"]), r["prefill_s"],
                                r["decode_s"], int(r["n_prefilled"]))
