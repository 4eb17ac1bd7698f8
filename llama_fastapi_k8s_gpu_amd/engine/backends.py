"""Inference backends behind the ``Llama`` facade.

Every backend implements one call the facade needs per request::

    generate(prompt_tokens, n_keep, max_new, params, stop_ids, poll=None, on_token=None)
        -> GenerationResult

``n_keep`` tokens of the KV cache are reused from the previous call (upstream
``Llama.generate`` prefix reuse); the rest of the prompt is
prefilled, then tokens are sampled until a stop id, ``max_new`` or a ``poll()``
that returns True (cooperative cancel of timed-out requests).

  * ``HipBackend``      - the MI355X engine (C++ runtime + gfx950 kernels,
                          hipGraph decode, GPU sampler, optional RCCL TP)
  * ``CpuBackend``      - the C++ CPU backend (n_gpu_layers = 0; OpenMP)
  * ``ReferenceBackend``- float32 torch reference (tests, debugging)
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from .sampling import SamplingParams, sample_token


@dataclass
class GenerationResult:
    tokens: List[int]
    finish_reason: str           # "stop" | "length" | "cancelled"
    n_evaluated: int             # tokens now resident in the KV cache (prompt + generated[:-1] ...)
    prefill_s: float = 0.0
    decode_s: float = 0.0
    n_prefilled: int = 0


class ReferenceBackend:
    name = "reference"

    def __init__(self, reader, n_ctx: int, **_):
        from ..models.llama import ReferenceLlama
        self.model = ReferenceLlama(reader, n_ctx=n_ctx)
        self.n_ctx = n_ctx

    def health(self):
        return {"ok": True, "backend": self.name}

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        t0 = time.perf_counter()
        history = list(prompt)
        logits = self.model.forward(history[n_keep:], n_keep).numpy()
        t1 = time.perf_counter()
        out: List[int] = []
        n_eval = len(history)
        reason = "length"
        stops = set(stop_ids)
        for step in range(max_new):
            if poll is not None and poll():
                reason = "cancelled"
                break
            tok = sample_token(logits, history[-params.last_n:] if params.last_n else [], params, step)
            out.append(tok)
            history.append(tok)
            if on_token:
                on_token(tok)
            if tok in stops:
                reason = "stop"
                break
            if step + 1 == max_new or n_eval >= self.n_ctx:
                break
            logits = self.model.forward([tok], n_eval).numpy()
            n_eval += 1
        return GenerationResult(out, reason, n_eval, t1 - t0, time.perf_counter() - t1, len(prompt) - n_keep)
