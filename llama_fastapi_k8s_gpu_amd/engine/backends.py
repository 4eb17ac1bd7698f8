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
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .sampling import HostSampler, SamplingParams, token_logprobs


@dataclass
class GenerationResult:
    tokens: List[int]
    finish_reason: str           # "stop" | "length" | "cancelled"
    n_evaluated: int             # tokens now resident in the KV cache (prompt + generated[:-1] ...)
    prefill_s: float = 0.0
    decode_s: float = 0.0
    n_prefilled: int = 0
    # per generated token: (log p(token), [(id, log p)] top-n) of the raw logits, when asked for
    logprobs: Optional[List[Tuple[float, List[Tuple[int, float]]]]] = None


def host_generate(forward: Callable[[Sequence[int], int], np.ndarray], prompt: Sequence[int], n_keep: int,
                  max_new: int, params: SamplingParams, stop_ids: Sequence[int], n_ctx: int,
                  poll: Optional[Callable[[], bool]] = None, on_token: Optional[Callable[[int], None]] = None,
                  sample_fn: Optional[Callable[[np.ndarray, List[int], int], int]] = None) -> GenerationResult:
    """The host-sampler generation loop every backend shares for what its native
    sampler does not cover (mirostat, tail-free/typical off-device, logit bias on the
    CPU, log-probabilities): ``forward(tokens, pos0)`` evaluates tokens into the KV
    cache and returns the last token's raw logits; sampling is :class:`HostSampler`
    (or ``sample_fn(logits, window, step)``)."""
    t0 = time.perf_counter()
    hist = list(prompt)
    n_keep = n_keep if 0 <= n_keep < len(hist) else 0
    logits = forward(hist[n_keep:], n_keep)
    t1 = time.perf_counter()
    sampler = HostSampler(params)
    sample = sample_fn or sampler.sample
    out: List[int] = []
    lps = [] if params.n_probs > 0 else None
    reason = "length"
    stops = set(stop_ids)
    for step in range(max_new):
        if poll is not None and poll():
            reason = "cancelled"
            break
        window = hist[-params.last_n:] if params.last_n > 0 else []
        raw = logits
        if params.logits_processor is not None:
            logits = np.asarray(params.logits_processor(np.asarray(hist, np.int64), np.array(raw, np.float32)),
                                np.float32)
        tok = int(sample(logits, window, step))
        if lps is not None:
            lps.append(token_logprobs(raw, tok, params.n_probs))
            if params.logprob_cb is not None:
                params.logprob_cb(lps[-1])
        out.append(tok)
        hist.append(tok)
        if on_token:
            on_token(tok)
        if tok in stops:
            reason = "stop"
            break
        if step + 1 == max_new or len(hist) > n_ctx - 1:
            break
        logits = forward([tok], len(hist) - 1)
    return GenerationResult(out, reason, len(prompt) + max(0, len(out) - 1), t1 - t0,
                            time.perf_counter() - t1, len(prompt) - n_keep, lps)


class ReferenceBackend:
    name = "reference"

    def __init__(self, reader, n_ctx: int, **_):
        from ..models.llama import ReferenceLlama
        self.model = ReferenceLlama(reader, n_ctx=n_ctx)
        self.n_ctx = n_ctx

    def health(self):
        return {"ok": True, "backend": self.name}

    def save_kv(self, n: int, on_device: bool = False):
        return self.model.k_cache[:, :n].clone(), self.model.v_cache[:, :n].clone()

    def load_kv(self, kv, n: int):
        self.model.k_cache[:, :n] = kv[0]
        self.model.v_cache[:, :n] = kv[1]

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        return host_generate(lambda toks, pos0: self.model.forward(list(toks), pos0).numpy(), prompt, n_keep,
                             max_new, params, stop_ids, self.n_ctx, poll, on_token)
