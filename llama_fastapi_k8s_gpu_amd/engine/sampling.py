"""Sampling: parameters, the counter-based RNG shared with the native code, and
the host reference of the upstream sampler chain.

Chain order (llama.cpp, as driven by llama-cpp-python 0.2.77):
  repetition/frequency/presence penalties over the last ``last_n`` tokens
  -> top-k -> tail-free (z=1: no-op) -> typical (p=1: no-op) -> top-p -> min-p
  -> temperature -> softmax -> draw.
Temperature is applied AFTER filtering, so the filters see temperature-1
probabilities. Penalty math per token with count c>0 in the window:
``l = l*rp if l <= 0 else l/rp ; l -= c*freq + presence``.

The draw uses ``philox_uniform(seed, step)`` - a SplitMix64 hash of (seed,
step) mapped to [0,1) - which the HIP sampler (csrc/kernels/sampler.hip) and the
C++ CPU backend implement bit-identically, so CPU/GPU runs at the same seed draw
the same uniforms. (The upstream mt19937 stream is not reproduced - fidelity is
in distribution)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

MASK64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def philox_uniform(seed: int, step: int) -> float:
    """Uniform in [0,1) with 24-bit resolution (exactly representable in f32)."""
    h = splitmix64((seed & MASK64) ^ ((step * 0xD1B54A32D192ED03) & MASK64))
    return (h >> 40) * (1.0 / (1 << 24))


@dataclass
class SamplingParams:
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.95
    min_p: float = 0.05
    typical_p: float = 1.0
    tfs_z: float = 1.0
    repeat_penalty: float = 1.1
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    last_n: int = 64
    seed: int = 0

    def greedy(self) -> bool:
        return self.temperature <= 0.0


def apply_penalties(logits: np.ndarray, last_tokens: Sequence[int], p: SamplingParams) -> np.ndarray:
    if (p.repeat_penalty == 1.0 and p.frequency_penalty == 0.0 and p.presence_penalty == 0.0) \
            or not len(last_tokens):
        return logits
    window = list(last_tokens)[-p.last_n:] if p.last_n > 0 else []
    counts = {}
    for t in window:
        counts[int(t)] = counts.get(int(t), 0) + 1
    out = logits.copy()
    for t, c in counts.items():
        l = out[t]
        l = l * p.repeat_penalty if l <= 0 else l / p.repeat_penalty
        l -= c * p.frequency_penalty + (1.0 if c > 0 else 0.0) * p.presence_penalty
        out[t] = l
    return out


def _softmax(x: np.ndarray) -> np.ndarray:
    m = x.max()
    e = np.exp((x - m).astype(np.float64))
    return e / e.sum()


def filtered_candidates(logits: np.ndarray, last_tokens: Sequence[int], p: SamplingParams):
    """Returns (token ids, final temperature-scaled logits) of the surviving candidates
    sorted by descending logit - the distribution the draw samples from."""
    l = apply_penalties(np.asarray(logits, np.float32), last_tokens, p).astype(np.float32)
    n = l.shape[0]
    k = p.top_k if 0 < p.top_k < n else n
    # stable descending order: ties broken by lower token id first
    order = np.lexsort((np.arange(n), -l))[:k]
    ids, vals = order, l[order]
    # top-p (temperature 1)
    if p.top_p < 1.0:
        probs = _softmax(vals)
        cum = np.cumsum(probs)
        last = int(np.searchsorted(cum, p.top_p, side="left")) + 1
        last = max(1, min(last, len(ids)))
        ids, vals = ids[:last], vals[:last]
    # min-p: keep p_i >= min_p * p_max  <=>  l_i >= l_max + log(min_p)
    if p.min_p > 0.0:
        thr = vals[0] + np.log(p.min_p)
        keep = max(1, int(np.sum(vals >= thr)))
        ids, vals = ids[:keep], vals[:keep]
    vals = vals / p.temperature
    return ids, vals


def sample_token(logits: np.ndarray, last_tokens: Sequence[int], p: SamplingParams, step: int) -> int:
    """Host reference sampler (also the fallback for parameters the GPU kernel
    does not cover, e.g. top_k <= 0 or > 256)."""
    if p.greedy():
        l = apply_penalties(np.asarray(logits, np.float32), last_tokens, p)
        return int(np.argmax(l))
    ids, vals = filtered_candidates(logits, last_tokens, p)
    probs = _softmax(vals)
    u = philox_uniform(p.seed, step)
    cum = np.cumsum(probs)
    idx = int(np.searchsorted(cum, u * cum[-1], side="right"))
    return int(ids[min(idx, len(ids) - 1)])
