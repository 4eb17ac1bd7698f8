"""Sampling: parameters, the counter-based RNG shared with the native code, and
the host reference of the upstream sampler chain.

Chain order (llama.cpp ``_LlamaSamplingContext.sample``, as driven by
llama-cpp-python 0.2.77 ``Llama.sample``):
  logit bias -> repetition/frequency/presence penalties over the last ``last_n``
  tokens -> [temp <= 0: argmax] -> [mirostat 1/2: temperature -> mirostat]
  -> top-k -> tail-free -> typical -> top-p -> min-p -> temperature -> softmax -> draw.
Temperature is applied AFTER filtering, so the filters see temperature-1
probabilities (each filter renormalises over the candidates that reach it, as
``llama_sample_softmax`` does). Penalty math per token with count c>0 in the
window: ``l = l*rp if l <= 0 else l/rp ; l -= c*freq + presence``. ``min_keep``
is 1 everywhere (upstream: ``max(1, n_probs)``, and n_probs is 0 for completions).

Mirostat keeps its ``mu`` across the tokens of one request (initialised to
2*tau), which is the algorithm's definition; llama-cpp-python 0.2.77 builds a new
sampling context per token and so re-initialises ``mu`` every step - that quirk
is not reproduced.

The draw uses ``philox_uniform(seed, step)`` - a SplitMix64 hash of (seed,
step) mapped to [0,1) - which the HIP sampler (csrc/kernels/sampler.hip) and the
C++ CPU backend implement bit-identically, so CPU/GPU runs at the same seed draw
the same uniforms. (The upstream mt19937 stream is not reproduced - fidelity is
in distribution)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

MASK64 = (1 << 64) - 1
MIROSTAT_M = 100          # llama-cpp-python's mirostat_m for v1
GPU_MAX_LOGIT_BIAS = 64   # entries the GPU sampler applies in its first stage


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
    logit_bias: Dict[int, float] = field(default_factory=dict)
    mirostat_mode: int = 0
    mirostat_tau: float = 5.0
    mirostat_eta: float = 0.1
    n_probs: int = 0          # > 0: the caller wants log-probabilities of each generated token
    # host-only hooks: ``logits_processor(input_ids, scores) -> scores`` (llama-cpp-python's
    # LogitsProcessorList contract) and a sink for each token's (logprob, top) entry
    logits_processor: Optional[Callable] = field(default=None, compare=False, repr=False)
    logprob_cb: Optional[Callable] = field(default=None, compare=False, repr=False)
    # engine.grammar.GrammarState of this request (grammar-constrained sampling, host only)
    grammar: Optional[object] = field(default=None, compare=False, repr=False)

    def greedy(self) -> bool:
        return self.temperature <= 0.0

    def gpu_compatible(self, vocab: int) -> bool:
        """Whether the on-device chain (csrc/kernels/sampler.hip) computes exactly this
        chain: top-k within its 64-candidate window, few enough bias entries, no
        mirostat, no host-side log-probabilities."""
        if self.mirostat_mode and not self.greedy():
            return False
        if self.n_probs > 0 or self.logits_processor is not None or self.grammar is not None \
                or len(self.logit_bias) > GPU_MAX_LOGIT_BIAS:
            return False
        if self.greedy():
            return True
        return 0 < self.top_k <= 64 or (self.top_k <= 0 and vocab <= 64)


def apply_logit_bias(logits: np.ndarray, p: SamplingParams) -> np.ndarray:
    if not p.logit_bias:
        return logits
    out = np.array(logits, np.float32, copy=True)
    n = out.shape[0]
    for t, b in p.logit_bias.items():
        if 0 <= int(t) < n:
            out[int(t)] += np.float32(b)
    return out


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


def _sorted_desc(l: np.ndarray, ids: Optional[np.ndarray] = None) -> np.ndarray:
    """Indices into ``l`` by descending value, ties by ascending token id."""
    ids = np.arange(l.shape[0]) if ids is None else ids
    return np.lexsort((ids, -l))


def _top_p_prefix(l: np.ndarray, top_p: float, min_p: float):
    """For an unlimited top-k on a large vocabulary: the sorted candidate prefix that
    top-p / min-p can keep, found without sorting the whole vocabulary, and the
    softmax normaliser of the WHOLE vocabulary (top-p's cumulative mass is relative
    to it). Returns None when the prefix is not provably inside a quarter of it."""
    n = l.shape[0]
    if n <= 1024 or (top_p >= 1.0 and min_p <= 0.0):
        return None
    mx = float(l.max())
    e = np.exp(l.astype(np.float64) - mx)
    z = float(e.sum())
    m = 256
    while m < n // 4:
        part = np.argpartition(-l, m)[:m]
        thr = l[part].min()
        sel = np.nonzero(l >= thr)[0]            # every tie of the m-th value included
        ok_p = top_p < 1.0 and e[sel].sum() / z >= top_p
        ok_m = min_p > 0.0 and thr < mx + math.log(min_p)
        if ok_p or ok_m:
            return sel[_sorted_desc(l[sel], sel)], z
        m *= 4
    return None


def tail_free(ids: np.ndarray, vals: np.ndarray, z: float, min_keep: int = 1):
    """llama_sample_tail_free: cut where the normalised |second derivative| of the
    sorted probabilities accumulates past z (candidates sorted descending)."""
    if z >= 1.0 or len(ids) <= 2:
        return ids, vals
    pr = _softmax(vals)
    d1 = pr[:-1] - pr[1:]
    d2 = np.abs(d1[:-1] - d1[1:])
    s = d2.sum()
    d2 = d2 / s if s > 1e-6 else np.full_like(d2, 1.0 / len(d2))
    cum = np.cumsum(d2)
    last = len(ids)
    hit = np.nonzero((cum > z) & (np.arange(len(d2)) >= min_keep))[0]
    if len(hit):
        last = int(hit[0])
    return ids[:last], vals[:last]


def typical(ids: np.ndarray, vals: np.ndarray, tp: float, min_keep: int = 1):
    """llama_sample_typical: keep the tokens whose surprise is closest to the entropy
    until their mass exceeds tp. Returns the kept set re-sorted by descending logit
    (the next filter's softmax sorts it again upstream)."""
    if tp >= 1.0:
        return ids, vals
    pr = _softmax(vals)
    ent = -np.sum(pr * np.log(np.maximum(pr, 1e-300)))
    shifted = np.abs(-np.log(np.maximum(pr, 1e-300)) - ent)
    order = np.lexsort((np.arange(len(ids)), shifted))   # ascending shifted score, stable
    cum = np.cumsum(pr[order])
    last = len(order)
    hit = np.nonzero((cum > tp) & (np.arange(len(order)) >= min_keep - 1))[0]
    if len(hit):
        last = int(hit[0]) + 1
    keep = np.sort(order[:last])                         # back to descending-logit order
    return ids[keep], vals[keep]


def prepare_logits(logits: np.ndarray, last_tokens: Sequence[int], p: SamplingParams) -> np.ndarray:
    """Logit bias, then the penalties: the values every later stage sees."""
    l = apply_logit_bias(np.asarray(logits, np.float32), p)
    return apply_penalties(l, last_tokens, p).astype(np.float32, copy=False)


def filtered_candidates(logits: np.ndarray, last_tokens: Sequence[int], p: SamplingParams):
    """Returns (token ids, final temperature-scaled logits) of the surviving candidates
    sorted by descending logit - the distribution the draw samples from."""
    return _filter_prepared(prepare_logits(logits, last_tokens, p), p)


def _filter_prepared(l: np.ndarray, p: SamplingParams):
    n = l.shape[0]
    k = p.top_k if 0 < p.top_k < n else n
    order, zfull = None, None
    if k == n and p.tfs_z >= 1.0 and p.typical_p >= 1.0:
        pref = _top_p_prefix(l, p.top_p, p.min_p)
        if pref is not None:
            order, zfull = pref
    if order is None:
        if k < n:
            part = np.argpartition(-l, k - 1)[:k]
            thr = l[part].min()
            sel = np.nonzero(l >= thr)[0]              # ties of the k-th value: lowest ids win
            order = sel[_sorted_desc(l[sel], sel)][:k]
        else:
            order = _sorted_desc(l)
    ids, vals = order, l[order]
    ids, vals = tail_free(ids, vals, p.tfs_z)
    ids, vals = typical(ids, vals, p.typical_p)
    # top-p (temperature 1)
    if p.top_p < 1.0:
        if zfull is not None:   # a prefix of the whole vocabulary: normalise by all of it
            probs = np.exp(vals.astype(np.float64) - vals[0]) / zfull
        else:
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


def _draw(probs: np.ndarray, u: float) -> int:
    cum = np.cumsum(probs)
    return min(int(np.searchsorted(cum, u * cum[-1], side="right")), len(probs) - 1)


def sample_token(logits: np.ndarray, last_tokens: Sequence[int], p: SamplingParams, step: int) -> int:
    """Stateless host reference sampler (everything but mirostat, whose ``mu`` is
    per-request state: use :class:`HostSampler`)."""
    if p.grammar is not None or p.mirostat_mode:
        return HostSampler(p).sample(logits, last_tokens, step)
    if p.greedy():
        return int(np.argmax(prepare_logits(logits, last_tokens, p)))
    ids, vals = filtered_candidates(logits, last_tokens, p)
    return int(ids[_draw(_softmax(vals), philox_uniform(p.seed, step))])


def log_softmax(logits: np.ndarray) -> np.ndarray:
    """``Llama.logits_to_logprobs`` (raw model logits -> natural-log probabilities)."""
    l = np.asarray(logits, np.float64)
    m = l.max()
    return (l - m - np.log(np.exp(l - m).sum())).astype(np.float32)


class HostSampler:
    """The host chain with per-request state (mirostat ``mu``)."""

    def __init__(self, p: SamplingParams):
        self.p = p
        self.mu = 2.0 * p.mirostat_tau

    def _mirostat(self, l: np.ndarray, step: int) -> int:
        p = self.p
        l = l / p.temperature
        order = _sorted_desc(l)
        vals = l[order]
        probs = _softmax(vals)
        u = philox_uniform(p.seed, step)
        if p.mirostat_mode == 1:
            n = float(l.shape[0])
            m = min(MIROSTAT_M, len(probs) - 1)
            t = np.log((np.arange(m) + 2.0) / (np.arange(m) + 1.0))
            b = np.log(np.maximum(probs[:m], 1e-300) / np.maximum(probs[1:m + 1], 1e-300))
            s_hat = float((t * b).sum() / (t * t).sum()) if m > 0 else 1.0
            eps = s_hat - 1.0
            try:
                k = ((eps * 2.0 ** self.mu) / (1.0 - n ** (-eps))) ** (1.0 / s_hat)
            except (OverflowError, ZeroDivisionError):
                k = float(len(probs))
            k = len(probs) if not math.isfinite(k) else int(max(1, min(k, len(probs))))
            kept = _softmax(vals[:k])
        else:
            surprise = -np.log2(np.maximum(probs, 1e-300))
            over = np.nonzero(surprise > self.mu)[0]
            k = int(over[0]) if len(over) else len(probs)
            k = max(k, 1)
            kept = _softmax(vals[:k])
        j = _draw(kept, u)
        self.mu -= p.mirostat_eta * (-math.log2(max(float(kept[j]), 1e-300)) - p.mirostat_tau)
        return int(order[j])

    def sample(self, logits: np.ndarray, last_tokens: Sequence[int], step: int) -> int:
        p = self.p
        l = prepare_logits(logits, last_tokens, p)
        if p.grammar is not None:
            tok = self._sample_grammar(l, step)
            p.grammar.accept_token(tok)
            return tok
        if p.greedy():
            return int(np.argmax(l))
        if p.mirostat_mode in (1, 2):
            return self._mirostat(l, step)
        ids, vals = _filter_prepared(l, p)
        return int(ids[_draw(_softmax(vals), philox_uniform(p.seed, step))])

    def _sample_grammar(self, l: np.ndarray, step: int) -> int:
        """Upstream masks every grammar-rejected token to -inf before the chain. The
        chain's top-k only sees the k best ALLOWED tokens, so with top_k > 0 (or greedy)
        candidates are checked in descending-logit order until k are found; otherwise
        the allowed set is enumerated by the grammar's vocabulary-trie walk."""
        p, gs = self.p, self.p.grammar
        n = l.shape[0]
        need = 1 if p.greedy() else (p.top_k if 0 < p.top_k < n and not p.mirostat_mode else 0)
        allowed: Optional[List[int]] = None
        if need:
            found: List[int] = []
            m = min(n, 256)
            done = 0
            while done < n and len(found) < need and done < 8192:
                part = np.argpartition(-l, m - 1)[:m] if m < n else np.arange(n)
                part = part[_sorted_desc(l[part], part)]
                for t in part[done:]:
                    if gs.allows(int(t)):
                        found.append(int(t))
                        if len(found) == need:
                            break
                done = m
                m = min(n, m * 4)
            if len(found) == need:
                allowed = found
        if allowed is None:
            allowed = gs.allowed_tokens()
        if not allowed:   # dead end (e.g. the token budget cut a structure): end the generation
            return int(min(gs.v.eog)) if gs.v.eog else int(np.argmax(l))
        masked = np.full(n, -np.inf, np.float32)
        idx = np.asarray(allowed, np.int64)
        masked[idx] = l[idx]
        if p.greedy():
            return int(np.argmax(masked))
        if p.mirostat_mode in (1, 2):
            return self._mirostat(masked, step)
        ids, vals = _filter_prepared(masked, p)
        return int(ids[_draw(_softmax(vals), philox_uniform(p.seed, step))])


def token_logprobs(logits: np.ndarray, token: int, n: int) -> Tuple[float, List[Tuple[int, float]]]:
    """(log p(token), top-n (id, log p)) of the RAW model logits - what llama-cpp-python
    reports as ``logprobs`` (``Llama.logits_to_logprobs`` of ``_scores``)."""
    lp = log_softmax(logits)
    n = max(0, min(int(n), lp.shape[0]))
    top: List[Tuple[int, float]] = []
    if n:
        part = np.argpartition(-lp, n - 1)[:n]
        part = part[_sorted_desc(lp[part], part)]
        top = [(int(i), float(lp[i])) for i in part]
    return float(lp[int(token)]), top
