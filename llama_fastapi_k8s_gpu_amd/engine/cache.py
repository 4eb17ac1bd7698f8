"""Prompt caches and saved states (llama-cpp-python ``LlamaState``, ``LlamaRAMCache``,
``Llama.set_cache``).

A state is the token list resident in the KV cache plus a snapshot of that KV (host
bytes, or an HBM buffer for :class:`LlamaDeviceCache`). With a cache set, a request
whose prompt shares a longer prefix with a cached state than with the live KV cache
restores that state first, so only the new suffix is prefilled; after the request
the new state is cached under its token list. On MI355X the device cache keeps the
snapshots in HBM (288 GB holds thousands of 1K-token Llama-3-8B states at 128 MiB
each) and a restore is one HBM-to-HBM strided copy.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Any, Optional, Sequence, Tuple

import numpy as np


@dataclass
class LlamaState:
    input_ids: np.ndarray          # tokens resident in the KV cache
    scores: Optional[np.ndarray]   # not kept (the engines keep last-token logits only)
    n_tokens: int
    llama_state: Any               # backend KV snapshot (host array / tensors / HBM buffer)
    llama_state_size: int          # bytes
    seed: int


def longest_token_prefix(a: Sequence[int], b: Sequence[int]) -> int:
    n = 0
    for x, y in zip(a, b):
        if x != y:
            break
        n += 1
    return n


class BaseLlamaCache:
    on_device = False

    def __init__(self, capacity_bytes: int = 2 << 30):
        self.capacity_bytes = int(capacity_bytes)

    @property
    def cache_size(self) -> int:
        raise NotImplementedError

    def __getitem__(self, key: Sequence[int]) -> LlamaState:
        raise NotImplementedError

    def __contains__(self, key: Sequence[int]) -> bool:
        raise NotImplementedError

    def __setitem__(self, key: Sequence[int], value: LlamaState) -> None:
        raise NotImplementedError


class LlamaRAMCache(BaseLlamaCache):
    """LRU of states keyed by token tuple; lookup returns the entry sharing the
    longest prefix with the key (KeyError if none shares any)."""

    def __init__(self, capacity_bytes: int = 2 << 30):
        super().__init__(capacity_bytes)
        self.cache_state: "OrderedDict[Tuple[int, ...], LlamaState]" = OrderedDict()

    @property
    def cache_size(self) -> int:
        return sum(s.llama_state_size for s in self.cache_state.values())

    def _find_longest_prefix_key(self, key: Tuple[int, ...]) -> Optional[Tuple[int, ...]]:
        best, best_len = None, 0
        for k in self.cache_state:
            n = longest_token_prefix(k, key)
            if n > best_len:
                best, best_len = k, n
        return best

    def __getitem__(self, key: Sequence[int]) -> LlamaState:
        k = self._find_longest_prefix_key(tuple(key))
        if k is None:
            raise KeyError("Key not found")
        self.cache_state.move_to_end(k)
        return self.cache_state[k]

    def __contains__(self, key: Sequence[int]) -> bool:
        return self._find_longest_prefix_key(tuple(key)) is not None

    def __setitem__(self, key: Sequence[int], value: LlamaState) -> None:
        key = tuple(key)
        if key in self.cache_state:
            del self.cache_state[key]
        self.cache_state[key] = value
        while self.cache_size > self.capacity_bytes and len(self.cache_state) > 1:
            self.cache_state.popitem(last=False)


class LlamaDeviceCache(LlamaRAMCache):
    """:class:`LlamaRAMCache` whose snapshots live in GPU memory (HIP backend; other
    backends fall back to host snapshots)."""
    on_device = True

    def __init__(self, capacity_bytes: int = 32 << 30):
        super().__init__(capacity_bytes)


LlamaCache = LlamaRAMCache
