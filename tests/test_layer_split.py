"""Upstream's split_mode=LAYER placement (runtime/layer_split_backend.py) on the CPU: llama.cpp's
layer -> device rule, and the stage chain (hidden states of each prompt chunk / decoded token
through every stage in order, logits from the last) with fake stages. The HIP stages run in
tests/test_layer_split_gpu.py."""
import types

import numpy as np
import pytest

from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams
from llama_fastapi_k8s_gpu_amd.runtime.layer_split_backend import LayerSplitBackend, layer_ranges


@pytest.mark.parametrize("n_layer,ts,want", [
    # l / (n_layer + 1) < c_i (the output layer counts as one more): 2 x 32 -> 17 + 15 (+ head)
    (32, [1, 1], [(0, 0, 17), (1, 17, 32)]),
    (32, [3, 1], [(0, 0, 25), (1, 25, 32)]),         # l / 33 < 0.75 -> l <= 24
    (80, [1] * 8, [(i, b, e) for i, (b, e) in enumerate(
        [(0, 11), (11, 21), (21, 31), (31, 41), (41, 51), (51, 61), (61, 71), (71, 80)])]),
    (4, [1, 0, 1], [(0, 0, 3), (2, 3, 4)]),          # a zero entry: that GPU gets no layer
    (3, [1, 1, 1, 1], [(0, 0, 1), (1, 1, 2), (2, 2, 3)]),  # more GPUs than layers (l / 4 < 1/4, 2/4, 3/4)
    (5, [2, 1], [(0, 0, 4), (1, 4, 5)]),             # l / 6 < 2/3 -> device 0 for l = 0..3
])
def test_layer_ranges_follow_llama_cpp(n_layer, ts, want):
    got = layer_ranges(n_layer, ts)
    assert got == want
    # contiguous cover of [0, n_layer)
    assert got[0][1] == 0 and got[-1][2] == n_layer
    assert all(a[2] == b[1] for a, b in zip(got, got[1:]))


def test_layer_ranges_rejects_empty_split():
    with pytest.raises(ValueError):
        layer_ranges(8, [0, 0])


class _Stage:
    """A fake stage over layers [b, e): hidden h -> h + (e - b) per row; the first stage embeds
    token t as a row of t; the last returns 'logits' with a peak at int(last row value) % V."""

    def __init__(self, b, e, device, n_layer, V, d, log):
        self.b, self.e, self.device, self.n_layer, self.V, self.d, self.log = b, e, device, n_layer, V, d, log
        self.healthy, self.last_error, self.device_bytes = True, "", 100

    def eval_stage(self, x, tokens, pos0):
        self.log.append((self.b, pos0, len(tokens) if x is None else x.shape[0]))
        h = np.repeat(np.asarray(tokens, np.float32)[:, None], self.d, 1) if x is None else np.asarray(x)
        h = h + (self.e - self.b)
        if self.e < self.n_layer:
            return h
        logits = np.zeros(self.V, np.float32)
        logits[int(h[-1, 0]) % self.V] = 1.0
        return logits


def _backend(ts, n_batch=4, V=50, n_layer=6):
    log = []
    hp = types.SimpleNamespace(n_layer=n_layer, n_vocab=V)
    be = LayerSplitBackend("unused.gguf", hp, tensor_split=ts, n_ctx=64, n_batch=n_batch,
                           stage_factory=lambda b, e, dv: _Stage(b, e, dv, n_layer, V, 3, log))
    return be, log


def test_stage_chain_order_and_chunks():
    be, log = _backend([1, 2], n_batch=4)
    assert [(s.b, s.e, s.device) for s in be.stages] == [(0, 3, 0), (3, 6, 1)]
    logits = be.eval_logits([5, 6, 7, 8, 9, 10], 3)
    # two prompt chunks (4 + 2 tokens) at positions 3 and 7, each through stage 0 then stage 1
    assert log == [(0, 3, 4), (3, 3, 4), (0, 7, 2), (3, 7, 2)]
    assert int(np.argmax(logits)) == (10 + 6) % 50       # token 10 plus 6 layers
    h = be.health()
    assert h["ok"] and h["backend"] == "layer" and h["stages"] == [[0, 0, 3], [1, 3, 6]]
    assert be.device_memory() == {"hip:0": 100, "hip:1": 100}


def test_stage_chain_generates_greedy():
    be, log = _backend([1, 1, 1], n_batch=8)
    r = be.generate([1, 2, 3], 0, 4, SamplingParams(temperature=0.0), [])
    # each next token = previous + 6 (the fake model), one decode position per token
    assert r.tokens == [9, 15, 21, 27]
    assert [p for b, p, _ in log if b == 0] == [0, 3, 4, 5]


def test_layer_devices_map_entries_to_devices():
    log = []
    hp = types.SimpleNamespace(n_layer=4, n_vocab=10)
    be = LayerSplitBackend("unused.gguf", hp, tensor_split=[1, 1], n_ctx=16, layer_devices=[0, 0],
                           stage_factory=lambda b, e, dv: _Stage(b, e, dv, 4, 10, 2, log))
    assert be.devices == [0, 0]
    with pytest.raises(ValueError):
        LayerSplitBackend("unused.gguf", hp, tensor_split=[1, 1], layer_devices=[0],
                          stage_factory=lambda b, e, dv: _Stage(b, e, dv, 4, 10, 2, log))


def test_facade_routes_multi_gpu_layer_splits():
    from llama_fastapi_k8s_gpu_amd.engine.llama import _layer_split
    assert _layer_split("layer", [1, 1])
    assert not _layer_split("layer", [1, 0])          # one GPU with weight: the plain engine
    assert not _layer_split("layer", None)
    assert not _layer_split("row", [1, 1])            # tensor parallelism
    assert not _layer_split("none", [1, 1])
