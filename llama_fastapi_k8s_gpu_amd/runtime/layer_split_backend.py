"""LayerSplitBackend: upstream's ``split_mode="layer"`` across several GPUs of one process.

The reference builds its engine with ``Llama(model_path, n_gpu_layers=-1, n_ctx=...)``
(reference api.py:23-27); llama-cpp-python's default ``split_mode`` is LAYER, which with
more than one visible GPU and a ``tensor_split`` puts contiguous layer ranges on the GPUs
in those proportions. The same placement here: one MI355X engine per stage, stage ``i``
on device ``i`` holding layers ``[begin_i, end_i)`` and its part of the KV cache; the
first stage gathers the embedding, the last holds the output norm and head. A token's
hidden states (``n_embd`` floats per row) pass from stage to stage once per prompt chunk
or decoded token (device to device, ``hipMemcpyPeerAsync``). Generation over HIP stages is one
native call (``Engine::chain_generate``, engine.cpp): each stage's decode step is a captured
hipGraph, the last stage samples on the device with the single-GPU engine's sampler and its
token / position state is copied back to every stage, and steps are ordered across devices by
events - the host only reads tokens, two steps in flight, exactly as the one-GPU ``generate``.
Sampling options the device sampler lacks (grammar, mirostat, ...) and non-HIP stage objects
take the host loop (host C++ sampling chain, bit-identical uniforms, as the hybrid backend).
One MI355X holds every BASELINE model (288 GB), so this is a capacity and compatibility
placement, not a speed-up: a single decode still walks every layer in order. Tensor
parallelism (``split_mode="row"``) is the multi-GPU speed path.

Layer assignment follows llama.cpp's full-offload rule: with ``tensor_split`` normalised to
cumulative fractions ``c_0 < c_1 < ... = 1``, layer ``l`` goes to the first device ``i`` with
``l / (n_layer + 1) < c_i`` - the divisor counts the output layer as one more offloaded layer,
which lands on the last device. (The reference ships no llama.cpp source, so this parity is
from the upstream rule as recalled, pinned by tests/test_layer_split.py, not checked against a
file.)
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from ..engine.backends import GenerationResult, host_generate
from ..engine.sampling import SamplingParams
from . import load_cpu, load_hip
from .cpu_backend import native_sampling, sampling_dict
from .hip_backend import gpu_sampling_dict


def layer_ranges(n_layer: int, tensor_split: Sequence[float]) -> List[Tuple[int, int, int]]:
    """(device index, first layer, end layer) for every device that receives a layer."""
    w = [max(0.0, float(v)) for v in tensor_split]
    tot = sum(w)
    if n_layer <= 0 or tot <= 0:
        raise ValueError("layer split needs n_layer > 0 and a tensor_split with a positive entry")
    cum, acc = [], 0.0
    for v in w:
        acc += v / tot
        cum.append(acc)
    cum[-1] = 1.0 + 1e-9  # (rounding: the last device with weight takes the remainder)
    dev_of = []
    for layer in range(n_layer):
        f = layer / (n_layer + 1)   # the output layer counts as layer n_layer
        dev_of.append(next(i for i, c in enumerate(cum) if f < c and w[i] > 0))
    out: List[Tuple[int, int, int]] = []
    for layer, dv in enumerate(dev_of):
        if out and out[-1][0] == dv:
            out[-1] = (dv, out[-1][1], layer + 1)
        else:
            out.append((dv, layer, layer + 1))
    return out


class LayerSplitBackend:
    name = "layer"

    def __init__(self, model_path: str, hparams, tensor_split: Sequence[float], n_ctx: int = 1024,
                 n_batch: int = 512, layer_devices: Optional[Sequence[int]] = None, stage_factory=None, **_):
        """``layer_devices[i]``: the HIP device of ``tensor_split`` entry ``i`` (default ``i``;
        the one-GPU rehearsal maps every entry to device 0). ``stage_factory(begin, end,
        device)`` builds one stage (default: a HIP engine over that layer range)."""
        n_layer = hparams.n_layer
        self.ranges = layer_ranges(n_layer, tensor_split)
        devs = list(layer_devices) if layer_devices is not None else list(range(len(tensor_split)))
        if len(devs) < len(tensor_split):
            raise ValueError("layer_devices needs one device per tensor_split entry")
        self.n_ctx = n_ctx
        self.n_batch = min(n_batch, n_ctx)
        self.n_vocab = int(hparams.n_vocab)
        self._hip = None
        if stage_factory is None:
            hip = load_hip()
            self._hip = hip

            def stage_factory(begin, end, device):
                return hip.Engine(model_path, n_ctx=n_ctx, n_batch=self.n_batch, device=device, use_graph=False,
                                  layer_begin=begin, layer_end=end)
        self.devices = [devs[i] for i, _, _ in self.ranges]
        self.stages = [stage_factory(b, e, d) for (_, b, e), d in zip(self.ranges, self.devices)]
        self._cpu_mod = None

    def health(self):
        ok = all(bool(getattr(s, "healthy", True)) for s in self.stages)
        err = next((s.last_error for s in self.stages if getattr(s, "last_error", "")), None)
        return {"ok": ok, "backend": self.name, "stages": [[d, b, e] for (_, b, e), d in zip(self.ranges, self.devices)],
                "error": err}

    def device_memory(self):
        mem = {}
        for s, d in zip(self.stages, self.devices):
            mem[f"hip:{d}"] = mem.get(f"hip:{d}", 0) + int(getattr(s, "device_bytes", 0))
        return mem

    def save_kv(self, n: int, on_device: bool = False):
        return [s.kv_save(int(n)) for s in self.stages]

    def load_kv(self, kv, n: int):
        for s, k in zip(self.stages, kv):
            s.kv_load(k, int(n))

    def _forward(self, tokens: Sequence[int], pos0: int) -> np.ndarray:
        """Tokens into every stage's KV cache (chunks of at most n_batch) -> last raw logits."""
        tokens = [int(t) for t in tokens]
        logits = None
        # HIP stages hand the hidden states over device to device (hipMemcpyPeerAsync into the
        # next stage's activation buffer); other stage objects through the host
        peer = len(self.stages) > 1 and all(hasattr(s, "eval_stage_peer") for s in self.stages)
        for p in range(0, len(tokens), self.n_batch):
            chunk, at = tokens[p:p + self.n_batch], int(pos0 + p)
            if peer:
                self.stages[0].eval_stage(None, chunk, at, False)
                for prev, st in zip(self.stages, self.stages[1:]):
                    logits = st.eval_stage_peer(prev, len(chunk), at)
                continue
            h = self.stages[0].eval_stage(None, chunk, at)
            for st in self.stages[1:]:
                h = st.eval_stage(h, [], at)
            logits = h
        return np.asarray(logits, np.float32).reshape(-1)

    def eval_logits(self, tokens: Sequence[int], pos0: int = 0) -> np.ndarray:
        return self._forward(tokens, pos0)

    def native_chain(self, params: Optional[SamplingParams] = None) -> bool:
        """Generation runs natively (``chain_generate``): HIP stages and device-sampler options."""
        hip = self._hip
        if hip is None or not hasattr(hip, "chain_generate") or not all(isinstance(s, hip.Engine) for s in self.stages):
            return False
        return params is None or params.gpu_compatible(self.n_vocab)

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        if self.native_chain(params):
            r = self._hip.chain_generate(self.stages, [int(t) for t in prompt], int(n_keep), int(max_new),
                                         gpu_sampling_dict(params, self.n_vocab), [int(t) for t in stop_ids],
                                         poll, on_token)
            return GenerationResult(list(r["tokens"]), r["finish"], int(r["n_evaluated"]), r["prefill_s"],
                                    r["decode_s"], int(r["n_prefilled"]))
        fn = None
        if native_sampling(params):
            if self._cpu_mod is None:
                self._cpu_mod = load_cpu()
            sp = sampling_dict(params)
            mod = self._cpu_mod
            fn = lambda logits, window, step: mod.sample(logits, window, sp, step)  # noqa: E731
        return host_generate(self._forward, prompt, n_keep, max_new, params, stop_ids, self.n_ctx, poll, on_token,
                             sample_fn=fn)
