"""HybridBackend: partial offload, ``0 < n_gpu_layers < n_layer``.

Upstream ``n_gpu_layers=N`` (reference api.py:26) keeps the
first ``n_layer - N`` layers on the CPU and offloads the last ``N``. Here the
C++ CPU engine owns the embedding and layers ``[0, n_layer - N)`` (with their
KV cache), the MI355X engine owns layers ``[n_layer - N, n_layer)``, the output
norm and the lm_head (upstream leaves the output layer on the CPU unless
``N > n_layer``; keeping it on the GPU is strictly faster and numerically the
same kernels). Hidden states cross the PCIe boundary once per token
(``n_embd`` floats), logits come back for the host sampler (the same C++
sampler chain as the CPU backend, bit-identical uniforms).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np

from ..engine.backends import GenerationResult, host_generate
from ..engine.sampling import SamplingParams
from . import load_cpu, load_hip
from .cpu_backend import native_sampling, sampling_dict


class HybridBackend:
    name = "hybrid"

    def __init__(self, model_path: str, hparams, n_gpu_layers: int, n_ctx: int = 1024, main_gpu: int = 0,
                 n_threads: Optional[int] = None, n_batch: int = 512, **_):
        n_layer = hparams.n_layer
        if not 0 < n_gpu_layers < n_layer:
            raise ValueError(f"hybrid placement needs 0 < n_gpu_layers < {n_layer}, got {n_gpu_layers}")
        self.n_cpu_layers = n_layer - n_gpu_layers
        cpu, hip = load_cpu(), load_hip()
        self._cpu_mod = cpu
        self.cpu = cpu.CpuEngine(model_path, n_ctx=n_ctx, n_threads=int(n_threads or 0), n_batch=64,
                                 layer_end=self.n_cpu_layers, load_head=False)
        self.gpu = hip.Engine(model_path, n_ctx=n_ctx, n_batch=min(n_batch, n_ctx), device=main_gpu,
                              use_graph=False, layer_begin=self.n_cpu_layers)
        self.n_batch = min(n_batch, n_ctx)
        self.n_ctx = n_ctx
        self.device = main_gpu

    def health(self):
        return {"ok": bool(self.gpu.healthy), "backend": self.name, "cpu_layers": self.n_cpu_layers,
                "error": self.gpu.last_error or None}

    def device_memory(self):
        return {f"hip:{self.device}": int(self.gpu.device_bytes)}

    def save_kv(self, n: int, on_device: bool = False):
        return self.cpu.kv_save(int(n)), self.gpu.kv_save(int(n))

    def load_kv(self, kv, n: int):
        self.cpu.kv_load(kv[0], int(n))
        self.gpu.kv_load(kv[1], int(n))

    def _forward(self, tokens: Sequence[int], pos0: int) -> np.ndarray:
        h = self.cpu.eval_hidden(list(tokens), int(pos0))
        logits = None
        for p in range(0, len(tokens), self.n_batch):
            logits = self.gpu.eval_hidden(h[p:p + self.n_batch], int(pos0 + p))
        return logits

    def eval_logits(self, tokens: Sequence[int], pos0: int = 0) -> np.ndarray:
        return self._forward(tokens, pos0)

    def generate(self, prompt: Sequence[int], n_keep: int, max_new: int, params: SamplingParams,
                 stop_ids: Sequence[int], poll: Optional[Callable[[], bool]] = None,
                 on_token: Optional[Callable[[int], None]] = None) -> GenerationResult:
        fn = None
        if native_sampling(params):
            sp = sampling_dict(params)
            fn = lambda logits, window, step: self._cpu_mod.sample(logits, window, sp, step)  # noqa: E731
        return host_generate(self._forward, prompt, n_keep, max_new, params, stop_ids, self.n_ctx, poll, on_token,
                             sample_fn=fn)
