"""Engine construction from Settings (reference api.py:24-28 made configurable)."""
from __future__ import annotations

from ..config import Settings


def build_engine(settings: Settings):
    if settings.engine == "fake":
        from .fake import FakeEngine
        return FakeEngine()
    from .llama import Llama
    tp = {}
    if settings.split_mode == "row":
        tp["tp_comm"] = settings.tp_comm
        if settings.tp_device is not None:
            tp["device"] = settings.tp_device
    return Llama(model_path=settings.model_path, n_gpu_layers=settings.n_gpu_layers,
                 n_ctx=settings.n_ctx, n_batch=settings.n_batch,
                 tensor_split=settings.tensor_split, split_mode=settings.split_mode,
                 main_gpu=settings.main_gpu, seed=settings.seed, chat_format=settings.chat_format,
                 use_graphs=settings.use_graphs, verbose=settings.verbose,
                 **({"max_batch": settings.max_batch} if settings.max_batch > 1 else {}), **tp)
