"""``Llama`` - the engine facade the service calls.

Compatible with the subset of ``llama_cpp.Llama`` the reference uses
(reference api.py:7, 24-28, 55-63)::

    llm = Llama(model_path=..., n_gpu_layers=-1, n_ctx=1024)
    llm.create_chat_completion(messages, stream=False, temperature=1.2, top_p=0.9,
                               frequency_penalty=0.7, presence_penalty=0.8)
    -> {"id", "object", "created", "model", "choices": [{"message": {...}}], "usage"}

plus ``tensor_split`` / ``split_mode`` / ``main_gpu`` / ``seed`` / ``n_batch`` and
``create_completion`` / ``tokenize`` / ``detokenize``. Upstream semantics kept:
``max_tokens=None`` => n_ctx - n_prompt; prompt >= n_ctx raises ValueError
("Requested tokens ... exceed context window"), KV prefix reuse across calls,
the default sampler chain and values.
"""
from __future__ import annotations

import logging
import os
import threading
import time
import uuid
from typing import Any, Dict, Iterator, List, Optional, Sequence, Union

from ..gguf.reader import GGUFReader
from ..models.llama import LlamaHParams
from .backends import GenerationResult, ReferenceBackend
from .chat_format import get_formatter
from .sampling import SamplingParams
from .tokenizer import tokenizer_from_metadata

logger = logging.getLogger(__name__)


def _select_backend(reader, hp: LlamaHParams, n_gpu_layers: int, backend: Optional[str]) -> str:
    if backend:
        return backend
    env = os.environ.get("LLAMA_BACKEND")
    if env:
        return env
    n_gpu = hp.n_layer + 1 if n_gpu_layers < 0 else n_gpu_layers
    if n_gpu == 0:
        return "cpu"
    try:
        import torch
        if torch.cuda.is_available():
            return "hip" if n_gpu >= hp.n_layer else "hybrid"
    except Exception:
        pass
    logger.warning("no GPU visible: n_gpu_layers=%d falls back to the CPU backend", n_gpu_layers)
    return "cpu"


class Llama:
    supports_cancel = True

    def __init__(self, model_path: str, n_gpu_layers: int = 0, n_ctx: int = 512, n_batch: int = 512,
                 tensor_split: Optional[Sequence[float]] = None, split_mode: str = "layer",
                 main_gpu: int = 0, seed: Optional[int] = None, chat_format: Optional[str] = None,
                 last_n_tokens_size: int = 64, use_graphs: bool = True, verbose: bool = True,
                 backend: Optional[str] = None, n_threads: Optional[int] = None, **kwargs):
        t0 = time.perf_counter()
        if not os.path.exists(model_path):
            raise ValueError(f"Model path does not exist: {model_path}")
        self.model_path = model_path
        reader = GGUFReader(model_path)
        self.metadata = reader.metadata
        self.hparams = LlamaHParams.from_metadata(self.metadata)
        self.tokenizer = tokenizer_from_metadata(self.metadata)
        if not self.hparams.n_vocab:
            self.hparams.n_vocab = self.tokenizer.n_vocab
        self._n_ctx = int(n_ctx) if n_ctx else self.hparams.n_ctx_train
        self.n_batch = n_batch
        self.last_n_tokens_size = last_n_tokens_size
        self.verbose = verbose
        self._seed = seed if seed is not None else int.from_bytes(os.urandom(4), "little")
        self._n_requests = 0
        self._lock = threading.Lock()
        bos = self.tokenizer.tokens[self.tokenizer.bos_id] if self.tokenizer.bos_id >= 0 else ""
        eos = self.tokenizer.tokens[self.tokenizer.eos_id] if self.tokenizer.eos_id >= 0 else ""
        self.chat_format, self._formatter = get_formatter(self.metadata, chat_format, bos, eos)
        kind = _select_backend(reader, self.hparams, n_gpu_layers, backend)
        self.backend_name = kind
        if kind == "reference":
            self._backend = ReferenceBackend(reader, self._n_ctx)
        elif kind == "cpu":
            from ..runtime.cpu_backend import CpuBackend
            self._backend = CpuBackend(model_path, self._n_ctx, n_threads=n_threads, split_mode=split_mode,
                                       tensor_split=tensor_split)
        elif kind == "hybrid":
            from ..runtime.hybrid_backend import HybridBackend
            self._backend = HybridBackend(model_path, self.hparams, n_gpu_layers=n_gpu_layers, n_ctx=self._n_ctx,
                                          main_gpu=main_gpu, n_threads=n_threads, n_batch=n_batch)
        elif kind == "hip":
            from ..runtime.hip_backend import HipBackend
            self._backend = HipBackend(model_path, self.hparams, n_ctx=self._n_ctx, n_gpu_layers=n_gpu_layers,
                                       tensor_split=tensor_split, split_mode=split_mode, main_gpu=main_gpu,
                                       n_batch=n_batch, use_graphs=use_graphs, **kwargs)
        else:
            raise ValueError(f"unknown backend {kind!r}")
        del reader
        self._kv_tokens: List[int] = []   # tokens resident in the KV cache (prefix reuse)
        self.load_time_s = time.perf_counter() - t0
        if verbose:
            logger.info("loaded %s (%s backend, chat_format=%s) in %.2fs", model_path, kind,
                        self.chat_format, self.load_time_s)

    # ---------------------------------------------------------------- basics
    def n_ctx(self) -> int:
        return self._n_ctx

    def n_vocab(self) -> int:
        return self.hparams.n_vocab

    def tokenize(self, text: Union[bytes, str], add_bos: bool = True, special: bool = False) -> List[int]:
        if isinstance(text, bytes):
            text = text.decode("utf-8", errors="replace")
        return self.tokenizer.encode(text, add_bos=add_bos, special=special)

    def detokenize(self, tokens: Sequence[int], special: bool = False) -> bytes:
        return self.tokenizer.detokenize_bytes(tokens, special)

    def health(self) -> Dict[str, Any]:
        h = {"ok": True, "backend": self.backend_name, "model": os.path.basename(self.model_path)}
        bh = getattr(self._backend, "health", None)
        if bh:
            h.update(bh())
        return h

    def device_memory(self) -> Dict[str, int]:
        f = getattr(self._backend, "device_memory", None)
        return f() if f else {}

    def reset(self):
        self._kv_tokens = []

    def close(self):
        c = getattr(self._backend, "close", None)
        if c:
            c()

    # ------------------------------------------------------------ generation
    def _generate(self, prompt_tokens: List[int], max_tokens: Optional[int], params: SamplingParams,
                  stop: List[str], cancel_event: Optional[threading.Event], on_token=None):
        n_prompt = len(prompt_tokens)
        if n_prompt >= self._n_ctx:
            raise ValueError(f"Requested tokens ({n_prompt}) exceed context window of {self._n_ctx}")
        if max_tokens is None or max_tokens <= 0:
            max_tokens = self._n_ctx - n_prompt
        if max_tokens + n_prompt >= self._n_ctx:
            max_tokens = self._n_ctx - n_prompt
        # special-token stop strings become stop ids; the rest are matched on text
        stop_ids = set(self.tokenizer.eog_ids)
        text_stops = []
        for s in stop:
            tid = self.tokenizer._special_map.get(s) if hasattr(self.tokenizer, "_special_map") else None
            if tid is not None:
                stop_ids.add(tid)
            elif s:
                text_stops.append(s)
        # KV prefix reuse (must re-evaluate at least one prompt token for logits)
        n_keep = 0
        for a, b in zip(self._kv_tokens, prompt_tokens):
            if a != b:
                break
            n_keep += 1
        n_keep = min(n_keep, n_prompt - 1)
        poll = cancel_event.is_set if cancel_event is not None else None
        with self._lock:
            res: GenerationResult = self._backend.generate(prompt_tokens, n_keep, max_tokens, params,
                                                           sorted(stop_ids), poll=poll, on_token=on_token)
            hist = list(prompt_tokens) + list(res.tokens)
            self._kv_tokens = hist[:res.n_evaluated]
        toks = list(res.tokens)
        reason = res.finish_reason
        if toks and toks[-1] in stop_ids:
            toks = toks[:-1]
            reason = "stop"
        text = self.detokenize(toks).decode("utf-8", errors="replace")
        for s in text_stops:
            i = text.find(s)
            if i >= 0:
                text = text[:i]
                reason = "stop"
        return text, toks, reason, res

    def _params(self, temperature, top_p, top_k, min_p, typical_p, tfs_z, repeat_penalty,
                frequency_penalty, presence_penalty, seed) -> SamplingParams:
        if seed is None:
            self._n_requests += 1
            seed = (self._seed * 1000003 + self._n_requests) & 0xFFFFFFFF
        return SamplingParams(temperature=temperature, top_k=top_k, top_p=top_p, min_p=min_p,
                              typical_p=typical_p, tfs_z=tfs_z, repeat_penalty=repeat_penalty,
                              frequency_penalty=frequency_penalty, presence_penalty=presence_penalty,
                              last_n=self.last_n_tokens_size, seed=int(seed))

    def create_completion(self, prompt: Union[str, List[int]], max_tokens: Optional[int] = 16,
                          temperature: float = 0.8, top_p: float = 0.95, min_p: float = 0.05,
                          typical_p: float = 1.0, stop: Optional[Union[str, List[str]]] = None,
                          frequency_penalty: float = 0.0, presence_penalty: float = 0.0,
                          repeat_penalty: float = 1.1, top_k: int = 40, stream: bool = False,
                          seed: Optional[int] = None, tfs_z: float = 1.0,
                          cancel_event: Optional[threading.Event] = None, add_bos: bool = True,
                          **unused) -> Union[Dict[str, Any], Iterator[Dict[str, Any]]]:
        if isinstance(prompt, str):
            tokens = self.tokenize(prompt, add_bos=add_bos, special=True)
        else:
            tokens = list(prompt)
        stops = [stop] if isinstance(stop, str) else list(stop or [])
        params = self._params(temperature, top_p, top_k, min_p, typical_p, tfs_z, repeat_penalty,
                              frequency_penalty, presence_penalty, seed)
        cid = f"cmpl-{uuid.uuid4()}"
        if stream:
            return self._stream(cid, tokens, max_tokens, params, stops, cancel_event)
        text, toks, reason, res = self._generate(tokens, max_tokens, params, stops, cancel_event)
        return {"id": cid, "object": "text_completion", "created": int(time.time()),
                "model": self.model_path,
                "choices": [{"text": text, "index": 0, "logprobs": None, "finish_reason": reason}],
                "usage": {"prompt_tokens": len(tokens), "completion_tokens": len(res.tokens),
                          "total_tokens": len(tokens) + len(res.tokens)},
                "timings": {"prefill_s": res.prefill_s, "decode_s": res.decode_s,
                            "n_prefilled": res.n_prefilled}}

    def _stream(self, cid, tokens, max_tokens, params, stops, cancel_event):
        import queue as _q
        q: "_q.Queue" = _q.Queue()
        done = object()
        box = {}

        def run():
            try:
                box["r"] = self._generate(tokens, max_tokens, params, stops, cancel_event,
                                          on_token=lambda t: q.put(t))
            except BaseException as e:  # surfaced to the consumer
                box["e"] = e
            q.put(done)
        th = threading.Thread(target=run, daemon=True)
        th.start()
        pending: List[int] = []
        emitted = ""
        while True:
            t = q.get()
            if t is done:
                break
            if t in self.tokenizer.eog_ids:
                continue
            pending.append(t)
            text = self.detokenize(pending).decode("utf-8", errors="ignore")
            if text and not text.endswith("�"):
                emitted += text
                pending = []
                yield {"id": cid, "object": "text_completion", "created": int(time.time()),
                       "model": self.model_path,
                       "choices": [{"text": text, "index": 0, "logprobs": None, "finish_reason": None}]}
        th.join()
        if "e" in box:
            raise box["e"]
        _, _, reason, _ = box["r"]
        yield {"id": cid, "object": "text_completion", "created": int(time.time()), "model": self.model_path,
               "choices": [{"text": "", "index": 0, "logprobs": None, "finish_reason": reason}]}

    def create_chat_completion(self, messages: List[Dict[str, str]], temperature: float = 0.2,
                               top_p: float = 0.95, top_k: int = 40, min_p: float = 0.05,
                               typical_p: float = 1.0, stream: bool = False,
                               stop: Optional[Union[str, List[str]]] = None, seed: Optional[int] = None,
                               max_tokens: Optional[int] = None, presence_penalty: float = 0.0,
                               frequency_penalty: float = 0.0, repeat_penalty: float = 1.1,
                               tfs_z: float = 1.0, cancel_event: Optional[threading.Event] = None,
                               **unused):
        fr = self._formatter(messages)
        stops = [stop] if isinstance(stop, str) else list(stop or [])
        if fr.stop:
            stops += [fr.stop] if isinstance(fr.stop, str) else list(fr.stop)
        tokens = self.tokenize(fr.prompt, add_bos=not fr.added_special, special=True)
        params = self._params(temperature, top_p, top_k, min_p, typical_p, tfs_z, repeat_penalty,
                              frequency_penalty, presence_penalty, seed)
        cid = f"chatcmpl-{uuid.uuid4()}"
        if stream:
            def gen():
                first = True
                for chunk in self._stream(cid, tokens, max_tokens, params, stops, cancel_event):
                    c = chunk["choices"][0]
                    delta = {"role": "assistant"} if first else {}
                    first = False
                    if c["text"]:
                        delta["content"] = c["text"]
                    yield {"id": cid, "object": "chat.completion.chunk", "created": chunk["created"],
                           "model": self.model_path,
                           "choices": [{"index": 0, "delta": delta, "finish_reason": c["finish_reason"]}]}
            return gen()
        text, toks, reason, res = self._generate(tokens, max_tokens, params, stops, cancel_event)
        return {"id": cid, "object": "chat.completion", "created": int(time.time()), "model": self.model_path,
                "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                             "logprobs": None, "finish_reason": reason}],
                "usage": {"prompt_tokens": len(tokens), "completion_tokens": len(res.tokens),
                          "total_tokens": len(tokens) + len(res.tokens)},
                "timings": {"prefill_s": res.prefill_s, "decode_s": res.decode_s,
                            "n_prefilled": res.n_prefilled}}
