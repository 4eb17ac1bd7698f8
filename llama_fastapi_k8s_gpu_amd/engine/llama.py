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

import itertools
import logging
import os
import threading
import time
import uuid
from typing import Any, Dict, Iterator, List, Optional, Sequence, Union

import numpy as np

from ..gguf.reader import GGUFReader
from ..models.llama import LlamaHParams
from .backends import GenerationResult, ReferenceBackend
from .cache import BaseLlamaCache, LlamaState, longest_token_prefix
from .chat_format import get_formatter
from .sampling import SamplingParams
from .tokenizer import tokenizer_from_metadata

logger = logging.getLogger(__name__)


def _layer_split(split_mode: str, tensor_split) -> bool:
    """upstream's multi-GPU layer placement: split_mode LAYER with weights on >1 GPUs"""
    return split_mode == "layer" and bool(tensor_split) and sum(1 for v in tensor_split if float(v) > 0) > 1


def _select_backend(reader, hp: LlamaHParams, n_gpu_layers: int, backend: Optional[str],
                    split_mode: str = "layer", tensor_split=None) -> str:
    if backend:
        return backend
    env = os.environ.get("LLAMA_BACKEND")
    if env:
        return env
    n_gpu = hp.n_layer + 1 if n_gpu_layers < 0 else n_gpu_layers
    if n_gpu == 0:
        return "cpu"
    # ask the runtime that will run the model (the _hip extension's HIP runtime): torch may
    # bundle a different HIP runtime that reports no device once ours initialised the GPU
    try:
        from ..runtime import load_hip
        if load_hip().device_count() > 0:
            if n_gpu < hp.n_layer:
                return "hybrid"
            return "layer" if _layer_split(split_mode, tensor_split) else "hip"
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
        self._request_ids = itertools.count(1)   # per-request seed derivation (thread-safe)
        self._lock = threading.Lock()
        self._gvocab_lock = threading.Lock()
        bos = self.tokenizer.tokens[self.tokenizer.bos_id] if self.tokenizer.bos_id >= 0 else ""
        eos = self.tokenizer.tokens[self.tokenizer.eos_id] if self.tokenizer.eos_id >= 0 else ""
        self.chat_format, self._formatter = get_formatter(self.metadata, chat_format, bos, eos)
        kind = _select_backend(reader, self.hparams, n_gpu_layers, backend, split_mode, tensor_split)
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
        elif kind == "layer":
            from ..runtime.layer_split_backend import LayerSplitBackend
            if int(kwargs.get("max_batch", 1) or 1) > 1:
                raise ValueError("split_mode='layer' across GPUs runs one generation at a time: max_batch > 1 "
                                 "needs split_mode='row' (tensor parallelism) or a single GPU")
            if main_gpu != 0:
                logger.warning("split_mode='layer': main_gpu=%d is ignored (stage i runs on device i)", main_gpu)
            self._backend = LayerSplitBackend(model_path, self.hparams, tensor_split=tensor_split or [1.0],
                                              n_ctx=self._n_ctx, n_batch=n_batch,
                                              layer_devices=kwargs.get("layer_devices"))
        elif kind == "hip":
            from ..runtime.hip_backend import HipBackend
            self._backend = HipBackend(model_path, self.hparams, n_ctx=self._n_ctx, n_gpu_layers=n_gpu_layers,
                                       tensor_split=tensor_split, split_mode=split_mode, main_gpu=main_gpu,
                                       n_batch=n_batch, use_graphs=use_graphs, **kwargs)
        else:
            raise ValueError(f"unknown backend {kind!r}")
        del reader
        self._kv_tokens: List[int] = []   # tokens resident in the KV cache (prefix reuse)
        self.cache: Optional[BaseLlamaCache] = None
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

    def count_chat_tokens(self, messages: List[Dict[str, str]]) -> int:
        """Prompt tokens create_chat_completion would evaluate for these messages."""
        fr = self._formatter(messages)
        return len(self.tokenize(fr.prompt, add_bos=not fr.added_special, special=True))

    def detokenize(self, tokens: Sequence[int], special: bool = False) -> bytes:
        return self.tokenizer.detokenize_bytes(tokens, special)

    def health(self) -> Dict[str, Any]:
        h = {"ok": True, "backend": self.backend_name, "model": os.path.basename(self.model_path)}
        bh = getattr(self._backend, "health", None)
        if bh:
            h.update(bh())
        return h

    @property
    def batch_width(self) -> int:
        """Generations the backend runs at once (its continuous batch; 1 without a scheduler)."""
        if getattr(self._backend, "sched", None) is not None:
            return max(1, int(getattr(self._backend, "max_batch", 1)))
        return 1

    @property
    def follows(self) -> bool:
        """This process is a follower rank of a tensor-parallel group (see follow())."""
        return bool(getattr(self._backend, "follows", False))

    def follow(self):
        """Follower ranks: replay rank 0's engine commands until rank 0 closes the group."""
        self._backend.follow()

    def device_memory(self) -> Dict[str, int]:
        f = getattr(self._backend, "device_memory", None)
        return f() if f else {}

    def reset(self):
        self._kv_tokens = []

    # ------------------------------------------------------------ states / caches
    def set_cache(self, cache: Optional[BaseLlamaCache]):
        self.cache = cache

    def _save_state(self, on_device: bool = False) -> LlamaState:
        n = len(self._kv_tokens)
        kv = self._backend.save_kv(n, on_device)
        if hasattr(kv, "nbytes"):
            size = int(kv.nbytes)
        elif hasattr(kv, "numel"):
            size = int(kv.numel() * kv.element_size())
        else:
            size = sum(int(getattr(x, "nbytes", 0) or x.numel() * x.element_size()) for x in kv)
        return LlamaState(np.asarray(self._kv_tokens, np.int32), None, n, kv, size, self._seed)

    def _load_state(self, state: LlamaState):
        self._backend.load_kv(state.llama_state, state.n_tokens)
        self._kv_tokens = [int(t) for t in state.input_ids[:state.n_tokens]]

    def save_state(self, on_device: bool = False) -> LlamaState:
        """Snapshot of the KV cache and its tokens (``on_device``: kept in GPU memory)."""
        with self._lock:
            return self._save_state(on_device)

    def load_state(self, state: LlamaState):
        with self._lock:
            self._load_state(state)

    def close(self):
        c = getattr(self._backend, "close", None)
        if c:
            c()

    # ------------------------------------------------------------ generation
    def _text_stops(self, stop: List[str]):
        """Special-token stop strings become stop ids; the rest are matched on text."""
        stop_ids = set(self.tokenizer.eog_ids)
        text_stops = []
        for s in stop:
            tid = self.tokenizer._special_map.get(s) if hasattr(self.tokenizer, "_special_map") else None
            if tid is not None:
                stop_ids.add(tid)
            elif s:
                text_stops.append(s)
        return stop_ids, text_stops

    def _generate(self, prompt_tokens: List[int], max_tokens: Optional[int], params: SamplingParams,
                  stop: List[str], cancel_event: Optional[threading.Event], on_token=None,
                  stopping_criteria=None):
        n_prompt = len(prompt_tokens)
        if n_prompt >= self._n_ctx:
            raise ValueError(f"Requested tokens ({n_prompt}) exceed context window of {self._n_ctx}")
        if max_tokens is None or max_tokens <= 0:
            max_tokens = self._n_ctx - n_prompt
        if max_tokens + n_prompt >= self._n_ctx:
            max_tokens = self._n_ctx - n_prompt
        stop_ids, text_stops = self._text_stops(stop)
        batches = getattr(self._backend, "batches", None)
        if batches is not None and batches(params):
            # a row of the backend's continuous batch: no facade lock (requests run
            # concurrently) and no facade KV bookkeeping (the scheduler reuses prefixes per slot)
            return self._generate_locked(prompt_tokens, max_tokens, params, stop_ids, text_stops, cancel_event,
                                         on_token, stopping_criteria, track_kv=False)
        self._lock.acquire()
        try:
            if self.cache is not None:   # restore a cached state that shares more of the prompt
                try:
                    item = self.cache[prompt_tokens]
                    if longest_token_prefix(item.input_ids.tolist(), prompt_tokens) > \
                            longest_token_prefix(self._kv_tokens, prompt_tokens):
                        self._load_state(item)
                except KeyError:
                    pass
            return self._generate_locked(prompt_tokens, max_tokens, params, stop_ids, text_stops, cancel_event,
                                         on_token, stopping_criteria)
        finally:
            self._lock.release()

    def _generate_locked(self, prompt_tokens, max_tokens, params, stop_ids, text_stops, cancel_event, on_token,
                         stopping_criteria, track_kv: bool = True):
        n_prompt = len(prompt_tokens)
        # KV prefix reuse (must re-evaluate at least one prompt token for logits)
        n_keep = min(longest_token_prefix(self._kv_tokens, prompt_tokens), n_prompt - 1) if track_kv else 0
        # upstream stops as soon as a stop string appears in the generated text (or a
        # stopping criterion fires): watch the token stream and end the backend's loop
        # through its cancel poll
        hit = {"stop": False}
        stops_b = [s.encode("utf-8") for s in text_stops]
        maxlen = max((len(b) for b in stops_b), default=0)
        buf = bytearray()
        gen: List[int] = []

        def watch(t: int):
            gen.append(t)
            if stops_b and t not in stop_ids:
                piece = self.tokenizer.detokenize_bytes([t], False)
                buf.extend(piece)
                region = bytes(buf[max(0, len(buf) - len(piece) - maxlen + 1):])
                if any(b in region for b in stops_b):
                    hit["stop"] = True
            if stopping_criteria is not None and not hit["stop"]:
                import numpy as np
                if stopping_criteria(np.asarray(list(prompt_tokens) + gen, np.int64), None):
                    hit["stop"] = True
            if on_token:
                on_token(t)

        def poll():
            return hit["stop"] or (cancel_event is not None and cancel_event.is_set())
        watched = bool(stops_b) or stopping_criteria is not None
        res: GenerationResult = self._backend.generate(
            prompt_tokens, n_keep, max_tokens, params, sorted(stop_ids),
            poll=poll if (watched or cancel_event is not None) else None,
            on_token=watch if (watched or on_token) else None)
        if track_kv:
            hist = list(prompt_tokens) + list(res.tokens)
            self._kv_tokens = hist[:res.n_evaluated]
            if self.cache is not None and self._kv_tokens:
                self.cache[tuple(self._kv_tokens)] = self._save_state(self.cache.on_device)
        toks = list(res.tokens)
        reason = res.finish_reason
        if toks and toks[-1] in stop_ids:
            toks = toks[:-1]
            reason = "stop"
        if hit["stop"] and reason == "cancelled":
            reason = "stop"
        text = self.detokenize(toks).decode("utf-8", errors="replace")
        cut = min((i for i in (text.find(s) for s in text_stops) if i >= 0), default=-1)
        if cut >= 0:
            text = text[:cut]
            reason = "stop"
        return text, toks, reason, res

    def _params(self, temperature, top_p, top_k, min_p, typical_p, tfs_z, repeat_penalty,
                frequency_penalty, presence_penalty, seed, logit_bias=None, mirostat_mode=0,
                mirostat_tau=5.0, mirostat_eta=0.1, n_probs=0, logits_processor=None,
                grammar=None) -> SamplingParams:
        if seed is None:
            seed = (self._seed * 1000003 + next(self._request_ids)) & 0xFFFFFFFF
        bias = {int(k): float(v) for k, v in (logit_bias or {}).items()}
        return SamplingParams(temperature=temperature, top_k=top_k, top_p=top_p, min_p=min_p,
                              typical_p=typical_p, tfs_z=tfs_z, repeat_penalty=repeat_penalty,
                              frequency_penalty=frequency_penalty, presence_penalty=presence_penalty,
                              last_n=self.last_n_tokens_size, seed=int(seed), logit_bias=bias,
                              mirostat_mode=int(mirostat_mode or 0), mirostat_tau=float(mirostat_tau),
                              mirostat_eta=float(mirostat_eta), n_probs=int(n_probs or 0),
                              logits_processor=logits_processor, grammar=self._grammar_state(grammar))

    def _grammar_state(self, grammar):
        """A per-request matcher for ``grammar`` (LlamaGrammar or GBNF text), or None."""
        if grammar is None:
            return None
        from .grammar import GrammarState, GrammarVocab, LlamaGrammar
        if isinstance(grammar, str):
            grammar = LlamaGrammar.from_string(grammar)
        with self._gvocab_lock:   # concurrent batched requests may build it at once
            if getattr(self, "_gvocab", None) is None:
                n = self.n_vocab()
                self._gvocab = GrammarVocab([self.tokenizer.detokenize_bytes([t], False) for t in range(n)],
                                            self.tokenizer.eog_ids)
        return GrammarState(grammar, self._gvocab)

    @staticmethod
    def _response_format_grammar(response_format):
        """OpenAI ``response_format`` -> grammar: json_object (optionally with ``schema``,
        llama-cpp-python's extension) or json_schema ({"json_schema": {"schema": ...}})."""
        if not response_format:
            return None
        from .grammar import JSON_GBNF, LlamaGrammar
        kind = response_format.get("type", "text")
        if kind == "text":
            return None
        if kind == "json_object":
            schema = response_format.get("schema")
            return LlamaGrammar.from_json_schema(schema) if schema else LlamaGrammar.from_string(JSON_GBNF)
        if kind == "json_schema":
            js = response_format.get("json_schema") or {}
            schema = js.get("schema", js) if isinstance(js, dict) else js
            return LlamaGrammar.from_json_schema(schema)
        raise ValueError(f"unsupported response_format type {kind!r}")

    @staticmethod
    def logits_to_logprobs(logits, axis: int = -1):
        """Natural-log softmax (``llama_cpp.Llama.logits_to_logprobs``)."""
        import numpy as np
        l = np.asarray(logits, np.float32)
        m = np.max(l, axis=axis, keepdims=True)
        return (l - m - np.log(np.sum(np.exp(l - m), axis=axis, keepdims=True))).astype(np.float32)

    def _piece(self, t: int) -> str:
        return self.detokenize([t]).decode("utf-8", errors="ignore")

    def _completion_logprobs(self, prompt_tokens: List[int], toks: List[int], res: GenerationResult, echo: bool,
                             prompt_text: str):
        """The OpenAI / llama-cpp-python ``logprobs`` block. Generated tokens carry the
        log-probabilities of the raw model logits; echoed prompt tokens carry None (the
        engine keeps only the last prompt position's logits - upstream needs
        ``logits_all=True`` for those)."""
        entries = list(res.logprobs or [])[:len(toks)]
        all_toks = (list(prompt_tokens) if echo else []) + list(toks)
        strs = [self._piece(t) for t in all_toks]
        offset = 0 if echo else len(prompt_text)
        out = {"tokens": [], "text_offset": [], "token_logprobs": [], "top_logprobs": []}
        n_echo = len(all_toks) - len(toks)
        run = 0
        for i, (t, ts) in enumerate(zip(all_toks, strs)):
            if echo and i == 0 and t == self.tokenizer.bos_id:
                continue
            out["tokens"].append(ts)
            out["text_offset"].append(offset + run)
            run += len(ts)
            if i < n_echo:
                out["token_logprobs"].append(None)
                out["top_logprobs"].append(None)
                continue
            lp, top = entries[i - n_echo] if i - n_echo < len(entries) else (None, [])
            out["token_logprobs"].append(lp)
            d = {self._piece(j): v for j, v in top}
            if lp is not None:
                d[ts] = lp
            out["top_logprobs"].append(d)
        return out

    def create_completion(self, prompt: Union[str, List[int]], suffix: Optional[str] = None,
                          max_tokens: Optional[int] = 16, temperature: float = 0.8, top_p: float = 0.95,
                          min_p: float = 0.05, typical_p: float = 1.0, logprobs: Optional[int] = None,
                          echo: bool = False, stop: Optional[Union[str, List[str]]] = None,
                          frequency_penalty: float = 0.0, presence_penalty: float = 0.0,
                          repeat_penalty: float = 1.1, top_k: int = 40, stream: bool = False,
                          seed: Optional[int] = None, tfs_z: float = 1.0, mirostat_mode: int = 0,
                          mirostat_tau: float = 5.0, mirostat_eta: float = 0.1, model: Optional[str] = None,
                          stopping_criteria=None, logits_processor=None, grammar=None,
                          logit_bias: Optional[Dict[int, float]] = None,
                          cancel_event: Optional[threading.Event] = None, add_bos: bool = True,
                          **unused) -> Union[Dict[str, Any], Iterator[Dict[str, Any]]]:
        if suffix:
            raise NotImplementedError("infill (suffix) is not supported by this engine")
        if isinstance(prompt, str):
            prompt_text = prompt
            tokens = self.tokenize(prompt, add_bos=add_bos, special=True)
        else:
            tokens = list(prompt)
            prompt_text = self.detokenize(tokens).decode("utf-8", errors="replace")
        stops = [stop] if isinstance(stop, str) else list(stop or [])
        params = self._params(temperature, top_p, top_k, min_p, typical_p, tfs_z, repeat_penalty,
                              frequency_penalty, presence_penalty, seed, logit_bias, mirostat_mode,
                              mirostat_tau, mirostat_eta, logprobs, logits_processor, grammar)
        cid = f"cmpl-{uuid.uuid4()}"
        mname = model or self.model_path
        if stream:
            return self._stream(cid, tokens, max_tokens, params, stops, cancel_event, mname,
                                echo_text=prompt_text if echo else None, stopping_criteria=stopping_criteria)
        text, toks, reason, res = self._generate(tokens, max_tokens, params, stops, cancel_event,
                                                 stopping_criteria=stopping_criteria)
        lp = self._completion_logprobs(tokens, toks, res, echo, prompt_text) if params.n_probs > 0 else None
        return {"id": cid, "object": "text_completion", "created": int(time.time()),
                "model": mname,
                "choices": [{"text": (prompt_text + text) if echo else text, "index": 0, "logprobs": lp,
                             "finish_reason": reason}],
                "usage": {"prompt_tokens": len(tokens), "completion_tokens": len(res.tokens),
                          "total_tokens": len(tokens) + len(res.tokens)},
                "timings": {"prefill_s": res.prefill_s, "decode_s": res.decode_s,
                            "n_prefilled": res.n_prefilled}}

    __call__ = create_completion

    def _stream(self, cid, tokens, max_tokens, params, stops, cancel_event, mname=None, echo_text=None,
                stopping_criteria=None):
        """Chunks as tokens arrive. Text that could still become a stop string is held
        back until it cannot (upstream behaviour); a stop string ends the stream and
        the generation."""
        import queue as _q
        mname = mname or self.model_path
        q: "_q.Queue" = _q.Queue()
        done = object()
        box = {}
        stop_now = threading.Event()
        ev = _AnyEvent(cancel_event, stop_now)
        lps: List[Any] = []
        if params.n_probs > 0:
            params.logprob_cb = lps.append

        def run():
            try:
                box["r"] = self._generate(tokens, max_tokens, params, stops, ev, on_token=lambda t: q.put(t),
                                          stopping_criteria=stopping_criteria)
            except BaseException as e:  # surfaced to the consumer
                box["e"] = e
            q.put(done)
        th = threading.Thread(target=run, daemon=True)
        th.start()
        _, text_stops = self._text_stops(stops)

        def chunk(text, reason=None, lp=None):
            return {"id": cid, "object": "text_completion", "created": int(time.time()), "model": mname,
                    "choices": [{"text": text, "index": 0, "logprobs": lp, "finish_reason": reason}]}
        if echo_text:
            yield chunk(echo_text)
        pending: List[int] = []
        text_all, emitted, n_tok = "", 0, 0
        stopped = False
        while True:
            t = q.get()
            if t is done:
                break
            if stopped or t in self.tokenizer.eog_ids:
                continue
            n_tok += 1
            pending.append(t)
            raw = self.detokenize(pending)
            try:
                piece = raw.decode("utf-8")
            except UnicodeDecodeError:      # a multi-byte character split across tokens
                if len(pending) < 4:
                    continue
                piece = raw.decode("utf-8", errors="replace")
            pending = []
            if not piece:
                continue
            text_all += piece
            cut = min((i for i in (text_all.find(s) for s in text_stops) if i >= 0), default=-1)
            if cut >= 0:
                stopped = True
                stop_now.set()
                if cut > emitted:
                    yield chunk(text_all[emitted:cut])
                emitted = cut
                continue
            hold = 0   # longest suffix that is a proper prefix of some stop string
            for s in text_stops:
                for k in range(min(len(s) - 1, len(text_all)), 0, -1):
                    if text_all.endswith(s[:k]):
                        hold = max(hold, k)
                        break
            safe = len(text_all) - hold
            if safe > emitted:
                lp = None
                if params.n_probs > 0 and n_tok <= len(lps):
                    l, top = lps[n_tok - 1]
                    lp = {"tokens": [piece], "text_offset": [emitted], "token_logprobs": [l],
                          "top_logprobs": [{self._piece(j): v for j, v in top}]}
                yield chunk(text_all[emitted:safe], lp=lp)
                emitted = safe
        th.join()
        if "e" in box:
            raise box["e"]
        _, _, reason, _ = box["r"]
        if stopped:
            reason = "stop"
        elif emitted < len(text_all):
            yield chunk(text_all[emitted:])
        yield chunk("", reason)

    def create_chat_completion(self, messages: List[Dict[str, str]], functions=None, function_call=None,
                               tools=None, tool_choice=None, temperature: float = 0.2,
                               top_p: float = 0.95, top_k: int = 40, min_p: float = 0.05,
                               typical_p: float = 1.0, stream: bool = False,
                               stop: Optional[Union[str, List[str]]] = None, seed: Optional[int] = None,
                               response_format=None, max_tokens: Optional[int] = None,
                               presence_penalty: float = 0.0, frequency_penalty: float = 0.0,
                               repeat_penalty: float = 1.1, tfs_z: float = 1.0, mirostat_mode: int = 0,
                               mirostat_tau: float = 5.0, mirostat_eta: float = 0.1, model: Optional[str] = None,
                               logits_processor=None, grammar=None, logit_bias: Optional[Dict[int, float]] = None,
                               logprobs: Optional[bool] = None, top_logprobs: Optional[int] = None,
                               cancel_event: Optional[threading.Event] = None, **unused):
        if grammar is None:
            grammar = self._response_format_grammar(response_format)
        if functions or tools:
            raise NotImplementedError("function / tool calling needs a chat handler this engine does not ship")
        fr = self._formatter(messages)
        stops = [stop] if isinstance(stop, str) else list(stop or [])
        if fr.stop:
            stops += [fr.stop] if isinstance(fr.stop, str) else list(fr.stop)
        tokens = self.tokenize(fr.prompt, add_bos=not fr.added_special, special=True)
        n_probs = (top_logprobs or 0) if logprobs else 0
        if logprobs and not n_probs:
            n_probs = 1   # the chosen token's log-probability is reported either way
        params = self._params(temperature, top_p, top_k, min_p, typical_p, tfs_z, repeat_penalty,
                              frequency_penalty, presence_penalty, seed, logit_bias, mirostat_mode,
                              mirostat_tau, mirostat_eta, n_probs, logits_processor, grammar)
        cid = f"chatcmpl-{uuid.uuid4()}"
        mname = model or self.model_path
        if stream:
            def gen():
                first = True
                for chunk in self._stream(cid, tokens, max_tokens, params, stops, cancel_event, mname):
                    c = chunk["choices"][0]
                    delta = {"role": "assistant"} if first else {}
                    first = False
                    if c["text"]:
                        delta["content"] = c["text"]
                    yield {"id": cid, "object": "chat.completion.chunk", "created": chunk["created"],
                           "model": mname,
                           "choices": [{"index": 0, "delta": delta, "logprobs": _chat_logprobs(c["logprobs"], top_logprobs),
                                        "finish_reason": c["finish_reason"]}]}
            return gen()
        text, toks, reason, res = self._generate(tokens, max_tokens, params, stops, cancel_event)
        lp = None
        if logprobs:
            lp = _chat_logprobs(self._completion_logprobs(tokens, toks, res, False, ""), top_logprobs)
        return {"id": cid, "object": "chat.completion", "created": int(time.time()), "model": mname,
                "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                             "logprobs": lp, "finish_reason": reason}],
                "usage": {"prompt_tokens": len(tokens), "completion_tokens": len(res.tokens),
                          "total_tokens": len(tokens) + len(res.tokens)},
                "timings": {"prefill_s": res.prefill_s, "decode_s": res.decode_s,
                            "n_prefilled": res.n_prefilled}}


def _chat_logprobs(lp: Optional[Dict[str, Any]], top_n: Optional[int]):
    """Text-completion logprobs -> the chat ``{"content": [...]}`` form."""
    if lp is None:
        return None
    content = []
    for tok, l, top in zip(lp["tokens"], lp["token_logprobs"], lp["top_logprobs"]):
        items = list((top or {}).items())[:max(0, int(top_n or 0))]
        content.append({"token": tok, "bytes": list(tok.encode("utf-8")), "logprob": l,
                        "top_logprobs": [{"token": t, "bytes": list(t.encode("utf-8")), "logprob": v}
                                         for t, v in items]})
    return {"content": content, "refusal": None}


class _AnyEvent:
    """``is_set()`` of either event (caller's cancel, or the stream's stop string)."""

    def __init__(self, a: Optional[threading.Event], b: threading.Event):
        self.a, self.b = a, b

    def is_set(self) -> bool:
        return self.b.is_set() or (self.a is not None and self.a.is_set())
