"""Typed service/engine settings read from the environment.

Defaults reproduce the reference exactly:
  * model path ``models/<file>``                       (reference api.py:13-15)
  * MAX_CONTEXT_TOKENS=1024, TIMEOUT_SECONDS=25,
    MAX_QUEUE_SIZE=5                                   (reference api.py:17-19)
  * Llama(n_gpu_layers=-1, n_ctx=1024)                 (reference api.py:24-28)
  * sampling temperature=1.2, top_p=0.9,
    frequency_penalty=0.7, presence_penalty=0.8        (reference api.py:55-63)

Unlike the reference (which hard-codes the model file in two places that
disagree: api.py:14 vs helm deployment.yaml:32) the model
location is ONE value (``MODEL_DIR`` + ``MODEL_FILE`` or ``MODEL_PATH``) that the
Helm chart renders into both the initContainer and the app container.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, fields
from typing import List, Optional

DEFAULT_MODEL_DIR = "models"
DEFAULT_MODEL_FILE = "Lexi-Llama-3-8B-Uncensored_Q4_K_M.gguf"


def _env(name: str, default, cast=str):
    raw = os.environ.get(name)
    if raw is None or raw == "":
        return default
    if cast is bool:
        return raw.strip().lower() in ("1", "true", "yes", "on")
    if cast is list:
        return [float(v) for v in raw.replace(";", ",").split(",") if v.strip()]
    return cast(raw)


@dataclass
class SamplingDefaults:
    """Sampling used by the /response route (reference api.py:55-63) plus the
    llama-cpp-python 0.2.77 defaults it inherits."""
    temperature: float = 1.2
    top_p: float = 0.9
    frequency_penalty: float = 0.7
    presence_penalty: float = 0.8
    top_k: int = 40
    min_p: float = 0.05
    typical_p: float = 1.0
    tfs_z: float = 1.0
    repeat_penalty: float = 1.1
    last_n_tokens: int = 64
    max_tokens: Optional[int] = None  # None => n_ctx - n_prompt (reference leaves it unset)
    seed: Optional[int] = None


@dataclass
class Settings:
    # --- model / engine (reference api.py:13-15, 24-28) ---
    model_dir: str = DEFAULT_MODEL_DIR
    model_file: str = DEFAULT_MODEL_FILE
    model_path_override: Optional[str] = None
    n_gpu_layers: int = -1
    n_ctx: int = 1024
    n_batch: int = 512
    tensor_split: Optional[List[float]] = None
    split_mode: str = "layer"  # none | layer | row  (row => tensor parallel over RCCL)
    main_gpu: int = 0
    seed: Optional[int] = None
    use_graphs: bool = True
    chat_format: Optional[str] = None
    engine: str = "native"  # native | fake
    verbose: bool = False
    # continuous batching (MI355X engine, one rank): up to max_batch generations decode
    # together as rows of one batched step. 1 = the reference's one-at-a-time serving.
    max_batch: int = 1
    # tensor parallelism (split_mode=row over torchrun ranks): the engine's collectives -
    # "auto" (one-shot P2P kernel for decode, RCCL for prefill), "rccl", or "ipc" (the P2P
    # kernel only: ranks may share a GPU). tp_device puts EVERY rank on that GPU (the one-GPU
    # rehearsal of an N-rank deployment; None = the rank's LOCAL_RANK GPU)
    tp_comm: str = "auto"
    tp_device: Optional[int] = None
    # --- service (reference api.py:17-19) ---
    max_context_tokens: int = 1024
    timeout_seconds: float = 25.0
    max_queue_size: int = 5
    # requests admitted at once (in flight + waiting); the next one gets 503. None = the reference's
    # capacity, max_queue_size + 1 (1 in flight + 5 queued, reference api.py:19,113,156-160), whatever
    # max_batch is: with max_batch = 6 all six admitted requests decode together. 0 = the uncapped
    # form (max_batch in flight + max_queue_size waiting)
    max_admitted: Optional[int] = None
    message_char_cap: int = 400        # reference api.py:36-39
    # True: the reference's prompt heuristics exactly (the 400-char cap applies to the system
    # message too, C6). False: system messages keep their full text.
    parity_mode: bool = True
    # after the char/4 trim, drop oldest messages by REAL token count so the
    # prompt stays below n_ctx - exact_token_reserve (no 500 on token-dense text)
    exact_token_guard: bool = False
    exact_token_reserve: int = 32       # tokens kept free for the answer under the guard
    cooperative_cancel: bool = True     # stop timed-out generations
    openai_api: bool = True             # /v1/models, /v1/completions, /v1/chat/completions
    sampling: SamplingDefaults = field(default_factory=SamplingDefaults)

    @property
    def admission_cap(self) -> int:
        """Requests admitted at once (in flight + queued), 0 = no cap beyond the queue's."""
        if self.max_admitted is None:
            return self.max_queue_size + 1
        return max(0, int(self.max_admitted))

    @property
    def model_path(self) -> str:
        if self.model_path_override:
            return self.model_path_override
        return f"{self.model_dir}/{self.model_file}"

    @classmethod
    def from_env(cls) -> "Settings":
        s = cls()
        s.model_dir = _env("MODEL_DIR", s.model_dir)
        s.model_file = _env("MODEL_FILE", s.model_file)
        s.model_path_override = _env("MODEL_PATH", None)
        s.n_gpu_layers = _env("N_GPU_LAYERS", s.n_gpu_layers, int)
        s.n_ctx = _env("N_CTX", s.n_ctx, int)
        s.n_batch = _env("N_BATCH", s.n_batch, int)
        s.tensor_split = _env("TENSOR_SPLIT", None, list)
        s.split_mode = _env("SPLIT_MODE", s.split_mode).lower()
        s.main_gpu = _env("MAIN_GPU", s.main_gpu, int)
        seed = _env("SEED", None)
        s.seed = int(seed) if seed is not None else None
        s.use_graphs = _env("USE_GRAPHS", s.use_graphs, bool)
        s.chat_format = _env("CHAT_FORMAT", None)
        s.engine = _env("ENGINE", s.engine).lower()
        s.verbose = _env("VERBOSE", s.verbose, bool)
        s.max_batch = max(1, _env("MAX_BATCH", s.max_batch, int))
        s.tp_comm = _env("TP_COMM", s.tp_comm).lower()
        tpd = _env("TP_DEVICE", None)
        s.tp_device = int(tpd) if tpd is not None else None
        s.max_context_tokens = _env("MAX_CONTEXT_TOKENS", s.max_context_tokens, int)
        s.timeout_seconds = _env("TIMEOUT_SECONDS", s.timeout_seconds, float)
        s.max_queue_size = _env("MAX_QUEUE_SIZE", s.max_queue_size, int)
        adm = _env("MAX_ADMITTED", None)
        s.max_admitted = int(adm) if adm is not None else None
        s.message_char_cap = _env("MESSAGE_CHAR_CAP", s.message_char_cap, int)
        s.parity_mode = _env("PARITY_MODE", s.parity_mode, bool)
        s.exact_token_guard = _env("EXACT_TOKEN_GUARD", s.exact_token_guard, bool)
        s.exact_token_reserve = max(1, _env("EXACT_TOKEN_RESERVE", s.exact_token_reserve, int))
        s.cooperative_cancel = _env("COOPERATIVE_CANCEL", s.cooperative_cancel, bool)
        s.openai_api = _env("OPENAI_API", s.openai_api, bool)
        sp = s.sampling
        for f in fields(SamplingDefaults):
            key = "SAMPLING_" + f.name.upper()
            if key in os.environ:
                cur = getattr(sp, f.name)
                cast = type(cur) if cur is not None else (int if f.name in ("max_tokens", "seed") else float)
                setattr(sp, f.name, _env(key, cur, cast))
        return s
