"""Random-init GGUF models of the BASELINE architectures (no network: real
checkpoints cannot be fetched, so every benchmark and test runs on synthetic
weights of the exact shapes and quant-type mixes - SURVEY §2.3, §7.2).

``SPECS`` holds the BASELINE.json configs plus tiny test models. Tensor types
follow the upstream Q4_K_M mix rule::

    use_more_bits(i, n) = i < n/8 or i >= 7n/8 or (i - n/8) % 3 == 2
    attn_v, ffn_down -> Q6_K when use_more_bits (70B: non-bumped attn_v -> Q5_K)
    8-expert models  -> attn_k/attn_v Q8_0
    output.weight    -> Q6_K ; token_embd -> Q4_K ; norms/router -> F32
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Tuple

import numpy as np

from .constants import (FTYPE_MOSTLY_Q4_K_M, FTYPE_MOSTLY_Q8_0, GGMLType, GGUFValueType,
                        TOKEN_TYPE_BYTE, TOKEN_TYPE_CONTROL, TOKEN_TYPE_NORMAL)
from .quants import random_blocks
from .writer import GGUFWriter

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")

LLAMA3_CHAT_TEMPLATE = (
    "{% set loop_messages = messages %}{% for message in loop_messages %}{% set content = "
    "'<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n'+ message['content'] | trim + "
    "'<|eot_id|>' %}{% if loop.index0 == 0 %}{% set content = bos_token + content %}{% endif %}"
    "{{ content }}{% endfor %}{% if add_generation_prompt %}{{ '<|start_header_id|>assistant"
    "<|end_header_id|>\n\n' }}{% endif %}")
ZEPHYR_CHAT_TEMPLATE = (
    "{% for message in messages %}\n{% if message['role'] == 'user' %}\n{{ '<|user|>\n' + "
    "message['content'] + eos_token }}\n{% elif message['role'] == 'system' %}\n{{ '<|system|>\n' + "
    "message['content'] + eos_token }}\n{% elif message['role'] == 'assistant' %}\n{{ '<|assistant|>\n'"
    "  + message['content'] + eos_token }}\n{% endif %}\n{% if loop.last and add_generation_prompt %}\n"
    "{{ '<|assistant|>' }}\n{% endif %}\n{% endfor %}")
MISTRAL_CHAT_TEMPLATE = (
    "{{ bos_token }}{% for message in messages %}{% if (message['role'] == 'user') != "
    "(loop.index0 % 2 == 0) %}{{ raise_exception('Conversation roles must alternate "
    "user/assistant/user/assistant/...') }}{% endif %}{% if message['role'] == 'user' %}"
    "{{ '[INST] ' + message['content'] + ' [/INST]' }}{% elif message['role'] == 'assistant' %}"
    "{{ message['content'] + eos_token}}{% else %}{{ raise_exception('Only user and assistant "
    "roles are supported!') }}{% endif %}{% endfor %}")

LLAMA3_SPECIALS = {0: "<|begin_of_text|>", 1: "<|end_of_text|>", 6: "<|start_header_id|>",
                   7: "<|end_header_id|>", 9: "<|eot_id|>"}


@dataclass
class ModelSpec:
    name: str
    n_embd: int
    n_layer: int
    n_head: int
    n_head_kv: int
    n_ff: int
    n_vocab: int
    rope_base: float
    tokenizer: str            # "bpe" | "spm"
    quant: str                # "q4_k_m" | "q8_0" | "f32" | "mixed-test"
    n_expert: int = 0
    n_expert_used: int = 0
    n_ctx_train: int = 8192
    rms_eps: float = 1e-5
    size_class: str = "8B"    # "8B" | "70B" (affects the Q4_K_M attn_v rule)
    weight_std: float = 0.02
    chat_template: Optional[str] = None

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head


SPECS: Dict[str, ModelSpec] = {
    "llama3-8b-q4_k_m": ModelSpec("Llama-3-8B", 4096, 32, 32, 8, 14336, 128256, 500000.0, "bpe", "q4_k_m"),
    "llama3-70b-q4_k_m": ModelSpec("Llama-3-70B", 8192, 80, 64, 8, 28672, 128256, 500000.0, "bpe", "q4_k_m",
                                   size_class="70B"),
    "mixtral-8x7b-q4_k_m": ModelSpec("Mixtral-8x7B", 4096, 32, 32, 8, 14336, 32000, 1e6, "spm", "q4_k_m",
                                     n_expert=8, n_expert_used=2, n_ctx_train=32768),
    "tinyllama-1.1b-q8_0": ModelSpec("TinyLlama-1.1B", 2048, 22, 32, 4, 5632, 32000, 10000.0, "spm", "q8_0",
                                     n_ctx_train=2048),
    # --- tiny models for tests (same code paths, seconds to build)
    "tiny-llama3-q4_k_m": ModelSpec("tiny-llama3", 256, 4, 4, 2, 512, 0, 500000.0, "bpe", "q4_k_m",
                                    n_ctx_train=1024),
    "tiny-llama3-mixed": ModelSpec("tiny-llama3-mixed", 256, 4, 4, 2, 512, 0, 500000.0, "bpe", "mixed-test",
                                   n_ctx_train=1024),
    "tiny-tinyllama-q8_0": ModelSpec("tiny-tinyllama", 512, 3, 8, 1, 768, 0, 10000.0, "spm", "q8_0",
                                     n_ctx_train=1024),
    "tiny-mixtral-q4_k_m": ModelSpec("tiny-mixtral", 256, 3, 4, 2, 512, 0, 1e6, "spm", "q4_k_m",
                                     n_expert=4, n_expert_used=2, n_ctx_train=1024),
    # tensor-parallel test shapes: per-rank head / FFN slices stay multiples of 256 at TP=2
    "tiny-llama3-tp": ModelSpec("tiny-llama3-tp", 512, 2, 8, 4, 1024, 0, 500000.0, "bpe", "q4_k_m",
                                n_ctx_train=1024),
    # 4 kv heads of 256 q columns each: uneven tensor_split ratios and TP=3 are representable
    "tiny-llama3-tp4": ModelSpec("tiny-llama3-tp4", 1024, 2, 8, 4, 1024, 0, 500000.0, "bpe", "q4_k_m",
                                 n_ctx_train=1024),
    "tiny-mixtral-tp": ModelSpec("tiny-mixtral-tp", 512, 2, 8, 4, 1024, 0, 1e6, "spm", "q4_k_m",
                                 n_expert=4, n_expert_used=2, n_ctx_train=1024),
    # wide enough for several 2048-feature FFN slices (fused decode FFN hand-off), partial last slice
    "tiny-llama3-wide": ModelSpec("tiny-llama3-wide", 1024, 3, 8, 2, 5120, 0, 500000.0, "bpe", "q4_k_m",
                                  n_ctx_train=1024),
    # Q8_0 with n_ff = 576: 2F = 1152 gate/up rows is NOT a multiple of 256 (the attention
    # weight touch's per-CU gate/up segments must clamp to the plane end)
    "tiny-q8-oddff": ModelSpec("tiny-q8-oddff", 256, 2, 4, 2, 576, 0, 10000.0, "spm", "q8_0",
                               n_ctx_train=1024),
    # one layer: each engine path against the rounding-emulating reference op for op (with more
    # layers, 1e-7 summation-order differences flip q8 / bf16 roundings downstream)
    "tiny-llama3-1l": ModelSpec("tiny-llama3-1l", 256, 1, 4, 2, 512, 0, 500000.0, "bpe", "q4_k_m",
                                n_ctx_train=1024),
    "tiny-mixed-1l": ModelSpec("tiny-mixed-1l", 256, 1, 4, 2, 512, 0, 500000.0, "bpe", "mixed-test",
                               n_ctx_train=1024),
    "tiny-q8-1l": ModelSpec("tiny-q8-1l", 512, 1, 8, 1, 768, 0, 10000.0, "spm", "q8_0", n_ctx_train=1024),
    "tiny-mixtral-1l": ModelSpec("tiny-mixtral-1l", 256, 1, 4, 2, 512, 0, 1e6, "spm", "q4_k_m",
                                 n_expert=4, n_expert_used=2, n_ctx_train=1024),
    # 32 layers (the 8B's depth) at d 1024: the Q4_K_M bump pattern over a full-depth stack
    "tiny-llama3-deep32": ModelSpec("tiny-llama3-deep32", 1024, 32, 8, 2, 512, 0, 500000.0, "bpe", "q4_k_m",
                                    n_ctx_train=1024),
    # d = 4096 with the Llama-3 GQA grouping (32 q heads on 8 kv heads), 4 layers (Q4_K_M mix:
    # layers 0 and 3 bump V/down to Q6_K): full-width kernels at test cost
    "pd-llama-g4": ModelSpec("pd-llama-g4", 4096, 4, 32, 8, 2048, 0, 500000.0, "bpe", "q4_k_m",
                             n_ctx_train=1024),
    # d = 8192 (the 70B's width) in one layer: six rows no longer fit the one-part staging, so the
    # batched step takes the prep (bprep) FFN path beside the split-K Q|K|V
    "tiny-llama3-d8k": ModelSpec("tiny-llama3-d8k", 8192, 1, 64, 8, 512, 0, 500000.0, "bpe", "q4_k_m",
                                 n_ctx_train=1024),
    # Llama-3-70B's layer shape in 2 layers (small vocabulary): the TP = 8 rehearsal's per-rank
    # shapes are the 70B's own (1 KV head, 8 query heads, 3584 FFN features per rank)
    "llama3-70b-2l": ModelSpec("llama3-70b-2l", 8192, 2, 64, 8, 28672, 0, 500000.0, "bpe", "q4_k_m",
                               n_ctx_train=1024, size_class="70B"),
    # Mixtral's width (d = 4096, 8 experts, top-2) in one layer: the single-row decode routes
    # inside the gate/up GEMV at this width (csrc/kernels/gemv.hip, GemvArgs::route_w)
    "tiny-mixtral-d4k": ModelSpec("tiny-mixtral-d4k", 4096, 1, 32, 8, 512, 0, 1e6, "spm", "q4_k_m",
                                  n_expert=8, n_expert_used=2, n_ctx_train=1024),
    "tiny-llama3-f32": ModelSpec("tiny-llama3-f32", 128, 2, 2, 1, 256, 0, 500000.0, "bpe", "f32",
                                 n_ctx_train=512),
}


def use_more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def tensor_types(spec: ModelSpec, layer: int) -> Dict[str, GGMLType]:
    """Per-layer ggml types of the 2-D weights for the spec's quant mix."""
    q = spec.quant
    if q == "q8_0":
        t = GGMLType.Q8_0
        return {k: t for k in ("attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up", "ffn_down")}
    if q == "f32":
        t = GGMLType.F32
        return {k: t for k in ("attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up", "ffn_down")}
    if q == "mixed-test":  # every quant format in one model, to test all kernels end to end
        cyc = [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0]
        names = ("attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_down")
        out = {k: cyc[(layer + j) % 4] for j, k in enumerate(names)}
        out["ffn_up"] = out["ffn_gate"]  # gate/up are one interleaved matrix on the GPU
        return out
    assert q == "q4_k_m"
    n = spec.n_layer
    bump = use_more_bits(layer, n)
    out = {k: GGMLType.Q4_K for k in ("attn_q", "attn_k", "attn_output", "ffn_gate", "ffn_up")}
    if spec.n_expert == 8:
        out["attn_k"] = GGMLType.Q8_0
        out["attn_v"] = GGMLType.Q8_0
    elif bump:
        out["attn_v"] = GGMLType.Q6_K
    else:
        out["attn_v"] = GGMLType.Q5_K if spec.size_class == "70B" else GGMLType.Q4_K
    out["ffn_down"] = GGMLType.Q6_K if bump else GGMLType.Q4_K
    return out


def _load_json(name):
    with open(os.path.join(ASSETS, name), encoding="utf-8") as f:
        return json.load(f)


def build_vocab(spec: ModelSpec) -> Tuple[Dict, int]:
    """Tokenizer metadata + final vocab size."""
    if spec.tokenizer == "bpe":
        v = _load_json("bpe_vocab.json")
        tokens = list(v["tokens"])
        n_regular = (spec.n_vocab - 256) if spec.n_vocab else len(tokens)
        existing = set(tokens)
        i = 0
        while len(tokens) < n_regular:
            cand = f"Ġfill{i}q"
            i += 1
            if cand not in existing:
                tokens.append(cand)
        base = len(tokens)
        types = [TOKEN_TYPE_NORMAL] * base
        for k in range(256):
            name = LLAMA3_SPECIALS.get(k, f"<|reserved_special_token_{k}|>")
            tokens.append(name)
            types.append(TOKEN_TYPE_CONTROL)
        md = {"tokenizer.ggml.model": "gpt2", "tokenizer.ggml.pre": "llama-bpe",
              "tokenizer.ggml.tokens": tokens, "tokenizer.ggml.token_type": types,
              "tokenizer.ggml.merges": v["merges"],
              "tokenizer.ggml.bos_token_id": base + 0, "tokenizer.ggml.eos_token_id": base + 9,
              "tokenizer.chat_template": spec.chat_template or LLAMA3_CHAT_TEMPLATE}
        return md, len(tokens)
    v = _load_json("spm_vocab.json")
    pieces, scores, types = list(v["pieces"]), list(v["scores"]), list(v["types"])
    target = spec.n_vocab or len(pieces)
    existing = set(pieces)
    i = 0
    while len(pieces) < target:
        cand = f"▁fill{i}q"
        i += 1
        if cand not in existing:
            pieces.append(cand)
            scores.append(-1e4 - i)
            types.append(TOKEN_TYPE_NORMAL)
    tmpl = spec.chat_template or (MISTRAL_CHAT_TEMPLATE if spec.n_expert else ZEPHYR_CHAT_TEMPLATE)
    md = {"tokenizer.ggml.model": "llama", "tokenizer.ggml.tokens": pieces,
          "tokenizer.ggml.scores": scores, "tokenizer.ggml.token_type": types,
          "tokenizer.ggml.bos_token_id": 1, "tokenizer.ggml.eos_token_id": 2,
          "tokenizer.ggml.unknown_token_id": 0, "tokenizer.ggml.add_bos_token": True,
          "tokenizer.ggml.add_space_prefix": True, "tokenizer.chat_template": tmpl}
    return md, len(pieces)


def tensor_plan(spec: ModelSpec, n_vocab: int) -> List[Tuple[str, GGMLType, Tuple[int, ...]]]:
    d, f, L = spec.n_embd, spec.n_ff, spec.n_layer
    dkv = spec.head_dim * spec.n_head_kv
    if spec.quant == "q8_0":
        emb_t, out_t = GGMLType.Q8_0, GGMLType.Q8_0
    elif spec.quant == "f32":
        emb_t, out_t = GGMLType.F32, GGMLType.F32
    else:
        emb_t, out_t = GGMLType.Q4_K, GGMLType.Q6_K
    plan = [("token_embd.weight", emb_t, (d, n_vocab))]
    for i in range(L):
        tt = tensor_types(spec, i)
        p = f"blk.{i}."
        plan += [(p + "attn_norm.weight", GGMLType.F32, (d,)),
                 (p + "attn_q.weight", tt["attn_q"], (d, d)),
                 (p + "attn_k.weight", tt["attn_k"], (d, dkv)),
                 (p + "attn_v.weight", tt["attn_v"], (d, dkv)),
                 (p + "attn_output.weight", tt["attn_output"], (d, d)),
                 (p + "ffn_norm.weight", GGMLType.F32, (d,))]
        if spec.n_expert:
            E = spec.n_expert
            plan += [(p + "ffn_gate_inp.weight", GGMLType.F32, (d, E)),
                     (p + "ffn_gate_exps.weight", tt["ffn_gate"], (d, f, E)),
                     (p + "ffn_down_exps.weight", tt["ffn_down"], (f, d, E)),
                     (p + "ffn_up_exps.weight", tt["ffn_up"], (d, f, E))]
        else:
            plan += [(p + "ffn_gate.weight", tt["ffn_gate"], (d, f)),
                     (p + "ffn_down.weight", tt["ffn_down"], (f, d)),
                     (p + "ffn_up.weight", tt["ffn_up"], (d, f))]
    plan += [("output_norm.weight", GGMLType.F32, (d,)), ("output.weight", out_t, (d, n_vocab))]
    return plan


def hparams_metadata(spec: ModelSpec, n_vocab: int) -> Dict:
    a = "llama"
    md = {"general.architecture": a, "general.name": spec.name + " (synthetic random-init)",
          "general.file_type": FTYPE_MOSTLY_Q8_0 if spec.quant == "q8_0" else FTYPE_MOSTLY_Q4_K_M,
          f"{a}.context_length": spec.n_ctx_train, f"{a}.embedding_length": spec.n_embd,
          f"{a}.block_count": spec.n_layer, f"{a}.feed_forward_length": spec.n_ff,
          f"{a}.rope.dimension_count": spec.head_dim, f"{a}.attention.head_count": spec.n_head,
          f"{a}.attention.head_count_kv": spec.n_head_kv,
          f"{a}.attention.layer_norm_rms_epsilon": float(spec.rms_eps),
          f"{a}.rope.freq_base": float(spec.rope_base), f"{a}.vocab_size": n_vocab}
    if spec.n_expert:
        md[f"{a}.expert_count"] = spec.n_expert
        md[f"{a}.expert_used_count"] = spec.n_expert_used
    return md


def write_synthetic_gguf(spec, path: str, seed: int = 0, log=None) -> str:
    """Stream a random-init GGUF for ``spec`` (a ModelSpec or a SPECS key) to ``path``."""
    if isinstance(spec, str):
        spec = SPECS[spec]
    rng = np.random.default_rng(seed)
    vocab_md, n_vocab = build_vocab(spec)
    tmp = path + ".tmp"
    w = GGUFWriter(tmp)
    for k, v in hparams_metadata(spec, n_vocab).items():
        w.add(k, v)
    for k, v in vocab_md.items():
        if k == "tokenizer.ggml.scores":
            w.add(k, v, GGUFValueType.ARRAY, GGUFValueType.FLOAT32)
        elif k == "tokenizer.ggml.token_type":
            w.add(k, v, GGUFValueType.ARRAY, GGUFValueType.INT32)
        elif k.endswith("_token_id"):
            w.add(k, int(v), GGUFValueType.UINT32)
        else:
            w.add(k, v)
    plan = tensor_plan(spec, n_vocab)
    for name, t, shape in plan:
        w.declare_tensor(name, t, shape)
    w.begin()
    for name, t, shape in plan:
        n = int(np.prod(shape))
        if name.endswith("norm.weight"):
            data = (1.0 + 0.1 * rng.standard_normal(n)).astype(np.float32)
        else:
            std = spec.weight_std
            if name == "token_embd.weight":
                std = 1.0  # keeps the first RMSNorm well conditioned
            data = random_blocks(t, n, rng, std=std)
        w.write_tensor_data(data)
        if log:
            log(name)
    w.close()
    os.replace(tmp, path)
    return path


def cached_synthetic_gguf(name: str, cache_dir: Optional[str] = None, seed: int = 0) -> str:
    """Path of a synthetic model, generated once per cache dir."""
    cache_dir = cache_dir or os.environ.get("SYNTH_MODEL_DIR") or os.path.join(
        os.environ.get("TMPDIR", "/tmp"), "llama_amd_models")
    os.makedirs(cache_dir, exist_ok=True)
    path = os.path.join(cache_dir, f"{name}-s{seed}.gguf")
    if not os.path.exists(path):
        write_synthetic_gguf(name, path, seed)
    return path
