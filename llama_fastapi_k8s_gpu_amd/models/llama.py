"""Llama-family hyper-parameters (dense + Mixtral MoE) and a plain PyTorch fp32
reference forward pass.

The reference forward is the numerics oracle for every native backend (T4 in
SURVEY §4.3): it dequantises each GGUF weight with the NumPy block decoders and
runs the upstream ``llm_build_llama`` op sequence in float32:

    x = embd[tok]
    for layer: h = rms(x)*w ; q,k,v = Wq h, Wk h, Wv h ; rope(q,k) (adjacent pairs,
               GGUF "normal" mode) ; attn = softmax(q k^T/sqrt(d) + causal) v ;
               x += Wo attn ; h = rms(x)*w ;
               x += Wdown(silu(Wgate h) * Wup h)          (dense)
               x += sum_e w_e Wdown_e(silu(Wgate_e h)*Wup_e h)  (MoE, top-k, renorm)
    logits = Wout rms(x)*w
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np


@dataclass
class LlamaHParams:
    n_vocab: int
    n_embd: int
    n_layer: int
    n_head: int
    n_head_kv: int
    head_dim: int
    n_ff: int
    n_expert: int
    n_expert_used: int
    rope_base: float
    rms_eps: float
    n_ctx_train: int

    @property
    def n_embd_kv(self) -> int:
        return self.head_dim * self.n_head_kv

    @property
    def gqa(self) -> int:
        return self.n_head // self.n_head_kv

    @classmethod
    def from_metadata(cls, md: Dict) -> "LlamaHParams":
        arch = md.get("general.architecture", "llama")
        if arch not in ("llama", "mistral", "mixtral"):
            raise NotImplementedError(f"architecture {arch!r} is not supported")
        g = lambda k, d=None: md.get(f"{arch}.{k}", d)
        n_embd = int(g("embedding_length"))
        n_head = int(g("attention.head_count"))
        n_vocab = int(g("vocab_size", 0) or len(md.get("tokenizer.ggml.tokens", [])))
        return cls(n_vocab=n_vocab, n_embd=n_embd, n_layer=int(g("block_count")), n_head=n_head,
                   n_head_kv=int(g("attention.head_count_kv", n_head)),
                   head_dim=int(g("rope.dimension_count", n_embd // n_head)),
                   n_ff=int(g("feed_forward_length")), n_expert=int(g("expert_count", 0) or 0),
                   n_expert_used=int(g("expert_used_count", 0) or 0),
                   rope_base=float(g("rope.freq_base", 10000.0)),
                   rms_eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)),
                   n_ctx_train=int(g("context_length", 2048)))


def rope_tables(hp: LlamaHParams, n_pos: int):
    """cos/sin [n_pos, head_dim/2] (float32), same formula the kernels use."""
    i = np.arange(hp.head_dim // 2, dtype=np.float64)
    inv = hp.rope_base ** (-2.0 * i / hp.head_dim)
    ang = np.arange(n_pos, dtype=np.float64)[:, None] * inv[None, :]
    return np.cos(ang).astype(np.float32), np.sin(ang).astype(np.float32)


class ReferenceLlama:
    """float32 torch forward over a GGUFReader (CPU; tiny models only)."""

    def __init__(self, reader, n_ctx: int = 512, device: str = "cpu"):
        import torch
        self.torch = torch
        self.hp = LlamaHParams.from_metadata(reader.metadata)
        hp = self.hp
        if not hp.n_vocab:
            hp.n_vocab = reader.tensors["token_embd.weight"].shape[1]
        self.n_ctx = n_ctx
        t = lambda name: torch.from_numpy(np.ascontiguousarray(reader.dequant(name))).to(device)
        self.tok_embd = t("token_embd.weight")
        self.out_norm = t("output_norm.weight")
        self.output = t("output.weight") if "output.weight" in reader.tensors else self.tok_embd
        self.layers: List[Dict] = []
        for i in range(hp.n_layer):
            p = f"blk.{i}."
            L = {k: t(p + k + ".weight") for k in ("attn_norm", "attn_q", "attn_k", "attn_v",
                                                   "attn_output", "ffn_norm")}
            if hp.n_expert:
                for k in ("ffn_gate_inp", "ffn_gate_exps", "ffn_up_exps", "ffn_down_exps"):
                    L[k] = t(p + k + ".weight")
            else:
                for k in ("ffn_gate", "ffn_up", "ffn_down"):
                    L[k] = t(p + k + ".weight")
            self.layers.append(L)
        cos, sin = rope_tables(hp, n_ctx)
        self.cos = torch.from_numpy(cos).to(device)
        self.sin = torch.from_numpy(sin).to(device)
        self.k_cache = torch.zeros(hp.n_layer, n_ctx, hp.n_head_kv, hp.head_dim, device=device)
        self.v_cache = torch.zeros_like(self.k_cache)

    def _rms(self, x, w):
        return x * self.torch.rsqrt((x * x).mean(-1, keepdim=True) + self.hp.rms_eps) * w

    def _rope(self, x, pos):
        # x [T, H, D]; adjacent pairs (2i, 2i+1)
        c = self.cos[pos][:, None, :]
        s = self.sin[pos][:, None, :]
        x0, x1 = x[..., 0::2], x[..., 1::2]
        out = self.torch.empty_like(x)
        out[..., 0::2] = x0 * c - x1 * s
        out[..., 1::2] = x0 * s + x1 * c
        return out

    def _ffn(self, L, h):
        torch = self.torch
        F = torch.nn.functional
        if not self.hp.n_expert:
            return (F.silu(h @ L["ffn_gate"].T) * (h @ L["ffn_up"].T)) @ L["ffn_down"].T
        logits = h @ L["ffn_gate_inp"].T                      # [T, E]
        probs = torch.softmax(logits, -1)
        w, ids = torch.topk(probs, self.hp.n_expert_used, dim=-1)
        w = w / w.sum(-1, keepdim=True)
        out = torch.zeros_like(h)
        for t in range(h.shape[0]):
            for j in range(self.hp.n_expert_used):
                e = int(ids[t, j])
                g = F.silu(L["ffn_gate_exps"][e] @ h[t]) * (L["ffn_up_exps"][e] @ h[t])
                out[t] += w[t, j] * (L["ffn_down_exps"][e] @ g)
        return out

    def forward(self, tokens, n_past: int, all_logits: bool = False, trace: Optional[List[Dict]] = None):
        """Evaluate ``tokens`` at positions n_past.. ; returns logits [T,V] or [V].
        ``trace`` (a list) receives per layer the last token's q / k / v (roped), the attention
        output, x after the attention residual, the SwiGLU output and x after the FFN residual."""
        torch = self.torch
        hp = self.hp
        T = len(tokens)
        pos = torch.arange(n_past, n_past + T)
        x = self.tok_embd[torch.as_tensor(list(tokens))]
        scale = 1.0 / np.sqrt(hp.head_dim)
        for li, L in enumerate(self.layers):
            h = self._rms(x, L["attn_norm"])
            q = (h @ L["attn_q"].T).view(T, hp.n_head, hp.head_dim)
            k = (h @ L["attn_k"].T).view(T, hp.n_head_kv, hp.head_dim)
            v = (h @ L["attn_v"].T).view(T, hp.n_head_kv, hp.head_dim)
            q, k = self._rope(q, pos), self._rope(k, pos)
            self.k_cache[li, n_past:n_past + T] = k
            self.v_cache[li, n_past:n_past + T] = v
            Lk = n_past + T
            K = self.k_cache[li, :Lk].repeat_interleave(hp.gqa, dim=1)   # [Lk, H, D]
            V = self.v_cache[li, :Lk].repeat_interleave(hp.gqa, dim=1)
            s = torch.einsum("thd,lhd->htl", q, K) * scale
            mask = torch.arange(Lk)[None, :] > pos[:, None]
            s = s.masked_fill(mask[None], float("-inf"))
            a = torch.einsum("htl,lhd->thd", torch.softmax(s, -1), V).reshape(T, -1)
            x = x + a @ L["attn_output"].T
            h = self._rms(x, L["ffn_norm"])
            if trace is not None and not self.hp.n_expert:
                F = torch.nn.functional
                hh = F.silu(h @ L["ffn_gate"].T) * (h @ L["ffn_up"].T)
                trace.append({"q": q[-1].reshape(-1).clone(), "k": k[-1].reshape(-1).clone(),
                              "v": v[-1].reshape(-1).clone(), "o": a[-1].clone(), "x_attn": x[-1].clone(),
                              "h": hh[-1].clone()})
            x = x + self._ffn(L, h)
            if trace is not None and not self.hp.n_expert:
                trace[-1]["x_ffn"] = x[-1].clone()
        x = self._rms(x, self.out_norm)
        if all_logits:
            return x @ self.output.T
        return x[-1] @ self.output.T
