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
    """float32 torch forward over a GGUFReader (CPU; tiny models only).

    ``forward(..., path=...)`` optionally reproduces the activation and weight rounding of
    one of the MI355X engine's compute paths, so engine-level tests can hold the engine to
    ~1e-3 instead of the ~5e-2 its roundings cost against the exact model:

      * ``"decode"`` (single-row GEMV, kernels/gemv.hip): every projection input quantised
        to q8 per 32 (scale amax/127, nearest) - of x * w_norm before the 1/rms scale for the
        normed inputs - exact weights; attention on f16 q * scale, f16 K/V;
      * ``"prefill"`` (MFMA GEMM, kernels/gemm.hip + attention.hip): bf16 activations and
        bf16-rounded dequantised weights; attention with q * scale * log2(e) in f16, f16 P and
        K/V, bf16 output; the logits row through the decode head (q8);
      * ``"prefill16"`` (the tile16 prefill GEMM, gemm_t16 in kernels/bmm.hip, engines with
        batching on): f16(x / rms * w) inputs, f16 attention and SwiGLU outputs, the tile16 copy's
        f16-arithmetic weights (MoE: the router on the bf16 norm as ``"prefill"``); attention and
        head as ``"prefill"``;
      * ``"batch"`` (batched MFMA projections, kernels/bmm.hip): f16(x * w_norm) with the
        1/rms applied to the f32 result (d = 4096, the folded norm; f16(x / rms * w) below), f16 weights from the tile16 copy's f16 arithmetic
        (quants.dequantize(arith="f16")), f16 attention output and SwiGLU output; the head
        input f16(x / rms * w).
    K/V are stored f16 in every emulated path (the engine's cache). ``path=None`` is the exact
    fp32 model.
    """

    def __init__(self, reader, n_ctx: int = 512, device: str = "cpu"):
        import torch
        self.torch = torch
        self.reader = reader
        self.device = device
        self._router_trace = None
        self.hp = LlamaHParams.from_metadata(reader.metadata)
        hp = self.hp
        if not hp.n_vocab:
            hp.n_vocab = reader.tensors["token_embd.weight"].shape[1]
        self.n_ctx = n_ctx
        t = lambda name: torch.from_numpy(np.ascontiguousarray(reader.dequant(name))).to(device)
        self.tok_embd = t("token_embd.weight")
        self.out_norm = t("output_norm.weight")
        self._out_name = "output.weight" if "output.weight" in reader.tensors else "token_embd.weight"
        self.output = t(self._out_name)
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
            L["_prefix"] = p
            self.layers.append(L)
        cos, sin = rope_tables(hp, n_ctx)
        self.cos = torch.from_numpy(cos).to(device)
        self.sin = torch.from_numpy(sin).to(device)
        self.k_cache = torch.zeros(hp.n_layer, n_ctx, hp.n_head_kv, hp.head_dim, device=device)
        self.v_cache = torch.zeros_like(self.k_cache)
        self._wcache: Dict = {}

    # ------------------------------------------------------------ rounding helpers
    def _f16(self, x):
        return x.half().float()

    def _bf16(self, x):
        return x.bfloat16().float()

    def _q8(self, x):
        """Per-32-block symmetric int8 quantise-dequantise along the last dim."""
        torch = self.torch
        shp = x.shape
        b = x.reshape(*shp[:-1], shp[-1] // 32, 32)
        amax = b.abs().amax(-1, keepdim=True)
        s = amax / 127.0
        q = torch.where(s > 0, torch.round(b / torch.where(s > 0, s, torch.ones_like(s))), torch.zeros_like(b))
        return (q * s).reshape(shp)

    def _weight(self, key: str, L: Optional[Dict], kind: str):
        """Weight `key` of layer L (or the output head, L None) as the path reads it."""
        if kind == "f32":
            return self.output if L is None else L[key]
        name = self._out_name if L is None else L["_prefix"] + key + ".weight"
        ck = (name, kind)
        if ck not in self._wcache:
            torch = self.torch
            if kind == "bf16":
                w = self._bf16(self.output if L is None else L[key])
            else:  # "f16": the batched path's tile16 dequantisation (F32/F16 tensors stay exact)
                ti = self.reader.tensors[name]
                arr = np.asarray(self.reader.raw(name))
                from ..gguf.quants import dequantize
                w = torch.from_numpy(np.ascontiguousarray(
                    dequantize(arr, ti.ggml_type, ti.n_elements, arith="f16").reshape(ti.shape[::-1]))).to(self.device)
            self._wcache[ck] = w
        return self._wcache[ck]

    def _rms(self, x, w):
        return x * self.torch.rsqrt((x * x).mean(-1, keepdim=True) + self.hp.rms_eps) * w

    def _normed_input(self, x, w, path, attn: bool = False):
        """The normalised projection input the path feeds its matmul (``attn``: the Q|K|V input)."""
        torch = self.torch
        rs = torch.rsqrt((x * x).mean(-1, keepdim=True) + self.hp.rms_eps)
        if path == "decode":
            return self._q8(x * w) * rs
        if path == "prefill":
            return self._bf16(x * rs * w)
        if path == "prefill16":
            return self._f16(x * rs * w)
        if path == "batch":
            # the split-K Q|K|V (any d) and, at d = 4096, the one-part gate/up stage f16(x * w) and
            # apply 1/rms to the f32 result; otherwise bmm's prep kernel stages f16(x / rms * w)
            return self._f16(x * w) * rs if attn or x.shape[-1] == 4096 else self._f16(x * rs * w)
        return x * rs * w

    def _plain_input(self, h, path):
        """A projection input that is not a norm output (attention out, SwiGLU out)."""
        if path == "decode":
            return self._q8(h)
        if path == "prefill":
            return self._bf16(h)
        if path in ("batch", "prefill16"):
            return self._f16(h)
        return h

    def _wkind(self, path):
        return {"prefill": "bf16", "batch": "f16", "prefill16": "f16"}.get(path, "f32")

    def _rope(self, x, pos):
        # x [T, H, D]; adjacent pairs (2i, 2i+1)
        c = self.cos[pos][:, None, :]
        s = self.sin[pos][:, None, :]
        x0, x1 = x[..., 0::2], x[..., 1::2]
        out = self.torch.empty_like(x)
        out[..., 0::2] = x0 * c - x1 * s
        out[..., 1::2] = x0 * s + x1 * c
        return out

    def _ffn(self, L, x, path):
        torch = self.torch
        F = torch.nn.functional
        wk = self._wkind(path)
        h = self._normed_input(x, L["ffn_norm"], path)
        if not self.hp.n_expert:
            a = F.silu(h @ self._weight("ffn_gate", L, wk).T) * (h @ self._weight("ffn_up", L, wk).T)
            return self._plain_input(a, path) @ self._weight("ffn_down", L, wk).T
        # MoE: the decode path runs the GEMV experts (q8) with the f32 router; the batched path
        # the stacked-expert bmm (f16 tile16 weights, f16 input, f32 router, the SwiGLU output
        # scaled by the routing weight before its f16 rounding)
        if path == "batch":
            hr = self._normed_input(x, L["ffn_norm"], None)
            probs = torch.softmax(hr @ L["ffn_gate_inp"].T, -1)
            w, ids = torch.topk(probs, self.hp.n_expert_used, dim=-1)
            w = w / w.sum(-1, keepdim=True)
            ge, ue, de = (self._weight(k, L, "f16") for k in ("ffn_gate_exps", "ffn_up_exps", "ffn_down_exps"))
            out = torch.zeros_like(h)
            for t in range(h.shape[0]):
                for j in range(self.hp.n_expert_used):
                    e = int(ids[t, j])
                    g = F.silu(ge[e] @ h[t]) * (ue[e] @ h[t])
                    out[t] += de[e] @ self._f16(g * w[t, j])
            return out
        if path == "prefill16":
            # the router GEMM reads the bf16 norm (planar gemm_dq); the experts run on the tile16
            # copies with the f16 norm, f16 SwiGLU output, routing weight applied after down
            hr = self._normed_input(x, L["ffn_norm"], "prefill")
            probs = torch.softmax(hr @ self._bf16(L["ffn_gate_inp"]).T, -1)
            w, ids = torch.topk(probs, self.hp.n_expert_used, dim=-1)
            w = w / w.sum(-1, keepdim=True)
            ge, ue, de = (self._weight(k, L, "f16") for k in ("ffn_gate_exps", "ffn_up_exps", "ffn_down_exps"))
            out = torch.zeros_like(h)
            for t in range(h.shape[0]):
                for j in range(self.hp.n_expert_used):
                    e = int(ids[t, j])
                    g = F.silu(ge[e] @ h[t]) * (ue[e] @ h[t])
                    out[t] += w[t, j] * (de[e] @ self._f16(g))
            return out
        rw = L["ffn_gate_inp"] if path != "prefill" else self._bf16(L["ffn_gate_inp"])
        hr = self._normed_input(x, L["ffn_norm"], None) if path == "decode" else h
        logits = hr @ rw.T                                    # [T, E]
        if self._router_trace is not None:
            self._router_trace.append(logits.clone())
        probs = torch.softmax(logits, -1)
        w, ids = torch.topk(probs, self.hp.n_expert_used, dim=-1)
        w = w / w.sum(-1, keepdim=True)
        out = torch.zeros_like(h)
        ge = L["ffn_gate_exps"] if path is None else self._bf16(L["ffn_gate_exps"]) if path == "prefill" else L["ffn_gate_exps"]
        ue = L["ffn_up_exps"] if path is None else self._bf16(L["ffn_up_exps"]) if path == "prefill" else L["ffn_up_exps"]
        de = L["ffn_down_exps"] if path is None else self._bf16(L["ffn_down_exps"]) if path == "prefill" else L["ffn_down_exps"]
        for t in range(h.shape[0]):
            for j in range(self.hp.n_expert_used):
                e = int(ids[t, j])
                g = F.silu(ge[e] @ h[t]) * (ue[e] @ h[t])
                out[t] += w[t, j] * (de[e] @ self._plain_input(g[None], path)[0])
        return out

    def _attention(self, q, li, pos, n_past, T, path):
        torch = self.torch
        hp = self.hp
        scale = 1.0 / np.sqrt(hp.head_dim)
        Lk = n_past + T
        K = self.k_cache[li, :Lk].repeat_interleave(hp.gqa, dim=1)   # [Lk, H, D]
        V = self.v_cache[li, :Lk].repeat_interleave(hp.gqa, dim=1)
        mask = torch.arange(Lk, device=pos.device)[None, :] > pos[:, None]
        if path in ("prefill", "prefill16"):
            l2e = 1.4426950408889634
            s = torch.einsum("thd,lhd->htl", self._f16(q * (scale * l2e)), K)
            s = s.masked_fill(mask[None], float("-inf"))
            p = torch.exp2(s - s.amax(-1, keepdim=True))
            a = torch.einsum("htl,lhd->thd", self._f16(p), V) / p.sum(-1).permute(1, 0)[..., None]
            return a.reshape(T, -1)
        if path in ("decode", "batch"):
            q = self._f16(q * scale)
            s = torch.einsum("thd,lhd->htl", q, K)
        else:
            s = torch.einsum("thd,lhd->htl", q, K) * scale
        s = s.masked_fill(mask[None], float("-inf"))
        return torch.einsum("htl,lhd->thd", torch.softmax(s, -1), V).reshape(T, -1)

    def forward(self, tokens, n_past: int, all_logits: bool = False, trace: Optional[List[Dict]] = None,
                path: Optional[str] = None, router_trace: Optional[List] = None):
        """Evaluate ``tokens`` at positions n_past.. ; returns logits [T,V] or [V].
        ``trace`` (a list) receives per layer the last token's q / k / v (roped), the attention
        output, x after the attention residual, the SwiGLU output and x after the FFN residual.
        ``path``: None (exact fp32) or the engine path whose rounding to reproduce (class doc).
        ``router_trace`` (a list, MoE, path None / decode / prefill) receives per layer the router
        logits [T, E] - the TP tests judge an expert flip by their top-k margin."""
        torch = self.torch
        hp = self.hp
        if path not in (None, "decode", "prefill", "prefill16", "batch"):
            raise ValueError(f"unknown path {path!r}")
        T = len(tokens)
        self._router_trace = router_trace
        pos = torch.arange(n_past, n_past + T, device=self.device)
        x = self.tok_embd[torch.as_tensor(list(tokens), device=self.device)]
        wk = self._wkind(path)
        for li, L in enumerate(self.layers):
            h = self._normed_input(x, L["attn_norm"], path, attn=True)
            q = (h @ self._weight("attn_q", L, wk).T).view(T, hp.n_head, hp.head_dim)
            k = (h @ self._weight("attn_k", L, wk).T).view(T, hp.n_head_kv, hp.head_dim)
            v = (h @ self._weight("attn_v", L, wk).T).view(T, hp.n_head_kv, hp.head_dim)
            q, k = self._rope(q, pos), self._rope(k, pos)
            if path is not None:   # the engine's KV cache is f16
                k, v = self._f16(k), self._f16(v)
            self.k_cache[li, n_past:n_past + T] = k
            self.v_cache[li, n_past:n_past + T] = v
            a = self._attention(q, li, pos, n_past, T, path)
            x = x + self._plain_input(a, path) @ self._weight("attn_output", L, wk).T
            if trace is not None and not self.hp.n_expert:
                F = torch.nn.functional
                hn = self._rms(x, L["ffn_norm"])
                hh = F.silu(hn @ L["ffn_gate"].T) * (hn @ L["ffn_up"].T)
                trace.append({"q": q[-1].reshape(-1).clone(), "k": k[-1].reshape(-1).clone(),
                              "v": v[-1].reshape(-1).clone(), "o": a[-1].clone(), "x_attn": x[-1].clone(),
                              "h": hh[-1].clone()})
            x = x + self._ffn(L, x, path)
            if trace is not None and not self.hp.n_expert:
                trace[-1]["x_ffn"] = x[-1].clone()
        # the logits: prefill and decode both end on the GEMV head (q8); the batched head
        # stages f16(x / rms * w) for the tile16 f16 output weights
        hpath = {"prefill": "decode", "prefill16": "decode"}.get(path, path)
        if hpath == "batch":
            rs = torch.rsqrt((x * x).mean(-1, keepdim=True) + hp.rms_eps)
            xo = self._f16(x * rs * self.out_norm)
        else:
            xo = self._normed_input(x, self.out_norm, hpath)
        W = self._weight(None, None, self._wkind(hpath))
        if all_logits:
            return xo @ W.T
        return xo[-1] @ W.T
