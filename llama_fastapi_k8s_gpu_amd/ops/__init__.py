"""Torch-facing wrappers of the gfx950 HIP kernels (``csrc/kernels``).

These are the kernels the C++ engine schedules, exposed on ``torch`` tensors for
tests, experiments and custom pipelines. Every wrapper validates shapes, dtypes,
devices and contiguity on the host BEFORE the launch (a mis-shaped operand would
otherwise be an out-of-bounds access on the GPU) and runs on the current torch
stream. There is no fallback: without the ``_hip`` extension they raise.

    W = QuantMatrix.from_ggml(raw_bytes, GGMLType.Q4_K, rows, K)    # planar repack + upload
    y = gemv(W, x)                                  # y[rows] = W . x   (q8 activations, v_dot4)
    y = gemv(W, x, norm=w_norm)                     # RMSNorm fused into the prologue
    gemv(W, x, out=resid, accumulate=True)          # resid += W . x
    h = gemv_swiglu(W_gu, x, norm=w)                # silu(gate) * up, gate/up interleaved by 32 rows
    Y = gemm(W, X_bf16)                             # [T, rows] on MFMA with LDS-dequantised tiles
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

EPI_STORE, EPI_ADD, EPI_SWIGLU = 0, 1, 2
GEMM_STORE, GEMM_ADD, GEMM_SWIGLU = 0, 1, 2


def _hip():
    from ..runtime import load_hip
    return load_hip()


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def _check(t, dtype, shape=None, name="tensor"):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    return t.data_ptr()


@dataclass
class QuantMatrix:
    """A [rows, K] ggml-quantised matrix in the planar device layout."""
    data: "object"        # torch.uint8 CUDA tensor
    qtype: int
    rows: int
    K: int
    expert_stride: int = 0

    @classmethod
    def from_ggml(cls, raw: np.ndarray, qtype: int, rows: int, K: int, interleave_gate_up: bool = False,
                  raw_up: Optional[np.ndarray] = None) -> "QuantMatrix":
        import torch
        hip = _hip()
        raw = np.ascontiguousarray(np.frombuffer(raw, np.uint8) if isinstance(raw, (bytes, bytearray)) else raw)
        if raw.nbytes != hip.qbytes(int(qtype), rows, K):
            raise ValueError("raw block bytes do not match (type, rows, K)")
        if not interleave_gate_up:
            planar = hip.repack(int(qtype), raw, K, 0, rows, 0, K, rows, 0, 0)
            return cls(torch.from_numpy(planar).cuda(), int(qtype), rows, K)
        if raw_up is None:
            raise ValueError("interleave_gate_up needs raw_up")
        g = hip.repack(int(qtype), raw, K, 0, rows, 0, K, 2 * rows, 32, 0)
        u = hip.repack(int(qtype), np.ascontiguousarray(raw_up), K, 0, rows, 0, K, 2 * rows, 32, 32)
        return cls(torch.from_numpy(g | u).cuda(), int(qtype), 2 * rows, K)


def _x_ptr(x, K, norm):
    import torch
    xp = _check(x, torch.float32, (K,), "x")
    if K % 256 and K % 32:
        raise ValueError("K must be a multiple of 32")
    np_ = _check(norm, torch.float32, (K,), "norm") if norm is not None else 0
    return xp, np_


def gemv(W: QuantMatrix, x, norm=None, eps: float = 1e-5, out=None, accumulate: bool = False):
    """y = W . x  (optionally x <- rmsnorm(x) * norm; optionally out += W . x)."""
    import torch
    xp, npp = _x_ptr(x, W.K, norm)
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = torch.empty(W.rows, device=x.device, dtype=torch.float32)
    op = _check(out, torch.float32, (W.rows,), "out")
    _hip().gemv(W.data.data_ptr(), W.qtype, W.rows, W.K, xp, npp, eps, op, W.rows,
                EPI_ADD if accumulate else EPI_STORE, _stream())
    return out


def gemv_swiglu(W_gu: QuantMatrix, x, norm=None, eps: float = 1e-5):
    """silu(gate . x) * (up . x) for a gate/up matrix interleaved in 32-row groups."""
    import torch
    if W_gu.rows % 64:
        raise ValueError("gate/up matrix must have a multiple of 64 rows")
    xp, npp = _x_ptr(x, W_gu.K, norm)
    F = W_gu.rows // 2
    out = torch.empty(F, device=x.device, dtype=torch.float32)
    _hip().gemv(W_gu.data.data_ptr(), W_gu.qtype, W_gu.rows, W_gu.K, xp, npp, eps, out.data_ptr(), F, EPI_SWIGLU,
                _stream())
    return out


def gemm(W: QuantMatrix, x_bf16, out=None, accumulate: bool = False):
    """Y[T, rows] = X[T, K] . W^T on MFMA (weights dequantised into LDS tiles)."""
    import torch
    if x_bf16.dim() != 2 or x_bf16.shape[1] != W.K:
        raise ValueError(f"x must be [T, {W.K}]")
    T = int(x_bf16.shape[0])
    xp = _check(x_bf16, torch.bfloat16, None, "x")
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = torch.empty(T, W.rows, device=x_bf16.device, dtype=torch.float32)
    op = _check(out, torch.float32, (T, W.rows), "out")
    _hip().gemm(W.data.data_ptr(), W.qtype, W.rows, W.K, xp, T, op, 0, W.rows,
                GEMM_ADD if accumulate else GEMM_STORE, _stream())
    return out


def rmsnorm_bf16(x, w, eps: float = 1e-5):
    import torch
    if x.dim() != 2:
        raise ValueError("x must be [T, d]")
    T, d = map(int, x.shape)
    xp = _check(x, torch.float32, (T, d), "x")
    wp = _check(w, torch.float32, (d,), "w")
    y = torch.empty(T, d, device=x.device, dtype=torch.bfloat16)
    _hip().rmsnorm_bf16(xp, wp, eps, T, d, y.data_ptr(), _stream())
    return y


def embed(W: QuantMatrix, tokens):
    """Dequantised rows W[tokens] -> float32 [T, K]."""
    import torch
    tp = _check(tokens, torch.int32, None, "tokens")
    T = int(tokens.numel())
    if T and (int(tokens.min()) < 0 or int(tokens.max()) >= W.rows):
        raise ValueError("token id out of range")
    out = torch.empty(T, W.K, device=tokens.device, dtype=torch.float32)
    _hip().embed(W.data.data_ptr(), W.qtype, W.rows, W.K, tp, T, out.data_ptr(), _stream())
    return out


def attention_decode(q, k_cache, v_cache, pos: int, scale: Optional[float] = None):
    """One query token per head against keys [0, pos] of an f16 cache [n_kv, n_ctx, hd]."""
    import torch
    n_kv, n_ctx, hd = map(int, k_cache.shape)
    n_head = int(q.numel()) // hd
    if n_head % n_kv or not 0 <= pos < n_ctx or hd not in (64, 128):
        raise ValueError("bad attention shapes")
    qp = _check(q, torch.float32, (n_head * hd,), "q")
    kp = _check(k_cache, torch.float16, (n_kv, n_ctx, hd), "k_cache")
    vp = _check(v_cache, torch.float16, (n_kv, n_ctx, hd), "v_cache")
    hip = _hip()
    part = torch.empty(hip.attn_decode_workspace_floats(n_ctx, n_head, hd), device=q.device, dtype=torch.float32)
    cnt = torch.zeros(64, device=q.device, dtype=torch.int32)
    p = torch.tensor([pos], device=q.device, dtype=torch.int32)
    out = torch.empty(n_head * hd, device=q.device, dtype=torch.float32)
    hip.attn_decode(qp, kp, vp, p.data_ptr(), n_ctx, n_head, n_kv, hd, scale or hd ** -0.5, part.data_ptr(),
                    out.data_ptr(), _stream(), cnt.data_ptr())
    return out


def attention_prefill(q, k_cache, v_cache, pos0: int, scale: Optional[float] = None):
    """Causal attention of T query tokens (positions pos0..pos0+T-1) -> [T, n_head*hd]."""
    import torch
    n_kv, n_ctx, hd = map(int, k_cache.shape)
    T = int(q.shape[0])
    n_head = int(q.shape[1]) // hd
    if n_head % n_kv or pos0 < 0 or pos0 + T > n_ctx or hd not in (64, 128):
        raise ValueError("bad attention shapes")
    qp = _check(q, torch.float32, (T, n_head * hd), "q")
    kp = _check(k_cache, torch.float16, (n_kv, n_ctx, hd), "k_cache")
    vp = _check(v_cache, torch.float16, (n_kv, n_ctx, hd), "v_cache")
    out = torch.empty(T, n_head * hd, device=q.device, dtype=torch.float32)
    _hip().attn_prefill(qp, kp, vp, T, pos0, n_ctx, n_head, n_kv, hd, scale or hd ** -0.5, out.data_ptr(),
                        _stream())
    return out


__all__ = ["QuantMatrix", "gemv", "gemv_swiglu", "gemm", "rmsnorm_bf16", "embed", "attention_decode",
           "attention_prefill"]
