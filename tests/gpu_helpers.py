"""Shared helpers for the GPU numerics tests: planar upload of NumPy-generated
blocks, q8 activation emulation, and torch fp32 references."""
import numpy as np

from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType
from llama_fastapi_k8s_gpu_amd.gguf.quants import dequantize, quantize, random_blocks


def hip():
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    return load_hip()


def stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def make_matrix(t, R, K, rng, std=0.05):
    """Random ggml blocks for an R x K matrix -> (ggml bytes, float32 [R,K] dequantised)."""
    if t in (GGMLType.F32, GGMLType.F16):
        w = (rng.standard_normal(R * K) * std).astype(np.float32)
        raw = quantize(w, t)
    else:
        raw = random_blocks(t, R * K, rng, std=std)
    deq = dequantize(raw, t, R * K).reshape(R, K)
    return raw, deq


def to_planar(t, raw, R, K, R_dst=None, G=0, off=0, r0=0, Rsel=None, c0=0, Kdst=None, K_src=None):
    return hip().repack(int(t), np.ascontiguousarray(raw), K_src or K, r0, Rsel if Rsel is not None else R,
                        c0, Kdst or K, R_dst or R, G, off)


def dev_bytes(arr):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


def q8_emulate(x):
    """Exactly the kernel prologue's per-32 int8 quantisation (round half to even)."""
    xb = x.astype(np.float32).reshape(-1, 32)
    amax = np.abs(xb).max(axis=1)
    d = (amax * np.float32(1.0 / 127.0)).astype(np.float32)
    inv = np.where(d > 0, np.float32(1.0) / np.where(d > 0, d, 1), 0).astype(np.float32)
    q = np.rint(xb * inv[:, None]).astype(np.float32)
    return (q * d[:, None]).reshape(-1)


def rmsnorm(x, w, eps=1e-5):
    x = x.astype(np.float64)
    return (x / np.sqrt(np.mean(x * x) + eps) * w).astype(np.float32)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
