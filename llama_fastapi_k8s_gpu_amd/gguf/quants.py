"""NumPy reference implementation of the ggml block formats used by Q4_K_M /
Q8_0 GGUF files: Q4_K, Q5_K, Q6_K, Q8_0 (+ F16/BF16/F32).

This is the *reference* every native path is tested against (T1 in SURVEY
§4.3): the C++ CPU backend, the GPU repack and the HIP kernels must reproduce
``dequantize`` exactly (up to f32 rounding).

Block layouts:
  Q8_0  34 B / 32 w : d f16 | qs int8[32]                 w = d*q
  Q4_K 144 B / 256 w: d f16 | dmin f16 | scales[12] | qs[128]
                      w = d*sc_j*q - dmin*m_j ; 6-bit (sc,m) packed, get_scale_min_k4
  Q5_K 176 B / 256 w: d | dmin | scales[12] | qh[32] | qs[128]  (5th bit from qh)
  Q6_K 210 B / 256 w: ql[128] | qh[64] | scales int8[16] | d f16  w = d*sc*(q-32)

The quantisers are simple (min/max per sub-block, no iterative search) - they
produce valid blocks with bounded error, which is all the synthetic-model and
test paths need; decoding is what must match real llama.cpp files.
"""
from __future__ import annotations

import numpy as np

from .constants import GGML_BLOCK, QK_K, GGMLType

# ----------------------------------------------------------------- helpers


def _f16(a) -> np.ndarray:
    return np.asarray(a, dtype=np.float32).astype(np.float16)


def _unpack_scale_min_k4(scales: np.ndarray):
    """scales: uint8 [nb, 12] -> (sc, m) uint8 [nb, 8] (ggml get_scale_min_k4)."""
    s = scales.astype(np.uint8)
    sc = np.empty((s.shape[0], 8), np.uint8)
    m = np.empty((s.shape[0], 8), np.uint8)
    sc[:, :4] = s[:, 0:4] & 63
    m[:, :4] = s[:, 4:8] & 63
    sc[:, 4:] = (s[:, 8:12] & 0xF) | ((s[:, 0:4] >> 6) << 4)
    m[:, 4:] = (s[:, 8:12] >> 4) | ((s[:, 4:8] >> 6) << 4)
    return sc, m


def _pack_scale_min_k4(sc: np.ndarray, m: np.ndarray) -> np.ndarray:
    """Inverse of _unpack_scale_min_k4; sc, m uint8 [nb, 8] with values < 64."""
    sc = sc.astype(np.uint8)
    m = m.astype(np.uint8)
    out = np.zeros((sc.shape[0], 12), np.uint8)
    out[:, 0:4] = (sc[:, 0:4] & 63) | ((sc[:, 4:8] >> 4) << 6)
    out[:, 4:8] = (m[:, 0:4] & 63) | ((m[:, 4:8] >> 4) << 6)
    out[:, 8:12] = (sc[:, 4:8] & 0xF) | ((m[:, 4:8] & 0xF) << 4)
    return out


def _blocks(data: np.ndarray, ggml_type) -> np.ndarray:
    bs, bb = GGML_BLOCK[GGMLType(ggml_type)]
    raw = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                               else data.view(np.uint8).reshape(-1))
    assert raw.size % bb == 0
    return raw.reshape(-1, bb)

# ------------------------------------------------------------- dequantise


def dequantize(data, ggml_type, n_elements: int | None = None, arith: str = "f32") -> np.ndarray:
    """Decode raw ggml bytes into float32 (flat).

    ``arith="f16"`` reproduces the batched decode projection's dequantisation bit for bit
    (kernels/bmm.hip on its tile16 copy): the per-sub-block scale d*sc and offset -dmin*m are
    rounded to f16 once, and every weight is ONE f16 rounding of q*scale + offset (a fused
    v_pk_fma_f16). Returned as float32 (exact f16 values)."""
    t = GGMLType(ggml_type)
    if arith == "f16" and t in (GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K):
        return _dequantize_f16(data, t, n_elements)
    if t == GGMLType.F32:
        return np.frombuffer(bytes(data) if not isinstance(data, np.ndarray) else data.tobytes(),
                             dtype=np.float32).copy()
    if t == GGMLType.F16:
        return np.asarray(data).view(np.uint8).reshape(-1).view(np.float16).astype(np.float32)
    if t == GGMLType.BF16:
        u = np.asarray(data).view(np.uint8).reshape(-1).view(np.uint16).astype(np.uint32) << 16
        return u.view(np.float32).copy()
    b = _blocks(data, t)
    nb = b.shape[0]
    if t == GGMLType.Q8_0:
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)  # [nb,1]
        q = b[:, 2:34].view(np.int8).astype(np.float32)
        out = d * q
    elif t in (GGMLType.Q4_K, GGMLType.Q5_K):
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
        dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)
        sc, m = _unpack_scale_min_k4(b[:, 4:16])
        if t == GGMLType.Q4_K:
            qs = b[:, 16:144]
            qh = None
        else:
            qh = b[:, 16:48]
            qs = b[:, 48:176]
        out = np.empty((nb, 256), np.float32)
        for j in range(4):
            grp = qs[:, 32 * j:32 * j + 32]
            lo = (grp & 0xF).astype(np.float32)
            hi = (grp >> 4).astype(np.float32)
            if qh is not None:
                lo += ((qh >> (2 * j)) & 1).astype(np.float32) * 16
                hi += ((qh >> (2 * j + 1)) & 1).astype(np.float32) * 16
            d1 = d[:, 0] * sc[:, 2 * j]
            m1 = dmin[:, 0] * m[:, 2 * j]
            d2 = d[:, 0] * sc[:, 2 * j + 1]
            m2 = dmin[:, 0] * m[:, 2 * j + 1]
            out[:, 64 * j:64 * j + 32] = d1[:, None] * lo - m1[:, None]
            out[:, 64 * j + 32:64 * j + 64] = d2[:, None] * hi - m2[:, None]
    elif t == GGMLType.Q6_K:
        ql = b[:, 0:128]
        qh = b[:, 128:192]
        scales = b[:, 192:208].view(np.int8).astype(np.float32)
        d = b[:, 208:210].copy().view(np.float16).astype(np.float32)[:, 0]
        out = np.empty((nb, 256), np.float32)
        for n in range(2):
            l_ = ql[:, 64 * n:64 * n + 64]
            h_ = qh[:, 32 * n:32 * n + 32]
            sc = scales[:, 8 * n:8 * n + 8]
            q1 = ((l_[:, 0:32] & 0xF) | (((h_ >> 0) & 3) << 4)).astype(np.float32) - 32
            q2 = ((l_[:, 32:64] & 0xF) | (((h_ >> 2) & 3) << 4)).astype(np.float32) - 32
            q3 = ((l_[:, 0:32] >> 4) | (((h_ >> 4) & 3) << 4)).astype(np.float32) - 32
            q4 = ((l_[:, 32:64] >> 4) | (((h_ >> 6) & 3) << 4)).astype(np.float32) - 32
            base = 128 * n
            for k, q in enumerate((q1, q2, q3, q4)):
                # 32 weights; scale index is = l/16 -> two scales per 32-run
                s = np.repeat(sc[:, [2 * k, 2 * k + 1]], 16, axis=1)
                out[:, base + 32 * k:base + 32 * k + 32] = d[:, None] * s * q
    else:
        raise NotImplementedError(f"dequantize {t.name}")
    out = out.reshape(-1)
    if n_elements is not None:
        assert out.size == n_elements
    return out

def _dequantize_f16(data, t, n_elements):
    b = _blocks(data, t)
    nb = b.shape[0]
    h = lambda v: np.asarray(v, np.float64).astype(np.float16).astype(np.float64)  # noqa: E731
    if t == GGMLType.Q8_0:
        d = b[:, 0:2].copy().view(np.float16).astype(np.float64)
        q = b[:, 2:34].view(np.int8).astype(np.float64)
        out = h(d * q)
    elif t in (GGMLType.Q4_K, GGMLType.Q5_K):
        d = b[:, 0:2].copy().view(np.float16).astype(np.float64)[:, 0]
        dmin = b[:, 2:4].copy().view(np.float16).astype(np.float64)[:, 0]
        sc, m = _unpack_scale_min_k4(b[:, 4:16])
        qs = b[:, 16:144] if t == GGMLType.Q4_K else b[:, 48:176]
        qh = None if t == GGMLType.Q4_K else b[:, 16:48]
        out = np.empty((nb, 256), np.float64)
        for j in range(4):
            grp = qs[:, 32 * j:32 * j + 32]
            lo = (grp & 0xF).astype(np.float64)
            hi = (grp >> 4).astype(np.float64)
            if qh is not None:
                lo += ((qh >> (2 * j)) & 1).astype(np.float64) * 16
                hi += ((qh >> (2 * j + 1)) & 1).astype(np.float64) * 16
            for half, q in ((0, lo), (1, hi)):
                sb = 2 * j + half
                a = h(d * sc[:, sb])
                mn = h(-dmin * m[:, sb])
                out[:, 64 * j + 32 * half:64 * j + 32 * half + 32] = h(q * a[:, None] + mn[:, None])
    else:  # Q6_K
        ql = b[:, 0:128]
        qh = b[:, 128:192]
        scales = b[:, 192:208].view(np.int8).astype(np.float64)
        d = b[:, 208:210].copy().view(np.float16).astype(np.float64)[:, 0]
        out = np.empty((nb, 256), np.float64)
        for n in range(2):
            l_ = ql[:, 64 * n:64 * n + 64]
            h_ = qh[:, 32 * n:32 * n + 32]
            sc = scales[:, 8 * n:8 * n + 8]
            q1 = ((l_[:, 0:32] & 0xF) | (((h_ >> 0) & 3) << 4)).astype(np.float64) - 32
            q2 = ((l_[:, 32:64] & 0xF) | (((h_ >> 2) & 3) << 4)).astype(np.float64) - 32
            q3 = ((l_[:, 0:32] >> 4) | (((h_ >> 4) & 3) << 4)).astype(np.float64) - 32
            q4 = ((l_[:, 32:64] >> 4) | (((h_ >> 6) & 3) << 4)).astype(np.float64) - 32
            for k, q in enumerate((q1, q2, q3, q4)):
                a = np.repeat(h(d[:, None] * sc[:, [2 * k, 2 * k + 1]]), 16, axis=1)
                out[:, 128 * n + 32 * k:128 * n + 32 * k + 32] = h(q * a)
    out = out.reshape(-1).astype(np.float32)
    if n_elements is not None:
        assert out.size == n_elements
    return out

# --------------------------------------------------------------- quantise


def quantize(x: np.ndarray, ggml_type) -> np.ndarray:
    """Encode float32 (flat, length multiple of the block) -> raw bytes (uint8)."""
    t = GGMLType(ggml_type)
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    if t == GGMLType.F32:
        return x.view(np.uint8).copy()
    if t == GGMLType.F16:
        return x.astype(np.float16).view(np.uint8).copy()
    if t == GGMLType.BF16:
        u = x.view(np.uint32)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        return r.view(np.uint8).copy()
    if t == GGMLType.Q8_0:
        xb = x.reshape(-1, 32)
        amax = np.abs(xb).max(axis=1)
        d = amax / 127.0
        inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0)
        q = np.clip(np.rint(xb * inv[:, None]), -127, 127).astype(np.int8)
        out = np.empty((xb.shape[0], 34), np.uint8)
        out[:, 0:2] = _f16(d).reshape(-1, 1).view(np.uint8)
        out[:, 2:] = q.view(np.uint8)
        return out.reshape(-1)
    if t in (GGMLType.Q4_K, GGMLType.Q5_K):
        nmax = 15 if t == GGMLType.Q4_K else 31
        xb = x.reshape(-1, 8, 32)
        mn = np.minimum(xb.min(axis=2), 0.0)          # [nb,8]  (min <= 0)
        mx = xb.max(axis=2)
        scale = (mx - mn) / nmax                      # per sub-block
        minv = -mn                                    # >= 0
        d = scale.max(axis=1) / 63.0                  # super-block scales
        dmin = minv.max(axis=1) / 63.0
        d16 = _f16(d).astype(np.float32)
        dm16 = _f16(dmin).astype(np.float32)
        sc = np.clip(np.rint(np.where(d16[:, None] > 0, scale / np.where(d16 > 0, d16, 1)[:, None], 0)), 0, 63)
        m = np.clip(np.rint(np.where(dm16[:, None] > 0, minv / np.where(dm16 > 0, dm16, 1)[:, None], 0)), 0, 63)
        eff_s = d16[:, None] * sc
        eff_m = dm16[:, None] * m
        q = np.where(eff_s[:, :, None] > 0,
                     np.rint((xb + eff_m[:, :, None]) / np.where(eff_s > 0, eff_s, 1)[:, :, None]), 0)
        q = np.clip(q, 0, nmax).astype(np.uint8)       # [nb,8,32]
        nb = xb.shape[0]
        packed = _pack_scale_min_k4(sc.astype(np.uint8), m.astype(np.uint8))
        qs = np.empty((nb, 128), np.uint8)
        for j in range(4):
            qs[:, 32 * j:32 * j + 32] = (q[:, 2 * j] & 0xF) | ((q[:, 2 * j + 1] & 0xF) << 4)
        head = np.empty((nb, 4), np.uint8)
        head[:, 0:2] = _f16(d).reshape(-1, 1).view(np.uint8)
        head[:, 2:4] = _f16(dmin).reshape(-1, 1).view(np.uint8)
        if t == GGMLType.Q4_K:
            return np.concatenate([head, packed, qs], axis=1).reshape(-1)
        qh = np.zeros((nb, 32), np.uint8)
        for j in range(8):
            qh |= ((q[:, j] >> 4) & 1).astype(np.uint8) << j
        return np.concatenate([head, packed, qh, qs], axis=1).reshape(-1)
    if t == GGMLType.Q6_K:
        xb = x.reshape(-1, 16, 16)
        amax_idx = np.argmax(np.abs(xb), axis=2)
        vmax = np.take_along_axis(xb, amax_idx[:, :, None], axis=2)[:, :, 0]
        scale = -vmax / 32.0                           # ggml uses the signed max
        smax_idx = np.argmax(np.abs(scale), axis=1)
        smax = np.take_along_axis(scale, smax_idx[:, None], axis=1)[:, 0]
        iscale = np.where(smax != 0, -128.0 / np.where(smax != 0, smax, 1), 0)
        d = np.where(iscale != 0, 1.0 / np.where(iscale != 0, iscale, 1), 0)
        d16 = _f16(d).astype(np.float32)
        sc = np.clip(np.rint(iscale[:, None] * scale), -128, 127).astype(np.int8)
        eff = d16[:, None] * sc.astype(np.float32)
        q = np.where(eff[:, :, None] != 0, np.rint(xb / np.where(eff != 0, eff, 1)[:, :, None]), 0)
        q = (np.clip(q, -32, 31) + 32).astype(np.uint8).reshape(-1, 256)
        nb = q.shape[0]
        ql = np.empty((nb, 128), np.uint8)
        qh = np.empty((nb, 64), np.uint8)
        for n in range(2):
            qq = q[:, 128 * n:128 * n + 128]
            for l in range(32):
                q1, q2, q3, q4 = qq[:, l], qq[:, l + 32], qq[:, l + 64], qq[:, l + 96]
                ql[:, 64 * n + l] = (q1 & 0xF) | ((q3 & 0xF) << 4)
                ql[:, 64 * n + l + 32] = (q2 & 0xF) | ((q4 & 0xF) << 4)
                qh[:, 32 * n + l] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
        out = np.concatenate([ql, qh, sc.view(np.uint8), _f16(d).reshape(-1, 1).view(np.uint8)], axis=1)
        return out.reshape(-1)
    raise NotImplementedError(f"quantize {t.name}")

# ------------------------------------------------------- synthetic blocks


def random_blocks(ggml_type, n_elements: int, rng: np.random.Generator, std: float = 0.02) -> np.ndarray:
    """Valid random blocks of ``ggml_type`` whose decoded weights have roughly
    zero mean and standard deviation ``std`` - generated directly in the block
    domain (random quants + bounded f16 scales), no float->quant pass, so a
    multi-GB synthetic GGUF streams out at memory speed."""
    t = GGMLType(ggml_type)
    bs, bb = GGML_BLOCK[t]
    nb = n_elements // bs
    if t == GGMLType.F32:
        return (rng.standard_normal(n_elements, dtype=np.float32) * std).view(np.uint8)
    if t in (GGMLType.F16, GGMLType.BF16):
        return quantize(rng.standard_normal(n_elements, dtype=np.float32) * std, t)
    raw = np.frombuffer(rng.bytes(nb * bb), dtype=np.uint8).reshape(nb, bb).copy()
    if t == GGMLType.Q8_0:
        # q uniform in [-128,127] -> rms ~73.9
        d = np.full(nb, std / 73.9, np.float32) * rng.uniform(0.5, 1.5, nb).astype(np.float32)
        raw[:, 0:2] = _f16(d).reshape(-1, 1).view(np.uint8)
    elif t in (GGMLType.Q4_K, GGMLType.Q5_K):
        nmax = 15 if t == GGMLType.Q4_K else 31
        # sc, m uniform in [0,63]; q uniform in [0,nmax]. dmin = d*nmax/2 centres w.
        var_sq = (63 * 127 / 6) * (nmax * (2 * nmax + 1) / 6) - (31.5 * nmax / 2) ** 2
        var = var_sq + (nmax / 2) ** 2 * (64 ** 2 - 1) / 12
        d = np.full(nb, std / np.sqrt(var), np.float32) * rng.uniform(0.5, 1.5, nb).astype(np.float32)
        raw[:, 0:2] = _f16(d).reshape(-1, 1).view(np.uint8)
        raw[:, 2:4] = _f16(d * nmax / 2).reshape(-1, 1).view(np.uint8)
    elif t == GGMLType.Q6_K:
        # scales int8 uniform [-128,127] (rms ~73.9); q-32 uniform [-32,31] (rms ~18.5)
        d = np.full(nb, std / (73.9 * 18.5), np.float32) * rng.uniform(0.5, 1.5, nb).astype(np.float32)
        raw[:, 208:210] = _f16(d).reshape(-1, 1).view(np.uint8)
    else:
        raise NotImplementedError(t.name)
    return raw.reshape(-1)
