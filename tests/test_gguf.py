"""T1 - GGUF container round trip and ggml block formats."""
import numpy as np
import pytest

from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType
from llama_fastapi_k8s_gpu_amd.gguf.quants import dequantize, quantize, random_blocks, _pack_scale_min_k4, _unpack_scale_min_k4
from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
from llama_fastapi_k8s_gpu_amd.gguf.synthetic import SPECS, tensor_types, use_more_bits, write_synthetic_gguf
from llama_fastapi_k8s_gpu_amd.gguf.writer import GGUFWriter


def _scalar_q4k(block: bytes):
    """Literal transcription of the ggml Q4_K decode loop (per-element)."""
    import struct
    d, dmin = np.frombuffer(block[0:4], np.float16).astype(np.float32)
    q = block[4:16]
    qs = block[16:144]

    def gsm(j):
        if j < 4:
            return q[j] & 63, q[j + 4] & 63
        return (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4), (q[j + 4] >> 4) | ((q[j] >> 6) << 4)
    y = []
    for j in range(4):
        s1, m1 = gsm(2 * j)
        s2, m2 = gsm(2 * j + 1)
        y += [d * s1 * (qs[32 * j + l] & 0xF) - dmin * m1 for l in range(32)]
        y += [d * s2 * (qs[32 * j + l] >> 4) - dmin * m2 for l in range(32)]
    return np.array(y, np.float32)


def test_scale_min_pack_roundtrip():
    rng = np.random.default_rng(0)
    sc = rng.integers(0, 64, (100, 8)).astype(np.uint8)
    m = rng.integers(0, 64, (100, 8)).astype(np.uint8)
    s2, m2 = _unpack_scale_min_k4(_pack_scale_min_k4(sc, m))
    assert (s2 == sc).all() and (m2 == m).all()


def test_q4k_vectorised_matches_scalar_decode():
    rng = np.random.default_rng(1)
    raw = random_blocks(GGMLType.Q4_K, 256 * 4, rng)
    vec = dequantize(raw, GGMLType.Q4_K)
    for b in range(4):
        ref = _scalar_q4k(bytes(raw[144 * b:144 * (b + 1)]))
        np.testing.assert_allclose(vec[256 * b:256 * (b + 1)], ref, rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("t,tol", [(GGMLType.Q8_0, 0.01), (GGMLType.Q4_K, 0.12), (GGMLType.Q5_K, 0.06),
                                   (GGMLType.Q6_K, 0.03), (GGMLType.F16, 1e-3), (GGMLType.BF16, 1e-2)])
def test_quantize_dequantize_error(t, tol):
    rng = np.random.default_rng(2)
    x = rng.standard_normal(256 * 64).astype(np.float32)
    y = dequantize(quantize(x, t), t)
    rel = np.sqrt(np.mean((y - x) ** 2)) / np.sqrt(np.mean(x ** 2))
    assert rel < tol, rel


@pytest.mark.parametrize("t", [GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K])
def test_random_blocks_statistics(t):
    rng = np.random.default_rng(3)
    y = dequantize(random_blocks(t, 256 * 512, rng, std=0.02), t)
    assert np.isfinite(y).all()
    assert 0.01 < y.std() < 0.04, y.std()
    assert abs(y.mean()) < 0.01


def test_q4_k_m_mix_rule():
    spec = SPECS["llama3-8b-q4_k_m"]
    bumped = [i for i in range(32) if use_more_bits(i, 32)]
    assert bumped == [0, 1, 2, 3, 6, 9, 12, 15, 18, 21, 24, 27, 28, 29, 30, 31]
    assert tensor_types(spec, 0)["attn_v"] == GGMLType.Q6_K
    assert tensor_types(spec, 4)["attn_v"] == GGMLType.Q4_K
    assert tensor_types(SPECS["llama3-70b-q4_k_m"], 20)["attn_v"] == GGMLType.Q5_K
    assert tensor_types(SPECS["mixtral-8x7b-q4_k_m"], 5)["attn_k"] == GGMLType.Q8_0


def test_writer_reader_roundtrip(tmp_path):
    p = str(tmp_path / "t.gguf")
    w = GGUFWriter(p)
    w.add("general.architecture", "llama")
    w.add("x.u32", 7)
    w.add("x.f32", 1.5)
    w.add("x.bool", True)
    w.add("x.arr_s", ["a", "bé", ""])
    w.add("x.arr_i", [1, -2, 3])
    rng = np.random.default_rng(0)
    a = rng.standard_normal(64).astype(np.float32)
    qb = random_blocks(GGMLType.Q4_K, 512, rng)
    w.declare_tensor("a", GGMLType.F32, (64,))
    w.declare_tensor("b", GGMLType.Q4_K, (256, 2))
    w.begin()
    w.write_tensor_data(a)
    w.write_tensor_data(qb)
    w.close()
    r = GGUFReader(p)
    assert r.metadata["x.u32"] == 7 and r.metadata["x.f32"] == 1.5 and r.metadata["x.bool"] is True
    assert r.metadata["x.arr_s"] == ["a", "bé", ""] and r.metadata["x.arr_i"] == [1, -2, 3]
    assert r.tensors["b"].offset % 32 == 0
    np.testing.assert_array_equal(r.dequant("a"), a)
    assert r.dequant("b").shape == (2, 256)
    np.testing.assert_array_equal(np.asarray(r.raw("b")), qb)


def test_synthetic_tiny_model(tmp_path):
    p = write_synthetic_gguf("tiny-llama3-mixed", str(tmp_path / "m.gguf"))
    r = GGUFReader(p)
    assert r.metadata["general.architecture"] == "llama"
    assert r.metadata["llama.block_count"] == 4
    types = {r.tensors[f"blk.0.{n}.weight"].ggml_type for n in ("attn_q", "attn_k", "attn_v", "attn_output")}
    assert types == {int(GGMLType.Q4_K), int(GGMLType.Q5_K), int(GGMLType.Q6_K), int(GGMLType.Q8_0)}
    emb = r.dequant("token_embd.weight")
    assert emb.shape == (len(r.metadata["tokenizer.ggml.tokens"]), 256)
    assert np.isfinite(emb).all()
