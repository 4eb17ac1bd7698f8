"""End-to-end facade tests on the float32 reference backend (CPU)."""
import numpy as np
import pytest
from fastapi.testclient import TestClient

from llama_fastapi_k8s_gpu_amd.config import Settings
from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams, filtered_candidates, philox_uniform, sample_token
from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
from llama_fastapi_k8s_gpu_amd.server.app import create_app


@pytest.fixture(scope="module")
def tiny_path(tmp_path_factory):
    return write_synthetic_gguf("tiny-llama3-q4_k_m", str(tmp_path_factory.mktemp("m") / "t.gguf"))


def test_chat_completion_reference(tiny_path):
    llm = Llama(tiny_path, n_ctx=128, backend="reference", seed=1)
    out = llm.create_chat_completion([{"role": "user", "content": "hello"}], max_tokens=8,
                                     temperature=1.2, top_p=0.9, frequency_penalty=0.7, presence_penalty=0.8)
    assert out["object"] == "chat.completion"
    assert isinstance(out["choices"][0]["message"]["content"], str)
    assert 1 <= out["usage"]["completion_tokens"] <= 8


def test_context_overflow_raises(tiny_path):
    llm = Llama(tiny_path, n_ctx=16, backend="reference")
    with pytest.raises(ValueError, match="exceed context window"):
        llm.create_completion("word " * 40, max_tokens=4)


def test_max_tokens_none_fills_context(tiny_path):
    llm = Llama(tiny_path, n_ctx=40, backend="reference", seed=3)
    toks = llm.tokenize(b"hi there", add_bos=True)
    out = llm.create_completion("hi there", max_tokens=None, temperature=0.0)
    # generates until EOG or n_ctx is full
    assert out["usage"]["completion_tokens"] <= 40 - len(toks)
    if out["choices"][0]["finish_reason"] == "length":
        assert out["usage"]["completion_tokens"] == 40 - len(toks)


def test_prefix_reuse_consistent(tiny_path):
    llm = Llama(tiny_path, n_ctx=128, backend="reference")
    a = llm.create_completion("the quick brown fox", max_tokens=6, temperature=0.0)
    b = llm.create_completion("the quick brown fox", max_tokens=6, temperature=0.0)  # reuses KV
    llm.reset()
    c = llm.create_completion("the quick brown fox", max_tokens=6, temperature=0.0)
    assert a["choices"][0]["text"] == b["choices"][0]["text"] == c["choices"][0]["text"]


def test_sampler_chain_semantics():
    rng = np.random.default_rng(0)
    logits = rng.standard_normal(1000).astype(np.float32) * 3
    p = SamplingParams(temperature=1.2, top_k=40, top_p=0.9, min_p=0.05, repeat_penalty=1.1,
                       frequency_penalty=0.7, presence_penalty=0.8, seed=5)
    ids, vals = filtered_candidates(logits, [int(np.argmax(logits))] * 3, p)
    assert len(ids) <= 40 and int(np.argmax(logits)) not in ids[:1]  # penalised top token
    assert np.all(np.diff(vals) <= 0)
    # min-p bound holds on the filtered set (temperature-1 probabilities)
    assert vals[-1] * 1.2 >= vals[0] * 1.2 + np.log(0.05) - 1e-5
    draws = {sample_token(logits, [], p, s) for s in range(200)}
    assert len(draws) > 3
    assert 0.0 <= philox_uniform(123, 7) < 1.0


def test_service_end_to_end_reference(tiny_path):
    s = Settings()
    s.n_ctx = 256
    llm = Llama(tiny_path, n_ctx=256, backend="reference", seed=2)
    app = create_app(s, engine=llm)
    with TestClient(app) as c:
        r = c.post("/response", json={"bot_profile": {"name": "Mia", "appearance": "a,b,c,d"},
                                      "user_profile": {"name": "u"},
                                      "context": [{"turn": "user", "message": "hello there"}]})
        assert r.status_code == 200, r.text
        assert isinstance(r.json()["response"], str)
        assert c.get("/health").json()["engine"]["backend"] == "reference"
