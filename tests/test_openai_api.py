"""OpenAI-compatible routes (server/openai_api.py): /v1/models, /v1/completions and
/v1/chat/completions, plain and server-sent-event streaming, over the real Llama facade
(C++ CPU backend, tiny synthetic model) and the shared admission queue."""
import asyncio
import json

import httpx
import pytest
from fastapi.testclient import TestClient

from llama_fastapi_k8s_gpu_amd.config import Settings
from llama_fastapi_k8s_gpu_amd.engine.fake import FakeEngine
from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
from llama_fastapi_k8s_gpu_amd.server.app import create_app


@pytest.fixture(scope="module")
def llm(tmp_path_factory):
    d = tmp_path_factory.mktemp("oai_models")
    path = write_synthetic_gguf("tiny-llama3-q4_k_m", str(d / "m.gguf"))
    return Llama(path, n_ctx=256, backend="cpu", seed=0, n_threads=2, verbose=False)


@pytest.fixture()
def client(llm):
    llm.reset()
    app = create_app(Settings(), engine=llm)
    with TestClient(app) as c:
        yield c


def _sse(text):
    out = []
    for line in text.splitlines():
        if line.startswith("data: "):
            out.append(line[6:])
    assert out[-1] == "[DONE]"
    return [json.loads(x) for x in out[:-1]]


def test_models_and_completion(client):
    m = client.get("/v1/models").json()
    assert m["object"] == "list" and m["data"][0]["object"] == "model"
    r = client.post("/v1/completions", json={"prompt": "the quick brown", "max_tokens": 6, "temperature": 0})
    assert r.status_code == 200, r.text
    j = r.json()
    assert j["object"] == "text_completion" and 1 <= j["usage"]["completion_tokens"] <= 6
    # streaming yields the same greedy text, then [DONE]
    r2 = client.post("/v1/completions", json={"prompt": "the quick brown", "max_tokens": 6, "temperature": 0,
                                              "stream": True})
    assert r2.status_code == 200 and r2.headers["content-type"].startswith("text/event-stream")
    chunks = _sse(r2.text)
    assert "".join(c["choices"][0]["text"] for c in chunks) == j["choices"][0]["text"]
    assert chunks[-1]["choices"][0]["finish_reason"] in ("stop", "length")


def test_chat_completion_stream_logprobs_and_bias(client, llm):
    body = {"messages": [{"role": "user", "content": [{"type": "text", "text": "hello"}]}], "max_tokens": 5,
            "temperature": 0, "logprobs": True, "top_logprobs": 2}
    r = client.post("/v1/chat/completions", json=body)
    assert r.status_code == 200, r.text
    j = r.json()
    msg = j["choices"][0]["message"]
    assert msg["role"] == "assistant" and j["object"] == "chat.completion"
    assert all(len(e["top_logprobs"]) == 2 for e in j["choices"][0]["logprobs"]["content"])
    r2 = client.post("/v1/chat/completions", json=dict(body, stream=True, logprobs=False))
    chunks = _sse(r2.text)
    assert chunks[0]["choices"][0]["delta"].get("role") == "assistant"
    assert "".join(c["choices"][0]["delta"].get("content", "") for c in chunks) == msg["content"]
    # logit_bias keys arrive as strings (JSON): token 42 forced
    r3 = client.post("/v1/completions", json={"prompt": "x", "max_tokens": 3, "temperature": 0,
                                              "logit_bias": {"42": 100}})
    assert r3.json()["choices"][0]["text"] == llm.detokenize([42] * 3).decode("utf-8", errors="replace")


def test_openai_errors(client):
    assert client.post("/v1/completions", json={"prompt": "x", "n": 2}).status_code == 400
    r = client.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "x"}],
                                                  "response_format": {"type": "xml"}})
    assert r.status_code == 400 and "error" in r.json()
    r = client.post("/v1/completions", json={"prompt": "x", "grammar": "root ::= missing"})
    assert r.status_code == 400 and "undefined rule" in r.json()["error"]["message"]
    r = client.post("/v1/completions", json={"prompt": "word " * 400, "max_tokens": 4})
    assert r.status_code == 400 and "context window" in r.json()["error"]["message"]
    assert client.post("/v1/completions", json={"prompt": "hi", "max_tokens": 2, "stop": ["\n"]}).status_code == 200


def test_openai_routes_share_the_admission_queue():
    """/response traffic and /v1 traffic queue behind one another: with a slow engine,
    the 7th concurrent request is rejected with 503 whichever route it used."""
    s = Settings()
    s.timeout_seconds = 20
    eng = FakeEngine("sleep:0.3")
    app = create_app(s, engine=eng)

    async def go():
        async with app.router.lifespan_context(app):
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://t", timeout=60) as c:
                async def one(i):
                    await asyncio.sleep(0.01 * i)
                    if i % 2:
                        return await c.post("/v1/chat/completions",
                                            json={"messages": [{"role": "user", "content": str(i)}]})
                    return await c.post("/response", json={"bot_profile": {"name": "a", "appearance": "a,b,c,d"},
                                                           "user_profile": {"name": "u"},
                                                           "context": [{"turn": "user", "message": str(i)}]})
                return await asyncio.gather(*[one(i) for i in range(8)])
    rs = asyncio.run(go())
    codes = [r.status_code for r in rs]
    assert codes.count(200) == 6 and codes.count(503) == 2, codes
    assert len(eng.calls) == 6


def test_openai_api_can_be_disabled(llm):
    s = Settings()
    s.openai_api = False
    app = create_app(s, engine=llm)
    with TestClient(app) as c:
        assert c.get("/v1/models").status_code == 404


def test_json_mode_and_grammar_routes(client):
    r = client.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "give json"}], "max_tokens": 40, "temperature": 0.5, "seed": 3,
        "response_format": {"type": "json_schema", "json_schema": {"name": "x", "schema": {
            "type": "object", "properties": {"ok": {"type": "boolean"}}, "required": ["ok"]}}}})
    assert r.status_code == 200, r.text
    text = r.json()["choices"][0]["message"]["content"]
    assert text.startswith("{")
    if r.json()["choices"][0]["finish_reason"] == "stop":
        assert isinstance(json.loads(text)["ok"], bool)
    r = client.post("/v1/completions", json={"prompt": "n:", "max_tokens": 6, "temperature": 0.8,
                                             "grammar": "root ::= [0-9]{1,3}"})
    assert r.status_code == 200 and r.json()["choices"][0]["text"].isdigit()
