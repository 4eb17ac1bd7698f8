"""Continuous batching end to end on the MI355X: the ``Llama`` facade with
``max_batch > 1`` serves concurrent requests as rows of one batched decode (native
scheduler, csrc/runtime/scheduler.cpp), requests the GPU sampler chain does not cover
still take the single-sequence path meanwhile, cancellation ends a row, and the
FastAPI service with ``MAX_BATCH`` answers concurrent ``/response`` calls."""
import asyncio
import threading

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    d = tmp_path_factory.mktemp("batch_serving")
    return write_synthetic_gguf("tiny-llama3-q4_k_m", str(d / "m.gguf"))


@pytest.fixture(scope="module")
def llm(model):
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    m = Llama(model, n_gpu_layers=-1, n_ctx=256, n_batch=64, seed=1, verbose=False, max_batch=4)
    assert m._backend.sched is not None
    yield m
    m.close()


def _msgs(i):
    return [{"role": "system", "content": "You are terse."},
            {"role": "user", "content": f"request number {i}: count to ten"}]


def test_concurrent_requests_decode_as_one_batch(llm):
    sched = llm._backend.sched
    st0 = sched.stats()
    out, errs = {}, []

    def client(i, k):
        try:
            out[i] = llm.create_chat_completion(_msgs(k), temperature=0.0, max_tokens=24)
        except Exception as e:  # pragma: no cover
            errs.append(e)
    keys = [0, 1, 2, 0, 1, 3]           # two pairs of identical requests
    th = [threading.Thread(target=client, args=(i, k)) for i, k in enumerate(keys)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    assert len(out) == 6
    for i, r in out.items():
        assert r["usage"]["completion_tokens"] <= 24
        assert r["choices"][0]["finish_reason"] in ("stop", "length")
    # identical greedy requests give identical answers whatever else shares the batch
    assert out[0]["choices"][0]["message"]["content"] == out[3]["choices"][0]["message"]["content"]
    assert out[1]["choices"][0]["message"]["content"] == out[4]["choices"][0]["message"]["content"]
    st = sched.stats()
    steps, rows = st["steps"] - st0["steps"], st["rows"] - st0["rows"]
    assert steps > 0 and rows > steps, (steps, rows)   # rows really shared steps
    assert llm.health()["ok"]


def test_host_sampler_request_runs_beside_the_batch(llm):
    """top_k > 64 is outside the GPU chain: the single-sequence host path (slot 0) serves
    it while batched rows run."""
    res, errs = {}, []

    def batched(i):
        try:
            res[i] = llm.create_chat_completion(_msgs(10 + i), temperature=0.8, seed=i, max_tokens=32)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    def host():
        try:
            res["host"] = llm.create_chat_completion(_msgs(99), temperature=0.8, top_k=100, seed=3, max_tokens=8)
        except Exception as e:  # pragma: no cover
            errs.append(e)
    th = [threading.Thread(target=batched, args=(i,)) for i in range(3)] + [threading.Thread(target=host)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    assert res["host"]["usage"]["completion_tokens"] <= 8
    assert all(res[i]["usage"]["completion_tokens"] <= 32 for i in range(3))


def test_cancel_event_ends_a_batched_row(llm):
    ev = threading.Event()
    box = {}

    def run():
        box["r"] = llm.create_chat_completion(_msgs(7), temperature=1.0, seed=5, cancel_event=ev)
    t = threading.Thread(target=run)
    t.start()
    import time
    time.sleep(0.3)
    ev.set()
    t.join(60)
    r = box["r"]
    assert r["choices"][0]["finish_reason"] in ("cancelled", "stop", "length")
    assert r["usage"]["completion_tokens"] < 256


def test_service_max_batch_concurrent_responses(llm):
    import httpx

    from llama_fastapi_k8s_gpu_amd.config import Settings
    from llama_fastapi_k8s_gpu_amd.server.app import create_app
    s = Settings()
    s.max_batch = 4
    s.sampling.max_tokens = 16
    app = create_app(s, engine=llm)
    body = {"bot_profile": {"name": "Ava.f", "appearance": "a, b, c, d"}, "user_profile": {"name": "u"},
            "context": [{"turn": "user", "message": "hello there"}]}

    async def go():
        async with app.router.lifespan_context(app):
            tr = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=tr, base_url="http://t", timeout=120) as c:
                rs = await asyncio.gather(*[c.post("/response", json=body) for _ in range(5)])
                return [r.status_code for r in rs], (await c.get("/health")).json()
    codes, health = asyncio.run(go())
    assert codes == [200] * 5
    assert health["engine"]["batching"]["max_batch"] == 4
