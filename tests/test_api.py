"""T0 - HTTP contract tests against the FakeEngine."""
import asyncio
import logging

import httpx
import pytest
from fastapi.testclient import TestClient

from llama_fastapi_k8s_gpu_amd.config import Settings
from llama_fastapi_k8s_gpu_amd.engine.fake import FakeEngine
from llama_fastapi_k8s_gpu_amd.server.app import create_app
from llama_fastapi_k8s_gpu_amd.server.policy import (count_tokens_roughly, default_system_prompt,
                                                     truncate_messages_to_fit_context)


def body(context=None, name="Mia", appearance="a,b,c,d,e", system_prompt=None):
    bp = {"name": name, "appearance": appearance}
    if system_prompt is not None:
        bp["system_prompt"] = system_prompt
    return {"bot_profile": bp, "user_profile": {"name": "u"},
            "context": context if context is not None else [{"turn": "user", "message": "hi"}]}


def make(mode="echo", **kw):
    s = Settings()
    for k, v in kw.items():
        setattr(s, k, v)
    eng = FakeEngine(mode)
    return create_app(s, engine=eng), eng


def test_response_ok_and_engine_call():
    app, eng = make()
    with TestClient(app) as c:
        r = c.post("/response", json=body([{"turn": "user", "message": "hello"},
                                           {"turn": "assistant", "message": "yo"}]))
    assert r.status_code == 200
    assert r.json() == {"response": "echo: yo"}
    call = eng.calls[0]
    assert call["stream"] is False
    assert call["temperature"] == 1.2 and call["top_p"] == 0.9
    assert call["frequency_penalty"] == 0.7 and call["presence_penalty"] == 0.8
    msgs = call["messages"]
    assert [m["role"] for m in msgs] == ["user", "system", "assistant"]  # index-1 insert


def test_empty_context_puts_system_first():
    app, eng = make()
    with TestClient(app) as c:
        r = c.post("/response", json=body([]))
    assert r.status_code == 200
    assert eng.calls[0]["messages"][0]["role"] == "system"


def test_default_persona_truncated_to_400_chars():
    app, eng = make()
    with TestClient(app) as c:
        c.post("/response", json=body(name="Zoe.f", appearance="1,2,3, tall, blue eyes"))
    sys_msg = eng.calls[0]["messages"][1]["content"]
    full = default_system_prompt("Zoe.f")
    assert len(full) == 423 + len("Zoe.f")
    assert sys_msg == full[:400]
    assert "You a girl." not in sys_msg  # Appendix C6: suffix always cut (preserved)


def test_custom_system_prompt_gender_and_appearance():
    app, eng = make()
    with TestClient(app) as c:
        c.post("/response", json=body(name="Zoe.f", appearance="1,2,3, tall, blue eyes",
                                      system_prompt="Be nice."))
        c.post("/response", json=body(name="Max", appearance="1,2", system_prompt="Be nice."))
    assert eng.calls[0]["messages"][1]["content"] == "Be nice. You a girl. tall blue eyes"
    assert eng.calls[1]["messages"][1]["content"] == "Be nice. You a boy."


def test_truncation_drops_oldest_after_index_1():
    msgs = [{"role": "user", "content": "a" * 1000}, {"role": "system", "content": "s" * 10}]
    msgs += [{"role": "user", "content": f"{i}" * 400} for i in range(12)]
    out = truncate_messages_to_fit_context(msgs, 1024)
    assert all(len(m["content"]) <= 400 for m in out)
    assert sum(count_tokens_roughly(m["content"]) for m in out) <= 1024
    assert out[0]["content"] == "a" * 400 and out[1]["role"] == "system"
    # the survivors are the NEWEST messages
    assert out[-1]["content"] == "b" * 0 + "11" * 200
    assert len(out) == 2 + 9  # 100 + 2 + 9*100 <= 1024


def test_invalid_body_422():
    app, _ = make()
    with TestClient(app) as c:
        r = c.post("/response", json={"bot_profile": {"name": "x"}})
    assert r.status_code == 422


def test_items_route():
    app, _ = make()
    with TestClient(app) as c:
        assert c.get("/items/5").json() == {"item_id": 5}
        assert c.get("/items/abc").status_code == 422
        assert c.get("/docs").status_code == 200
        assert c.get("/openapi.json").status_code == 200


def test_engine_exception_500_nesting():
    app, _ = make("raise:boom")
    with TestClient(app) as c:
        r = c.post("/response", json=body())
    assert r.status_code == 500
    assert r.json()["detail"] == "Internal server error: 500: Error during message generation: boom"


def test_nondict_500_nesting():
    app, _ = make("nondict")
    with TestClient(app) as c:
        r = c.post("/response", json=body())
    assert r.status_code == 500
    assert r.json()["detail"] == ("Internal server error: 500: Error during message generation: "
                                  "500: Unexpected response from model")


def test_multichoice_concatenated():
    app, _ = make("multichoice")
    with TestClient(app) as c:
        r = c.post("/response", json=body())
    resp = r.json()["response"]
    assert resp.startswith("echo: ") and resp.endswith("|second")


async def _concurrent(app, n):
    async with app.router.lifespan_context(app):
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t", timeout=60) as c:
            async def one(i):
                await asyncio.sleep(0.01 * i)  # deterministic arrival order
                return await c.post("/response", json=body([{"turn": "user", "message": str(i)}]))
            return await asyncio.gather(*[one(i) for i in range(n)])


def test_backpressure_503_and_fifo():
    app, eng = make("sleep:0.3", timeout_seconds=20)
    rs = asyncio.run(_concurrent(app, 8))
    codes = [r.status_code for r in rs]
    assert codes.count(200) == 6 and codes.count(503) == 2, codes
    assert rs[7].json() == {"detail": "Server too busy. Please try again later."}
    served = [c["messages"][0]["content"] for c in eng.calls]
    assert served == sorted(served, key=int)  # FIFO


def test_timeout_408_and_cooperative_cancel():
    app, eng = make("sleep:3", timeout_seconds=0.5)
    rs = asyncio.run(_concurrent(app, 3))
    assert [r.status_code for r in rs] == [408, 408, 408]
    assert rs[0].json() == {"detail": "Generation timed out"}
    # queued-then-cancelled futures are skipped, and every generation that did start
    # was stopped early through the cancel event instead of running to completion
    assert 1 <= len(eng.calls) <= 3
    assert eng.cancelled == len(eng.calls) and eng.completed == 0


def test_health_and_metrics():
    app, _ = make()
    with TestClient(app) as c:
        h = c.get("/health")
        assert h.status_code == 200 and h.json()["ready"] is True
        c.post("/response", json=body())
        m = c.get("/metrics").text
    assert 'chat_requests_total{outcome="ok"} 1.0' in m


def test_request_log_line(caplog):
    app, _ = make()
    with caplog.at_level(logging.INFO, logger="api"):
        with TestClient(app) as c:
            c.get("/items/1")
    lines = [r.getMessage() for r in caplog.records if r.name == "api"]
    assert any(l.startswith("Request at ") and "GET http://testserver/items/1 completed in " in l
               and l.endswith("s") for l in lines)


def test_parity_mode_off_keeps_full_system_prompt():
    """PARITY_MODE=0: the system message is exempt from the 400-char cap, so the persona's
    gender / appearance suffix survives (Appendix C6); turns are still capped."""
    app, eng = make(parity_mode=False)
    with TestClient(app) as c:
        c.post("/response", json=body([{"turn": "user", "message": "x" * 900}], name="Zoe.f",
                                      appearance="1,2,3, tall, blue eyes"))
    msgs = eng.calls[0]["messages"]
    assert msgs[1]["content"].endswith("You a girl. tall blue eyes")
    assert len(msgs[0]["content"]) == 400


class _TokenCountingFake(FakeEngine):
    """A fake engine whose 'tokenizer' counts one token per character (worst-case dense
    text: the char/4 estimate undercounts it 4x)."""

    def __init__(self, n_ctx):
        super().__init__("echo")
        self._n = n_ctx

    def n_ctx(self):
        return self._n

    def count_chat_tokens(self, messages):
        return sum(len(m["content"]) + 4 for m in messages)

    def create_chat_completion(self, messages, **kw):
        if self.count_chat_tokens(messages) >= self._n:
            raise ValueError("Requested tokens exceed context window")
        return super().create_chat_completion(messages, **kw)


@pytest.mark.parametrize("guard", [False, True])
def test_exact_token_guard(guard):
    """EXACT_TOKEN_GUARD=1 drops the oldest turns by real token count (never the first two
    messages) so a token-dense prompt fits n_ctx; without it the request 500s as in the
    reference (api.py:35-46)."""
    s = Settings()
    s.exact_token_guard = guard
    s.exact_token_reserve = 16
    eng = _TokenCountingFake(1024)
    ctx = [{"turn": "user" if i % 2 == 0 else "assistant", "message": f"{i}" * 300} for i in range(8)]
    with TestClient(create_app(s, engine=eng)) as c:
        r = c.post("/response", json=body(ctx, system_prompt="S" * 50))
    if not guard:
        assert r.status_code == 500 and "exceed context window" in r.json()["detail"]
        return
    assert r.status_code == 200, r.text
    msgs = eng.calls[-1]["messages"]
    assert eng.count_chat_tokens(msgs) < 1024 - 16
    assert msgs[0]["content"] == "0" * 300 and msgs[1]["role"] == "system"
    assert msgs[-1]["content"] == "7" * 300        # the newest turn survives


def test_exact_token_trim_shortens_last_message():
    from llama_fastapi_k8s_gpu_amd.server.policy import exact_token_trim
    count = lambda ms: sum(len(m["content"]) for m in ms)   # noqa: E731
    msgs = [{"role": "system", "content": "s" * 10}, {"role": "user", "content": "a" * 50 + "b" * 50}]
    out = exact_token_trim(msgs, count, 60)
    assert count(out) == 59 and out[1]["content"].endswith("b" * 49)
    with pytest.raises(ValueError):
        exact_token_trim([{"role": "system", "content": "s" * 80}, {"role": "user", "content": "u"}], count, 60)
    # the reference's order puts the persona at index 1: with [ctx0, system] left, the context
    # message is shortened, never the system prompt
    msgs = [{"role": "user", "content": "c" * 40 + "d" * 40}, {"role": "system", "content": "p" * 30}]
    out = exact_token_trim(msgs, count, 60)
    assert out[1]["content"] == "p" * 30 and out[0]["content"] == "d" * 29 and count(out) == 59
    with pytest.raises(ValueError):   # only the system prompt left: a clear error, not a cut persona
        exact_token_trim([{"role": "system", "content": "p" * 80}], count, 60)


def test_batched_admission_keeps_reference_capacity():
    """MAX_BATCH=6 (the chart default): the reference's capacity (1 in flight + 5 queued = 6
    admitted, reference api.py:19,113,156-160) is kept as a TOTAL cap - the 7th and 8th concurrent
    requests get 503 - while the 6 admitted ones run at once instead of one after another."""
    import time
    app, eng = make("sleep:0.4", timeout_seconds=20, max_batch=6)
    t0 = time.perf_counter()
    rs = asyncio.run(_concurrent(app, 8))
    wall = time.perf_counter() - t0
    codes = [r.status_code for r in rs]
    assert codes[:6] == [200] * 6 and codes[6:] == [503, 503], codes
    assert rs[6].json() == {"detail": "Server too busy. Please try again later."}
    assert len(eng.calls) == 6
    assert wall < 6 * 0.4 * 0.6, wall   # concurrent (a serial run of 6 would take >= 2.4 s)


def test_admission_slot_freed_when_consumer_finishes():
    """An admitted request holds its place until its consumer is done with it: after the
    first wave completes, a new wave of 6 is admitted in full."""
    app, eng = make("sleep:0.2", timeout_seconds=20, max_batch=6)

    async def two_waves():
        async with app.router.lifespan_context(app):
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://t", timeout=60) as c:
                first = await asyncio.gather(*[c.post("/response", json=body()) for _ in range(6)])
                second = await asyncio.gather(*[c.post("/response", json=body()) for _ in range(7)])
                h = (await c.get("/health")).json()
                return first, second, h
    first, second, h = asyncio.run(two_waves())
    assert [r.status_code for r in first] == [200] * 6
    assert sorted(r.status_code for r in second) == [200] * 6 + [503]
    assert h["admitted"] == 0 and h["admission_cap"] == 6


def test_uncapped_admission_mode():
    """MAX_ADMITTED=0: the uncapped form - M generations in flight plus MAX_QUEUE_SIZE waiting."""
    app, eng = make("sleep:0.3", timeout_seconds=20, max_batch=2, max_admitted=0)
    rs = asyncio.run(_concurrent(app, 9))
    codes = [r.status_code for r in rs]
    assert codes.count(200) == 7 and codes.count(503) == 2, codes
