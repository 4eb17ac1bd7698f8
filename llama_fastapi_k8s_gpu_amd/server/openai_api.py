"""OpenAI-compatible routes (``/v1/models``, ``/v1/completions``, ``/v1/chat/completions``,
with server-sent-event streaming) over the same engine and the same admission queue as
``POST /response``.

The reference exposes only ``/response`` (reference api.py:118-173); its engine library
(llama-cpp-python 0.2.77) ships this API as ``llama_cpp.server``. Here the
routes are an extension (``OPENAI_API=1``, default on) that keeps the reference's serving
semantics: requests wait in the one FIFO queue (503 when it is full), run one at a time,
and a non-streaming request that does not finish within ``TIMEOUT_SECONDS`` gets 408 and
its generation is cancelled cooperatively. A streaming request is bounded by the timeout
until its first chunk; a client that disconnects mid-stream cancels the generation.
"""
from __future__ import annotations

import asyncio
import json
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Union

from fastapi.responses import JSONResponse, StreamingResponse
from pydantic import BaseModel, ConfigDict


class _Base(BaseModel):
    model_config = ConfigDict(extra="allow")
    model: Optional[str] = None
    max_tokens: Optional[int] = 16
    temperature: float = 0.8
    top_p: float = 0.95
    top_k: int = 40
    min_p: float = 0.05
    typical_p: float = 1.0
    tfs_z: float = 1.0
    stop: Optional[Union[str, List[str]]] = None
    stream: bool = False
    seed: Optional[int] = None
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repeat_penalty: float = 1.1
    logit_bias: Optional[Dict[str, float]] = None
    mirostat_mode: int = 0
    mirostat_tau: float = 5.0
    mirostat_eta: float = 0.1
    n: int = 1
    user: Optional[str] = None
    grammar: Optional[str] = None        # GBNF text (llama-cpp-python server extension)


class CompletionRequest(_Base):
    prompt: Union[str, List[str], List[int]] = ""
    logprobs: Optional[int] = None
    echo: bool = False
    suffix: Optional[str] = None


class ChatCompletionRequest(_Base):
    messages: List[Dict[str, Any]]
    max_tokens: Optional[int] = None
    logprobs: bool = False
    top_logprobs: Optional[int] = None
    response_format: Optional[Dict[str, Any]] = None


def _error(status: int, message: str, typ: str = "invalid_request_error"):
    return JSONResponse(status_code=status, content={"error": {"message": message, "type": typ, "param": None,
                                                               "code": None}})


def _sampling_kwargs(req: _Base) -> Dict[str, Any]:
    kw = dict(temperature=req.temperature, top_p=req.top_p, top_k=req.top_k, min_p=req.min_p,
              typical_p=req.typical_p, tfs_z=req.tfs_z, stop=req.stop, seed=req.seed,
              presence_penalty=req.presence_penalty, frequency_penalty=req.frequency_penalty,
              repeat_penalty=req.repeat_penalty, mirostat_mode=req.mirostat_mode,
              mirostat_tau=req.mirostat_tau, mirostat_eta=req.mirostat_eta, max_tokens=req.max_tokens)
    if req.logit_bias:
        kw["logit_bias"] = {int(k): float(v) for k, v in req.logit_bias.items()}
    return kw


def _text_content(content: Any) -> str:
    """OpenAI message content: a string or a list of typed parts (text parts joined)."""
    if content is None:
        return ""
    if isinstance(content, str):
        return content
    return "".join(p.get("text", "") for p in content if isinstance(p, dict) and p.get("type", "text") == "text")


def add_openai_routes(app, settings, metrics, submit: Callable[[Callable, threading.Event], "asyncio.Future"],
                      model_name: Callable[[], str]):
    """``submit(job, cancel)`` enqueues ``job(engine, cancel)`` (run in a worker thread by the
    admission consumer) and returns the future of its result; it raises HTTPException(503)
    when the queue is full."""

    @app.get("/v1/models")
    async def list_models():
        return {"object": "list", "data": [{"id": model_name(), "object": "model", "owned_by": "me",
                                            "permissions": []}]}

    async def _run(req: _Base, call: Callable[[Any, Dict[str, Any]], Any]):
        if req.n != 1:
            return _error(400, "n > 1 is not supported")
        cancel = threading.Event()
        kw = _sampling_kwargs(req)
        t0 = time.monotonic()
        if not req.stream:
            def job(eng, cancel_event):
                if getattr(eng, "supports_cancel", False):
                    kw["cancel_event"] = cancel_event
                return call(eng, kw)
            fut = submit(job, cancel)
            try:
                out = await asyncio.wait_for(fut, timeout=settings.timeout_seconds)
            except asyncio.TimeoutError:
                fut.cancel()
                cancel.set()
                metrics.requests.labels("timeout_408").inc()
                return _error(408, "Generation timed out", "timeout")
            except ValueError as e:       # e.g. prompt longer than the context window, bad grammar
                metrics.requests.labels("error_400").inc()
                return _error(400, str(e))
            except NotImplementedError as e:
                metrics.requests.labels("error_400").inc()
                return _error(400, str(e))
            except Exception as e:
                metrics.requests.labels("error_500").inc()
                return _error(500, f"Internal server error: {e}", "server_error")
            metrics.requests.labels("ok").inc()
            metrics.latency.observe(time.monotonic() - t0)
            metrics.observe_engine(out)
            return out

        loop = asyncio.get_running_loop()
        chunks: "asyncio.Queue" = asyncio.Queue()
        done = object()

        def job(eng, cancel_event):
            if getattr(eng, "supports_cancel", False):
                kw["cancel_event"] = cancel_event
            try:
                for ch in call(eng, dict(kw, stream=True)):
                    loop.call_soon_threadsafe(chunks.put_nowait, ch)
            except BaseException as e:
                loop.call_soon_threadsafe(chunks.put_nowait, e)
            finally:
                loop.call_soon_threadsafe(chunks.put_nowait, done)
            return None
        fut = submit(job, cancel)
        try:
            first = await asyncio.wait_for(chunks.get(), timeout=settings.timeout_seconds)
        except asyncio.TimeoutError:
            fut.cancel()
            cancel.set()
            metrics.requests.labels("timeout_408").inc()
            return _error(408, "Generation timed out", "timeout")
        if isinstance(first, BaseException):
            metrics.requests.labels("error_400" if isinstance(first, (ValueError, NotImplementedError))
                                    else "error_500").inc()
            return _error(400 if isinstance(first, (ValueError, NotImplementedError)) else 500, str(first))

        async def sse():
            item = first
            try:
                while item is not done:
                    if isinstance(item, BaseException):
                        yield f"data: {json.dumps({'error': {'message': str(item), 'type': 'server_error'}})}\n\n"
                        break
                    yield f"data: {json.dumps(item)}\n\n"
                    item = await chunks.get()
                yield "data: [DONE]\n\n"
                metrics.requests.labels("ok").inc()
                metrics.latency.observe(time.monotonic() - t0)
            finally:
                cancel.set()      # client gone (or finished): stop the generation if still running
        return StreamingResponse(sse(), media_type="text/event-stream")

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        prompt = req.prompt
        if isinstance(prompt, list) and prompt and isinstance(prompt[0], str):
            if len(prompt) != 1:
                return _error(400, "batched prompts are not supported")
            prompt = prompt[0]

        def call(eng, kw):
            extra = {"grammar": req.grammar} if req.grammar else {}
            return eng.create_completion(prompt, logprobs=req.logprobs, echo=req.echo, suffix=req.suffix, **extra,
                                         **kw)
        return await _run(req, call)

    @app.post("/v1/chat/completions")
    async def chat_completions(req: ChatCompletionRequest):
        messages = [{"role": m.get("role", "user"), "content": _text_content(m.get("content"))}
                    for m in req.messages]

        def call(eng, kw):
            extra = {}
            if req.logprobs:
                extra = {"logprobs": True, "top_logprobs": req.top_logprobs}
            if req.response_format:
                extra["response_format"] = req.response_format
            if req.grammar:
                extra["grammar"] = req.grammar
            return eng.create_chat_completion(messages=messages, **extra, **kw)
        return await _run(req, call)
