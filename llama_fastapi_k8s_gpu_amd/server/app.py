"""FastAPI service: ``POST /response`` with FIFO admission, 25 s timeout and
context truncation, plus ``GET /items/{id}``, ``/health`` and ``/metrics``.

Parity map (reference file:line):
  * queue/semaphore created at startup, single consumer task      api.py:110-116
  * consumer skips futures cancelled while queued                  api.py:80-107
  * generation wrapper + error-string nesting                      api.py:48-78
  * /response handler (503 on QueueFull, 408 on timeout, 500)      api.py:118-173
  * /items/{item_id}                                               api.py:175-177
  * request-timing middleware log line                             api.py:179-194

Documented deviations:
  * ``/health`` and ``/metrics`` exist (C2, §5.5);
  * the consumer task handle is retained and cancelled at shutdown (C10);
  * lifespan instead of the deprecated ``on_event`` (C14), same ordering;
  * a timed-out in-flight generation is stopped cooperatively through a
    ``threading.Event`` the engine polls every decode step (C9) - the HTTP
    result (408) is unchanged;
  * OpenAI-compatible ``/v1/*`` routes (``OPENAI_API``, server/openai_api.py) share
    the admission queue and the one-at-a-time consumer.
  * ``EXACT_TOKEN_GUARD=1``: after the reference's char/4 trim, the oldest messages
    are dropped by the real (chat-templated) token count, so a token-dense prompt
    no longer fails at the context limit; ``PARITY_MODE=0`` exempts
    the system message from the 400-char cap (Appendix C6).
  * ``MAX_BATCH=M`` (1 = the reference; the chart ships 6): M consumer tasks and a
    Semaphore(M) feed the engine's continuous batch, so M generations run at once.
    Admission keeps the reference's capacity: at most ``MAX_QUEUE_SIZE + 1`` requests
    (6) are admitted at once, in flight or waiting, and the next one gets 503 - with
    M = 6 every admitted request decodes as a row of one batch instead of waiting its
    turn (``MAX_ADMITTED`` overrides the cap; 0 = M in flight + the queue). An admitted
    request counts until its consumer finishes with it (a timed-out generation still
    running holds its place, as the reference's in-flight thread does). FIFO admission,
    timeouts and error strings are unchanged. M is capped by the engine's
    ``batch_width`` (1 for engines without a batch scheduler).
"""
from __future__ import annotations

import asyncio
import logging
import threading
import time
from contextlib import asynccontextmanager
from datetime import datetime
from typing import Any, Callable, Optional

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, Response

from ..config import Settings
from .policy import build_messages, exact_token_trim, truncate_messages_to_fit_context
from .schema import BotMessageRequest

logging.basicConfig(level=logging.INFO)
# Same logger name as the reference module ("api") so log scrapers keep working.
logger = logging.getLogger("api")


class _Metrics:
    """Prometheus metrics on a private registry (one per app instance)."""

    def __init__(self):
        from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram
        self.registry = CollectorRegistry()
        r = self.registry
        self.requests = Counter("chat_requests_total", "POST /response requests by outcome",
                                ["outcome"], registry=r)
        self.queue_depth = Gauge("chat_queue_depth", "requests waiting in the admission queue",
                                 registry=r)
        self.in_flight = Gauge("chat_in_flight", "generations running", registry=r)
        self.latency = Histogram("chat_response_seconds", "end-to-end /response latency",
                                 buckets=(0.1, 0.25, 0.5, 1, 2, 4, 8, 16, 25, 60), registry=r)
        self.queue_wait = Histogram("chat_queue_wait_seconds", "time from enqueue to generation start",
                                    buckets=(0.001, 0.01, 0.1, 0.5, 1, 2, 5, 10, 25), registry=r)
        self.prompt_tokens = Counter("chat_prompt_tokens_total", "prompt tokens processed", registry=r)
        self.completion_tokens = Counter("chat_completion_tokens_total", "tokens generated", registry=r)
        self.ttft = Histogram("chat_ttft_seconds", "time to first token (prefill)",
                              buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2), registry=r)
        self.decode_tps = Gauge("chat_decode_tokens_per_second", "decode rate of the last request",
                                registry=r)
        self.prefill_tps = Gauge("chat_prefill_tokens_per_second", "prefill rate of the last request",
                                 registry=r)
        self.gpu_mem = Gauge("chat_gpu_memory_bytes", "device memory held by the engine", ["device"],
                             registry=r)

    def observe_engine(self, answer: Any):
        if not isinstance(answer, dict):
            return
        usage = answer.get("usage") or {}
        self.prompt_tokens.inc(usage.get("prompt_tokens", 0) or 0)
        self.completion_tokens.inc(usage.get("completion_tokens", 0) or 0)
        timings = answer.get("timings") or {}
        if timings.get("prefill_s"):
            self.ttft.observe(timings["prefill_s"])
            n = usage.get("prompt_tokens") or 0
            if n:
                self.prefill_tps.set(n / max(timings["prefill_s"], 1e-9))
        if timings.get("decode_s") and usage.get("completion_tokens"):
            self.decode_tps.set(usage["completion_tokens"] / max(timings["decode_s"], 1e-9))


def _default_engine_factory(settings: Settings):
    from ..engine.factory import build_engine
    return build_engine(settings)


def create_app(settings: Optional[Settings] = None, engine: Any = None,
               engine_factory: Optional[Callable[[Settings], Any]] = None) -> FastAPI:
    settings = settings or Settings.from_env()
    factory = engine_factory or _default_engine_factory
    metrics = _Metrics()
    sampling = settings.sampling

    async def try_to_truncate_and_generate(messages, semaphore, cancel_event):
        # reference api.py:48-78 (semaphore redundant with the single consumer; kept)
        async with semaphore:
            try:
                messages = truncate_messages_to_fit_context(
                    messages, settings.max_context_tokens, settings.message_char_cap,
                    cap_system=settings.parity_mode)
                eng = app.state.engine
                kwargs = dict(messages=messages, stream=False,
                              temperature=sampling.temperature, top_p=sampling.top_p,
                              frequency_penalty=sampling.frequency_penalty,
                              presence_penalty=sampling.presence_penalty)
                if sampling.max_tokens is not None:  # parity default None: generate to EOS / context end
                    kwargs["max_tokens"] = sampling.max_tokens
                if settings.cooperative_cancel and getattr(eng, "supports_cancel", False):
                    kwargs["cancel_event"] = cancel_event
                count = getattr(eng, "count_chat_tokens", None)
                if settings.exact_token_guard and count is not None:
                    n_ctx = int(getattr(eng, "n_ctx", lambda: settings.n_ctx)())
                    limit = max(1, n_ctx - settings.exact_token_reserve)

                    def guarded(**kw):   # tokenisation off the event loop, with the generation
                        kw["messages"] = exact_token_trim(kw["messages"], count, limit)
                        return eng.create_chat_completion(**kw)
                    call = guarded
                else:
                    call = eng.create_chat_completion
                metrics.in_flight.inc()
                try:
                    answer = await asyncio.to_thread(call, **kwargs)
                finally:
                    metrics.in_flight.dec()

                if not isinstance(answer, dict):
                    logger.error(f"Unexpected response type: {type(answer)}. Response: {answer}")
                    raise HTTPException(status_code=500, detail="Unexpected response from model")
                metrics.observe_engine(answer)
                response = ''
                for choice in answer.get('choices', []):
                    if 'message' in choice:
                        response += choice['message']['content']
                return response
            except Exception as e:
                logger.error(f"Error during message generation: {str(e)}")
                raise HTTPException(status_code=500, detail=f"Error during message generation: {str(e)}")

    async def consumer(app_: FastAPI):
        # reference api.py:80-107
        queue = app_.state.queue
        semaphore = app_.state.semaphore
        while True:
            request_data = await queue.get()
            metrics.queue_depth.set(queue.qsize())
            messages = request_data.get('messages')
            future = request_data['future']
            if future.cancelled():
                logger.info("Future was cancelled before processing; skipping.")
                queue.task_done()
                _release(app_)
                continue
            metrics.queue_wait.observe(time.monotonic() - request_data['t_enqueue'])
            try:
                job = request_data.get('job')
                if job is not None:   # an OpenAI-route request: same queue, same one-at-a-time
                    async with semaphore:
                        metrics.in_flight.inc()
                        try:
                            response = await asyncio.to_thread(job, app_.state.engine, request_data['cancel'])
                        finally:
                            metrics.in_flight.dec()
                else:
                    response = await try_to_truncate_and_generate(messages, semaphore,
                                                                  request_data['cancel'])
                if not future.cancelled():
                    future.set_result(response)
                else:
                    logger.info("Future was cancelled during processing; result not set.")
            except Exception as e:
                if not future.cancelled():
                    future.set_exception(e)
                else:
                    logger.info("Future was cancelled during processing; exception not set.")
            finally:
                queue.task_done()
                _release(app_)

    def _release(app_: FastAPI):
        app_.state.admitted = max(0, app_.state.admitted - 1)

    def _admit(app_: FastAPI, request_data: dict):
        """Enqueue under the admission cap (503 past it, or when the queue is full)."""
        cap = settings.admission_cap
        if cap and app_.state.admitted >= cap:
            raise asyncio.QueueFull
        app_.state.queue.put_nowait(request_data)
        app_.state.admitted += 1

    @asynccontextmanager
    async def lifespan(app_: FastAPI):
        if getattr(app_.state, "engine", None) is None:
            # The reference loads the model at import (api.py:24-28); we load it
            # before the server accepts traffic, off the event loop.
            app_.state.engine = await asyncio.to_thread(factory, settings)
        # (under the admission cap the queue may hold every admitted request: the cap is the bound)
        cap = settings.admission_cap
        app_.state.queue = asyncio.Queue(maxsize=max(settings.max_queue_size, cap) if cap else settings.max_queue_size)
        app_.state.admitted = 0
        # generations in flight: MAX_BATCH, capped by what the engine actually runs at once
        # (its continuous batch); an engine without a scheduler (CPU, hybrid, a backend that
        # fell back to one row) keeps the reference's one-at-a-time consumer, so requests
        # never wait on a facade lock while their 408 clock runs
        width = max(1, int(settings.max_batch))
        eng_width = getattr(app_.state.engine, "batch_width", None)
        if eng_width is not None:
            width = max(1, min(width, int(eng_width)))
        app_.state.semaphore = asyncio.Semaphore(width)
        app_.state.consumer_tasks = [asyncio.create_task(consumer(app_)) for _ in range(width)]
        app_.state.consumer_task = app_.state.consumer_tasks[0]
        app_.state.ready = True
        try:
            yield
        finally:
            app_.state.ready = False
            for t in app_.state.consumer_tasks:
                t.cancel()
            for t in app_.state.consumer_tasks:
                try:
                    await t
                except (asyncio.CancelledError, Exception):
                    pass
            close = getattr(app_.state.engine, "close", None)
            if close is not None and engine is None:
                await asyncio.to_thread(close)

    app = FastAPI(lifespan=lifespan)
    app.state.engine = engine
    app.state.settings = settings
    app.state.metrics = metrics
    app.state.ready = False

    @app.post("/response")
    async def generate_response(request_body: BotMessageRequest, request: Request):
        # reference api.py:118-173
        t0 = time.monotonic()
        queue = request.app.state.queue
        messages = build_messages(request_body)
        loop = asyncio.get_running_loop()
        future = loop.create_future()
        cancel = threading.Event()
        request_data = {'messages': messages, 'future': future, 'cancel': cancel,
                        't_enqueue': time.monotonic()}
        try:
            _admit(request.app, request_data)
        except asyncio.QueueFull:
            metrics.requests.labels("rejected_503").inc()
            raise HTTPException(status_code=503, detail="Server too busy. Please try again later.")
        metrics.queue_depth.set(queue.qsize())
        try:
            response = await asyncio.wait_for(future, timeout=settings.timeout_seconds)
            metrics.requests.labels("ok").inc()
            metrics.latency.observe(time.monotonic() - t0)
            return {"response": response}
        except asyncio.TimeoutError:
            logger.warning("Generation timed out")
            future.cancel()
            cancel.set()  # cooperative stop of an in-flight generation (C9)
            metrics.requests.labels("timeout_408").inc()
            raise HTTPException(status_code=408, detail="Generation timed out")
        except Exception as e:
            logger.error(f"Internal server error: {str(e)}")
            metrics.requests.labels("error_500").inc()
            raise HTTPException(status_code=500, detail=f"Internal server error: {str(e)}")

    def submit(job, cancel: threading.Event):
        """Enqueue an engine job (OpenAI routes) behind the same FIFO as /response."""
        fut = asyncio.get_running_loop().create_future()
        try:
            _admit(app, {'job': job, 'future': fut, 'cancel': cancel, 't_enqueue': time.monotonic()})
        except asyncio.QueueFull:
            metrics.requests.labels("rejected_503").inc()
            raise HTTPException(status_code=503, detail="Server too busy. Please try again later.")
        metrics.queue_depth.set(app.state.queue.qsize())
        return fut

    if settings.openai_api:
        from .openai_api import add_openai_routes
        add_openai_routes(app, settings, metrics, submit,
                          lambda: getattr(app.state.engine, "model_path", None) or settings.model_file)

    @app.get("/items/{item_id}")
    async def read_item(item_id: int):
        return {"item_id": item_id}

    @app.get("/health")
    async def health(request: Request):
        st = request.app.state
        eng = getattr(st, "engine", None)
        info = {"status": "ok", "ready": bool(getattr(st, "ready", False)) and eng is not None}
        q = getattr(st, "queue", None)
        info["queue_depth"] = q.qsize() if q is not None else 0
        info["admitted"] = int(getattr(st, "admitted", 0))
        info["admission_cap"] = settings.admission_cap
        healthy = True
        if eng is not None and hasattr(eng, "health"):
            try:
                h = eng.health()
                info["engine"] = h
                healthy = bool(h.get("ok", True))
            except Exception as e:  # engine fault => pod restart via liveness probe
                info["engine"] = {"ok": False, "error": str(e)}
                healthy = False
        if not healthy or not info["ready"]:
            info["status"] = "unhealthy" if not healthy else "starting"
            return JSONResponse(status_code=503, content=info)
        return info

    @app.get("/health/live")
    async def health_live(request: Request):
        """Liveness: the process serves HTTP and the engine has not faulted (a model
        still loading is alive; readiness is ``/health``)."""
        eng = getattr(request.app.state, "engine", None)
        if eng is not None and hasattr(eng, "health"):
            try:
                h = eng.health()
                if not h.get("ok", True):
                    return JSONResponse(status_code=503, content={"status": "unhealthy", "engine": h})
            except Exception as e:
                return JSONResponse(status_code=503, content={"status": "unhealthy", "error": str(e)})
        return {"status": "alive"}

    @app.get("/metrics")
    async def metrics_endpoint(request: Request):
        from prometheus_client import CONTENT_TYPE_LATEST, generate_latest
        eng = getattr(request.app.state, "engine", None)
        mem = getattr(eng, "device_memory", None)
        if callable(mem):
            try:
                for dev, nbytes in mem().items():
                    metrics.gpu_mem.labels(str(dev)).set(nbytes)
            except Exception:
                pass
        return Response(generate_latest(metrics.registry), media_type=CONTENT_TYPE_LATEST)

    @app.middleware("http")
    async def log_request_time(request: Request, call_next):
        # reference api.py:179-194
        start_time = time.time()
        response = await call_next(request)
        time_of_day = datetime.now().strftime("%Y-%m-%d %H:%M:%S")
        process_time = time.time() - start_time
        formatted_time = f"{process_time:.4f}s"
        logger.info(f"Request at {time_of_day}: {request.method} {request.url} completed in {formatted_time}")
        return response

    return app
