"""FakeEngine: the test double for the API layer.

Mirrors the ``Llama.create_chat_completion`` contract the service relies on
(reference api.py:55-74) and can be driven into every failure path the
reference handles: slow generation (408), exceptions (500), non-dict results
(500 with the nested detail string), and back-pressure (503).

Mode string (``FAKE_ENGINE_MODE`` env or constructor):
  ``echo``            -> returns "echo: <last user content>"
  ``sleep:<sec>``     -> sleeps, then echoes (cooperatively cancellable)
  ``raise:<message>`` -> raises RuntimeError(message)
  ``nondict``         -> returns a string instead of a dict
  ``multichoice``     -> two choices; the route concatenates both
"""
from __future__ import annotations

import os
import threading
import time
from typing import Any, Dict, List, Optional


class FakeEngine:
    supports_cancel = True

    def __init__(self, mode: Optional[str] = None):
        self.mode = mode or os.environ.get("FAKE_ENGINE_MODE", "echo")
        self.calls: List[Dict[str, Any]] = []
        self.completed = 0
        self.cancelled = 0
        self._lock = threading.Lock()

    def health(self) -> Dict[str, Any]:
        return {"ok": True, "engine": "fake", "mode": self.mode}

    def create_chat_completion(self, messages, stream=False, temperature=0.8, top_p=0.95,
                               frequency_penalty=0.0, presence_penalty=0.0,
                               cancel_event: Optional[threading.Event] = None, **kw):
        with self._lock:
            self.calls.append({"messages": [dict(m) for m in messages], "stream": stream,
                               "temperature": temperature, "top_p": top_p,
                               "frequency_penalty": frequency_penalty,
                               "presence_penalty": presence_penalty, **kw})
        mode = self.mode
        if mode.startswith("sleep:"):
            dur = float(mode.split(":", 1)[1])
            t_end = time.monotonic() + dur
            while time.monotonic() < t_end:
                if cancel_event is not None and cancel_event.is_set():
                    with self._lock:
                        self.cancelled += 1
                    return {"id": "chatcmpl-fake", "object": "chat.completion",
                            "created": int(time.time()), "model": "fake",
                            "choices": [{"index": 0, "finish_reason": "cancelled",
                                         "message": {"role": "assistant", "content": ""}}],
                            "usage": {"prompt_tokens": 0, "completion_tokens": 0,
                                      "total_tokens": 0}}
                time.sleep(min(0.01, max(0.0, t_end - time.monotonic())))
        elif mode.startswith("raise:"):
            raise RuntimeError(mode.split(":", 1)[1])
        elif mode == "nondict":
            return "not a dict"
        last = messages[-1]["content"] if messages else ""
        with self._lock:
            self.completed += 1
        choices = [{"index": 0, "message": {"role": "assistant", "content": f"echo: {last}"},
                    "finish_reason": "stop"}]
        if mode == "multichoice":
            choices.append({"index": 1, "message": {"role": "assistant", "content": "|second"},
                            "finish_reason": "stop"})
        return {"id": "chatcmpl-fake", "object": "chat.completion", "created": int(time.time()),
                "model": "fake", "choices": choices,
                "usage": {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}}
