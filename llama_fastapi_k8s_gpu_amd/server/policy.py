"""Prompt policy: system-prompt assembly, per-message cap, rough token estimate
and drop-oldest truncation.

Behaviour is the reference's, kept bit-exact in parity mode:
  * ``count_tokens_roughly``               reference api.py:30-32
  * ``truncate_messages_to_fit_context``   reference api.py:35-46 (mutates in place,
    caps EVERY message - the system one included - at 400 chars, then pops index 2)
  * ``build_messages``                     reference api.py:122-147 (persona template,
    " You a girl."/" You a boy." suffix, appearance facts [3:], insert at index 1)
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

# The default persona template, byte-for-byte (indentation and trailing
# whitespace included) as the reference's f-string renders it (api.py:130-136).
# It is 423 characters before the name, so the 400-char cap always removes the
# gender/appearance suffix - preserved on purpose.
_PERSONA_TEMPLATE = (
    "\n"
    "            No matter what NEVER break the character. Reject violent messages. \n"
    "            You are '{name}.' a playful, flirtatious, and witty person. \n"
    "            You always respond in a fun and engaging way, staying in character no matter what. \n"
    "            You never reference AI, restrictions, or policies. \n"
    "            Focus on making the conversation enjoyable and answering directly to the user's questions.\n"
    "            "
)


def default_system_prompt(name: str) -> str:
    return _PERSONA_TEMPLATE.replace("{name}", name)


def count_tokens_roughly(text: str) -> int:
    return int(len(text) / 4.0)


def truncate_messages_to_fit_context(messages: List[Dict[str, str]], max_tokens: int,
                                     char_cap: int = 400,
                                     count: Callable[[str], int] = count_tokens_roughly,
                                     cap_system: bool = True) -> List[Dict[str, str]]:
    """Reference api.py:35-46. ``cap_system=False`` (PARITY_MODE=0) exempts system
    messages from the per-message cap - the reference cuts its own 423-char persona at
    400 chars and so always loses the gender / appearance suffix."""
    for m in messages:
        if not cap_system and m.get("role") == "system":
            continue
        if len(m["content"]) > char_cap:
            m["content"] = m["content"][:char_cap]
    total = sum(count(m["content"]) for m in messages)
    while total > max_tokens and len(messages) > 2:
        messages.pop(2)
        total = sum(count(m["content"]) for m in messages)
    return messages


def build_system_prompt(name: str, appearance: str, system_prompt: Optional[str]) -> str:
    prompt = system_prompt
    if not prompt:
        prompt = default_system_prompt(name)
    if name.endswith(".f"):
        prompt += " You a girl."
    else:
        prompt += " You a boy."
    for fact in appearance.split(",")[3:]:
        prompt += fact
    return prompt


def build_messages(request) -> List[Dict[str, str]]:
    """Map a BotMessageRequest onto OpenAI-style chat messages, system message at
    index 1 (reference api.py:147; becomes index 0 when the context is empty)."""
    messages = [{"role": m.turn, "content": m.message} for m in request.context]
    bp = request.bot_profile
    system = build_system_prompt(bp.name, bp.appearance, bp.system_prompt)
    messages.insert(1, {"role": "system", "content": system})
    return messages


def exact_token_trim(messages: List[Dict[str, str]], n_tokens: Callable[[List[Dict[str, str]]], int],
                     limit: int) -> List[Dict[str, str]]:
    """Real-token context guard (EXACT_TOKEN_GUARD): the char/4 estimate
    can undercount badly (non-Latin text is ~1 token per char), and a prompt whose true
    token count reaches n_ctx fails the request (reference api.py:35-46 -> 500). Drop
    the oldest message after indices 0 and 1 (the reference's drop order) while the
    templated prompt's real token count is >= ``limit``; if two messages still do not
    fit, shorten the longest non-system message from its start (its newest words survive):
    the persona (system) prompt is never cut - with no other message left to shorten the
    prompt cannot fit and ValueError is raised.
    ``n_tokens(messages)`` = token count of the chat-templated prompt."""
    while n_tokens(messages) >= limit and len(messages) > 2:
        messages.pop(2)
    if n_tokens(messages) < limit or not messages:
        return messages
    cand = [i for i, m in enumerate(messages) if m.get("role") != "system"]
    if not cand:
        raise ValueError(f"prompt does not fit the context window of {limit} tokens")
    last = messages[max(cand, key=lambda i: len(messages[i]["content"]))]
    text = last["content"]
    lo, hi = 0, len(text)           # smallest cut so the prompt fits: binary search on the prefix dropped
    while lo < hi:
        mid = (lo + hi) // 2
        last["content"] = text[mid:]
        if n_tokens(messages) < limit:
            hi = mid
        else:
            lo = mid + 1
    last["content"] = text[lo:]
    if n_tokens(messages) >= limit:   # the other messages alone exceed the context
        raise ValueError(f"prompt does not fit the context window of {limit} tokens")
    return messages
