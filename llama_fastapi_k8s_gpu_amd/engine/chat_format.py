"""Chat templating: named formatters + a Jinja2 fallback that renders
the GGUF ``tokenizer.chat_template``.

Format selection mirrors llama-cpp-python's ``guess_chat_format_from_gguf_metadata``
(reached by the reference through api.py:55-63): an exact match on a known
template string selects the named formatter, any other template is rendered with
Jinja2, and no template at all falls back to ``llama-2``.

Named formats return ``(prompt, stop)``. The ``llama-3`` prompt carries no BOS -
it is added by ``tokenize(add_bos=True)`` exactly as upstream does.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Union

from ..gguf.synthetic import LLAMA3_CHAT_TEMPLATE, MISTRAL_CHAT_TEMPLATE

Messages = List[Dict[str, str]]

CHATML_CHAT_TEMPLATE = (
    "{% for message in messages %}{{'<|im_start|>' + message['role'] + '\n' + message['content'] + "
    "'<|im_end|>' + '\n'}}{% endfor %}{% if add_generation_prompt %}{{ '<|im_start|>assistant\n' }}"
    "{% endif %}")


@dataclass
class ChatFormatterResponse:
    prompt: str
    stop: Union[str, List[str], None] = None
    added_special: bool = False  # True when the prompt already contains BOS


def _content(m) -> str:
    c = m.get("content")
    return "" if c is None else str(c)


def format_llama3(messages: Messages) -> ChatFormatterResponse:
    roles = {"system": "<|start_header_id|>system<|end_header_id|>\n\n",
             "user": "<|start_header_id|>user<|end_header_id|>\n\n",
             "assistant": "<|start_header_id|>assistant<|end_header_id|>\n\n"}
    sep = "<|eot_id|>"
    out = ""
    for m in messages:
        role = roles.get(m["role"], f"<|start_header_id|>{m['role']}<|end_header_id|>\n\n")
        c = _content(m)
        out += role + c + sep if c else role
    out += roles["assistant"]
    return ChatFormatterResponse(out, stop=sep)


def format_llama2(messages: Messages) -> ChatFormatterResponse:
    system_template = "<s>[INST] <<SYS>>\n{system_message}\n<</SYS>>"
    sys_msgs = [m for m in messages if m["role"] == "system"]
    system = system_template.format(system_message=_content(sys_msgs[0])) if sys_msgs else "<s>[INST]"
    out = system
    for m in messages:
        if m["role"] == "user":
            out += " " + _content(m) + " [/INST]"
        elif m["role"] == "assistant":
            out += " " + _content(m) + " </s><s>[INST]"
    return ChatFormatterResponse(out, stop="</s>", added_special=True)


def format_chatml(messages: Messages) -> ChatFormatterResponse:
    out = ""
    for m in messages:
        out += f"<|im_start|>{m['role']}\n{_content(m)}<|im_end|>\n"
    out += "<|im_start|>assistant\n"
    return ChatFormatterResponse(out, stop="<|im_end|>")


def format_mistral_instruct(messages: Messages) -> ChatFormatterResponse:
    out = "<s>"
    for m in messages:
        if m["role"] == "user" and m.get("content") is not None:
            out += "[INST] " + _content(m)
        elif m["role"] == "assistant" and m.get("content") is not None:
            out += " [/INST]" + _content(m) + "</s>"
    out += " [/INST]"
    return ChatFormatterResponse(out, stop="</s>", added_special=True)


def format_zephyr(messages: Messages) -> ChatFormatterResponse:
    out = ""
    for m in messages:
        out += f"<|{m['role']}|>\n{_content(m)}</s>\n"
    out += "<|assistant|>\n"
    return ChatFormatterResponse(out, stop="</s>")


FORMATTERS: Dict[str, Callable[[Messages], ChatFormatterResponse]] = {
    "llama-3": format_llama3, "llama-2": format_llama2, "chatml": format_chatml,
    "mistral-instruct": format_mistral_instruct, "zephyr": format_zephyr,
}

KNOWN_TEMPLATES = {LLAMA3_CHAT_TEMPLATE: "llama-3", MISTRAL_CHAT_TEMPLATE: "mistral-instruct",
                   CHATML_CHAT_TEMPLATE: "chatml"}


class Jinja2ChatFormatter:
    def __init__(self, template: str, bos_token: str, eos_token: str):
        import jinja2
        from jinja2.sandbox import ImmutableSandboxedEnvironment
        self.env = ImmutableSandboxedEnvironment(loader=jinja2.BaseLoader(), trim_blocks=True,
                                                 lstrip_blocks=True)
        self.template = self.env.from_string(template)
        self.bos_token, self.eos_token = bos_token, eos_token

    def __call__(self, messages: Messages) -> ChatFormatterResponse:
        def raise_exception(message):
            raise ValueError(message)
        prompt = self.template.render(messages=messages, eos_token=self.eos_token,
                                      bos_token=self.bos_token, raise_exception=raise_exception,
                                      add_generation_prompt=True)
        return ChatFormatterResponse(prompt, stop=[self.eos_token], added_special=True)


def guess_chat_format(metadata: dict) -> Optional[str]:
    tmpl = metadata.get("tokenizer.chat_template")
    if tmpl is None:
        return None
    return KNOWN_TEMPLATES.get(tmpl)


def get_formatter(metadata: dict, chat_format: Optional[str], bos_token: str, eos_token: str):
    if chat_format is None:
        chat_format = guess_chat_format(metadata)
    if chat_format is not None:
        return chat_format, FORMATTERS[chat_format]
    tmpl = metadata.get("tokenizer.chat_template")
    if tmpl:
        return "jinja", Jinja2ChatFormatter(tmpl, bos_token, eos_token)
    return "llama-2", FORMATTERS["llama-2"]
