"""JSON Schema -> GBNF (the subset llama-cpp-python's ``json_schema_to_gbnf`` is used for
with ``response_format={"type": "json_object", "schema": ...}`` / ``json_schema``).

Supported: ``type`` (object / array / string / number / integer / boolean / null, or a
list of them), ``properties`` + ``required`` (required properties first in declaration
order, then the optional ones, each optional one may be omitted), ``additionalProperties``
false/absent (no extra keys) , ``items``, ``minItems`` / ``maxItems``, ``enum``, ``const``,
``anyOf`` / ``oneOf``, ``$ref`` into ``#/definitions`` or ``#/$defs``, string
``minLength`` / ``maxLength``. Anything else falls back to a generic JSON value.
"""
from __future__ import annotations

import json
import re
from typing import Any, Dict

_PRIMS = r'''
value  ::= object | array | string | number | ("true" | "false" | "null") ws
object ::= "{" ws ( string ":" ws value ("," ws string ":" ws value)* )? "}" ws
array  ::= "[" ws ( value ("," ws value)* )? "]" ws
char   ::= [^"\\\x7F\x00-\x1F] | "\\" (["\\bfnrt] | "u" [0-9a-fA-F]{4})
string ::= "\"" char* "\"" ws
number ::= ("-"? ([0-9] | [1-9] [0-9]{0,15})) ("." [0-9]+)? ([eE] [-+]? [0-9] [1-9]{0,15})? ws
integer ::= ("-"? ([0-9] | [1-9] [0-9]{0,15})) ws
boolean ::= ("true" | "false") ws
null   ::= "null" ws
ws ::= | " " | "\n" [ \t]{0,20}
'''


def _lit(v: Any) -> str:
    """A GBNF literal matching the JSON encoding of v."""
    s = json.dumps(v)
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


class _Conv:
    def __init__(self, root: Dict[str, Any]):
        self.root = root
        self.rules: Dict[str, str] = {}
        self.refs: Dict[str, str] = {}

    def name(self, hint: str) -> str:
        base = re.sub(r"[^a-zA-Z0-9-]+", "-", hint).strip("-") or "r"
        n, k = base, 1
        while n in self.rules or n in ("value", "object", "array", "char", "string", "number", "integer",
                                       "boolean", "null", "ws", "root"):
            k += 1
            n = f"{base}{k}"
        self.rules[n] = ""
        return n

    def ref(self, path: str) -> str:
        if path in self.refs:
            return self.refs[path]
        if not (path.startswith("#/definitions/") or path.startswith("#/$defs/")):
            raise ValueError(f"unsupported $ref {path!r}")
        node = self.root
        for part in path[2:].split("/"):
            node = node[part]
        n = self.name(path.split("/")[-1])
        self.refs[path] = n
        self.rules[n] = self.visit(node, n)
        return n

    def visit(self, s: Dict[str, Any], hint: str) -> str:
        if not isinstance(s, dict) or not s:
            return "value"
        if "$ref" in s:
            return self.ref(s["$ref"])
        if "const" in s:
            return f"{_lit(s['const'])} ws"
        if "enum" in s:
            return "(" + " | ".join(_lit(v) for v in s["enum"]) + ") ws"
        for key in ("anyOf", "oneOf"):
            if key in s:
                return "(" + " | ".join(self.sub(x, f"{hint}-{i}") for i, x in enumerate(s[key])) + ")"
        t = s.get("type")
        if isinstance(t, list):
            return "(" + " | ".join(self.sub(dict(s, type=x), f"{hint}-{x}") for x in t) + ")"
        if t == "object" or (t is None and "properties" in s):
            props = s.get("properties", {})
            if not props:
                return "object"
            req = [k for k in props if k in set(s.get("required", []))]
            opt = [k for k in props if k not in set(s.get("required", []))]
            parts = []
            for k in req:
                parts.append(("req", f'{_lit(k)} ws ":" ws {self.sub(props[k], f"{hint}-{k}")}'))
            for k in opt:
                parts.append(("opt", f'{_lit(k)} ws ":" ws {self.sub(props[k], f"{hint}-{k}")}'))
            return '"{" ws ' + self._members(parts, hint) + ' "}" ws'
        if t == "array":
            item = self.sub(s.get("items", {}), f"{hint}-item")
            lo, hi = int(s.get("minItems", 0)), s.get("maxItems")
            if hi is not None and int(hi) == 0:
                return '"[" ws "]" ws'
            if lo == 0 and hi is None:
                return f'"[" ws ( {item} ( "," ws {item} )* )? "]" ws'
            first_lo = max(lo, 1)
            rest_lo = first_lo - 1
            rest = (f'( "," ws {item} ){{{rest_lo},}}' if hi is None
                    else f'( "," ws {item} ){{{rest_lo},{int(hi) - 1}}}')
            body = f"{item} {rest}"
            return f'"[" ws ( {body} ){"" if lo > 0 else "?"} "]" ws'
        if t == "string":
            lo, hi = s.get("minLength"), s.get("maxLength")
            if lo is None and hi is None:
                return "string"
            rep = f"{{{int(lo or 0)},{'' if hi is None else int(hi)}}}"
            return f'"\\"" char{rep} "\\"" ws'
        if t in ("number", "integer", "boolean", "null"):
            return t
        return "value"

    def sub(self, s: Dict[str, Any], hint: str) -> str:
        body = self.visit(s, hint)
        if re.fullmatch(r"[a-zA-Z0-9-]+", body):
            return body
        n = self.name(hint)
        self.rules[n] = body
        return n

    def _members(self, parts, hint: str) -> str:
        """Required members in declaration order; each optional member (in order) may be
        present or not. A comma precedes every member but the first one present."""
        req = [p for k, p in parts if k == "req"]
        opt = [p for k, p in parts if k == "opt"]
        if req:
            return ' "," ws '.join(req) + "".join(f' ( "," ws {p} )?' for p in opt)
        if not opt:
            return ""
        alts = [opt[i] + "".join(f' ( "," ws {p} )?' for p in opt[i + 1:]) for i in range(len(opt))]
        return "( " + " | ".join(alts) + " )?"


def json_schema_to_gbnf(schema: Any) -> str:
    if isinstance(schema, str):
        schema = json.loads(schema)
    c = _Conv(schema)
    root = c.visit(schema, "root")
    lines = [f"root ::= {root}"]
    lines += [f"{k} ::= {v}" for k, v in c.rules.items()]
    return "\n".join(lines) + "\n" + _PRIMS
