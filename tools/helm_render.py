"""Minimal renderer for the Go-template subset used by ``helm/`` (no helm binary
in the build image). Supports ``{{ }}`` with ``-`` trimming,
``.Values/.Release/.Chart`` lookups, pipelines, parenthesised sub-expressions,
``if / else if / else / end``, ``define`` + ``include`` and the functions
``quote default printf eq ne gt lt int not toString``.

    python tools/helm_render.py helm [--set gpu.perPod=8 ...]   # prints the manifests
"""
from __future__ import annotations

import os
import re
import shlex
import sys
from typing import Any, Dict, List, Tuple

import yaml

_ACTION = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


def _tokens(src: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip(" \t\n")
        if out and out[-1][0] == "trim_next":
            out.pop()
            text = text.lstrip(" \t\n")
        out.append(("text", text))
        out.append(("act", m.group(2)))
        if m.group(3):
            out.append(("trim_next", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "trim_next":
        out.pop()
        text = text.lstrip(" \t\n")
    out.append(("text", text))
    return out


def _parse(tokens, i=0, stop=("end",)):
    """-> (nodes, index, terminator)"""
    nodes = []
    while i < len(tokens):
        kind, val = tokens[i]
        if kind == "text":
            nodes.append(("text", val))
            i += 1
            continue
        word = val.split(None, 1)[0] if val else ""
        if val.startswith("/*"):
            i += 1
            continue
        if word in ("end", "else"):
            return nodes, i, val
        if word == "if":
            branches = []
            cond = val[2:].strip()
            i += 1
            while True:
                body, i, term = _parse(tokens, i)
                branches.append((cond, body))
                i += 1
                if term == "end":
                    break
                rest = term[4:].strip()           # "else" or "else if <cond>"
                cond = rest[2:].strip() if rest.startswith("if") else None
            nodes.append(("if", branches))
            continue
        if word == "define":
            name = shlex.split(val[6:].strip())[0]
            body, i, _ = _parse(tokens, i + 1)
            nodes.append(("define", name, body))
            i += 1
            continue
        nodes.append(("expr", val))
        i += 1
    return nodes, i, None


def _split_args(expr: str) -> List[str]:
    out, depth, cur, q = [], 0, "", False
    for ch in expr:
        if ch == '"' and depth == 0:
            q = not q
        if not q and ch == "(":
            depth += 1
        if not q and ch == ")":
            depth -= 1
        if ch.isspace() and depth == 0 and not q:
            if cur:
                out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        out.append(cur)
    return out


def _split_pipe(expr: str) -> List[str]:
    out, depth, cur, q = [], 0, "", False
    for ch in expr:
        if ch == '"':
            q = not q
        if not q and ch == "(":
            depth += 1
        if not q and ch == ")":
            depth -= 1
        if ch == "|" and depth == 0 and not q:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    out.append(cur.strip())
    return out


class Renderer:
    def __init__(self, values: Dict[str, Any], chart: Dict[str, Any], release: str = "chat"):
        self.ctx = {"Values": values, "Chart": {k[0].upper() + k[1:]: v for k, v in chart.items()},
                    "Release": {"Name": release, "Namespace": values.get("namespace", "default")}}
        self.defines: Dict[str, list] = {}

    def _fmt(self, v) -> str:
        if v is None:
            return ""
        if isinstance(v, bool):
            return "true" if v else "false"
        return str(v)

    def _value(self, a: str, dot):
        if a.startswith("("):
            return self._pipeline(a[1:-1], dot)
        if a.startswith('"'):
            return a[1:-1]
        if a == ".":
            return dot
        if a.startswith("."):
            cur = dot
            for part in a[1:].split("."):
                cur = cur.get(part) if isinstance(cur, dict) else None
            return cur
        if a in ("true", "false"):
            return a == "true"
        if re.fullmatch(r"-?\d+", a):
            return int(a)
        if re.fullmatch(r"-?\d+\.\d*", a):
            return float(a)
        return self._call(a, [], dot)

    def _call(self, fn: str, args: list, dot):
        if fn == "quote":
            return '"' + self._fmt(args[0]).replace('"', '\\"') + '"'
        if fn == "default":
            return args[1] if args[1] not in (None, "", 0, False) else args[0]
        if fn == "printf":
            return args[0].replace("%s", "{}").format(*[self._fmt(a) for a in args[1:]])
        if fn == "eq":
            return args[0] == args[1]
        if fn == "ne":
            return args[0] != args[1]
        if fn == "gt":
            return args[0] > args[1]
        if fn == "lt":
            return args[0] < args[1]
        if fn == "int":
            return int(args[0] or 0)
        if fn == "not":
            return not args[0]
        if fn == "toString":
            return self._fmt(args[0])
        if fn == "include":
            return self._render(self.defines[args[0]], args[1])
        raise ValueError(f"unsupported template function {fn!r}")

    def _command(self, cmd: str, dot, piped=None, has_pipe=False):
        parts = _split_args(cmd)
        head = parts[0]
        if len(parts) == 1 and not has_pipe and (head.startswith((".", '"', "(")) or head[0].isdigit()):
            return self._value(head, dot)
        if head.startswith((".", '"', "(")):
            return self._value(head, dot)
        args = [self._value(a, dot) for a in parts[1:]]
        if has_pipe:
            args.append(piped)
        return self._call(head, args, dot)

    def _pipeline(self, expr: str, dot):
        cmds = _split_pipe(expr)
        v = self._command(cmds[0], dot)
        for c in cmds[1:]:
            v = self._command(c, dot, v, True)
        return v

    def _render(self, nodes, dot) -> str:
        out = []
        for n in nodes:
            if n[0] == "text":
                out.append(n[1])
            elif n[0] == "expr":
                out.append(self._fmt(self._pipeline(n[1], dot)))
            elif n[0] == "define":
                self.defines[n[1]] = n[2]
            elif n[0] == "if":
                for cond, body in n[1]:
                    if cond is None or self._pipeline(cond, dot):
                        out.append(self._render(body, dot))
                        break
        return "".join(out)

    def render(self, src: str) -> str:
        nodes, _, _ = _parse(_tokens(src))
        return self._render(nodes, self.ctx)


def _set(values: Dict[str, Any], assignment: str):
    key, raw = assignment.split("=", 1)
    cur = values
    parts = key.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = yaml.safe_load(raw)


def render_chart(chart_dir: str, overrides: List[str] = (), release: str = "chat") -> Dict[str, str]:
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        values = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    for o in overrides:
        _set(values, o)
    r = Renderer(values, chart, release)
    tdir = os.path.join(chart_dir, "templates")
    names = sorted(os.listdir(tdir))
    for n in names:                           # helpers first: defines are global
        if n.endswith(".tpl"):
            with open(os.path.join(tdir, n)) as f:
                r.render(f.read())
    out = {}
    for n in names:
        if n.endswith((".yaml", ".yml")):
            with open(os.path.join(tdir, n)) as f:
                out[n] = r.render(f.read())
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    chart = args[0] if args else "helm"
    sets = [args[i + 1] for i, a in enumerate(args) if a == "--set"]
    for name, text in render_chart(chart, sets).items():
        if text.strip():
            print(f"---\n# Source: {name}\n{text.strip()}")
