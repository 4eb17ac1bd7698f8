"""Grammar-constrained sampling: GBNF grammars (llama.cpp ``grammar-parser.cpp`` syntax,
``llama_cpp.LlamaGrammar`` API) and the token filter the host sampler applies.

Semantics follow upstream ``llama_sample_grammar`` + ``llama_grammar_accept_token``:
a token is allowed iff the grammar can consume its text from the current state; an
end-of-generation token is allowed iff the grammar can be complete; tokens without
text (other specials) are never allowed. Upstream masks the whole vocabulary before
the sampler chain; here the chain's result is computed exactly without masking every
token: with ``top_k > 0`` the k best allowed tokens are found by checking candidates in
descending-logit order (the chain only ever sees those k), otherwise (or when the
first candidates are mostly rejected) the allowed set is enumerated by walking a
code-point trie of the vocabulary under the grammar, pruning dead prefixes.

Grammar syntax: ``name ::= alternatives``; literals ``"..."`` (escapes ``\\n \\r \\t
\\\\ \\" \\xHH \\uHHHH \\UHHHHHHHH``); classes ``[a-z]``/``[^...]``; ``.`` any char; rule
references; ``( ... )`` groups; postfix ``* + ?`` and ``{m}``, ``{m,}``, ``{m,n}``;
``#`` comments. A rule body runs until the next ``name ::=`` (so alternatives may
continue on following lines).
"""
from __future__ import annotations

import re
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

Elem = Tuple  # ("c", ((lo, hi), ...), negated) | ("r", rule_id)
Pos = Tuple[int, int, int]  # (rule, alternative, element index)
Stack = Tuple[Pos, ...]
State = FrozenSet[Stack]

_NAME = re.compile(r"[a-zA-Z0-9_-]+")
_RULE_START = re.compile(r"(?m)^[ \t]*([a-zA-Z0-9_-]+)[ \t]*::=")


class GrammarError(ValueError):
    pass


def _strip_comments(text: str) -> str:
    out = []
    for line in text.splitlines():
        buf, in_str, in_cls, i = [], False, False, 0
        while i < len(line):
            ch = line[i]
            if ch == "\\" and (in_str or in_cls) and i + 1 < len(line):
                buf.append(line[i:i + 2])
                i += 2
                continue
            if ch == '"' and not in_cls:
                in_str = not in_str
            elif ch == "[" and not in_str:
                in_cls = True
            elif ch == "]" and in_cls:
                in_cls = False
            elif ch == "#" and not in_str and not in_cls:
                break
            buf.append(ch)
            i += 1
        out.append("".join(buf))
    return "\n".join(out)


class _Parser:
    def __init__(self):
        self.rules: List[List[List[Elem]]] = []
        self.names: Dict[str, int] = {}
        self.defined: set = set()

    def rule_id(self, name: str) -> int:
        if name not in self.names:
            self.names[name] = len(self.rules)
            self.rules.append([])
        return self.names[name]

    def new_rule(self, base: str, alts: List[List[Elem]]) -> int:
        k = 1
        while f"{base}_{k}" in self.names:
            k += 1
        rid = self.rule_id(f"{base}_{k}")
        self.rules[rid] = alts
        self.defined.add(f"{base}_{k}")
        return rid

    # --- lexical helpers
    @staticmethod
    def _esc(s: str, i: int) -> Tuple[int, int]:
        """Escape at s[i] == '\\' -> (code point, next index)."""
        c = s[i + 1]
        simple = {"n": 10, "r": 13, "t": 9, "\\": 92, '"': 34, "[": 91, "]": 93, "-": 45, "^": 94, "/": 47}
        if c in simple:
            return simple[c], i + 2
        n = {"x": 2, "u": 4, "U": 8}.get(c)
        if n:
            h = s[i + 2:i + 2 + n]
            if len(h) != n or not all(ch in "0123456789abcdefABCDEF" for ch in h):
                raise GrammarError(f"bad escape at {s[i:i + 2 + n]!r}")
            return int(h, 16), i + 2 + n
        raise GrammarError(f"unknown escape \\{c}")

    def _char(self, s: str, i: int) -> Tuple[int, int]:
        if s[i] == "\\":
            return self._esc(s, i)
        return ord(s[i]), i + 1

    @staticmethod
    def _ws(s: str, i: int) -> int:
        while i < len(s) and s[i] in " \t\r\n":
            i += 1
        return i

    # --- grammar
    def parse_alternates(self, s: str, i: int, name: str, close: Optional[str]) -> Tuple[List[List[Elem]], int]:
        alts = []
        while True:
            seq, i = self.parse_sequence(s, i, name)
            alts.append(seq)
            i = self._ws(s, i)
            if i < len(s) and s[i] == "|":
                i += 1
                continue
            break
        if close is not None:
            if i >= len(s) or s[i] != close:
                raise GrammarError(f"expected {close!r} in rule {name}")
            i += 1
        return alts, i

    def parse_sequence(self, s: str, i: int, name: str) -> Tuple[List[Elem], int]:
        seq: List[Elem] = []
        last_start = None   # index in seq where the last atom starts (for postfix operators)
        while True:
            i = self._ws(s, i)
            if i >= len(s) or s[i] in "|)":
                return seq, i
            c = s[i]
            if c == '"':
                i += 1
                last_start = len(seq)
                while True:
                    if i >= len(s):
                        raise GrammarError(f"unterminated literal in rule {name}")
                    if s[i] == '"':
                        i += 1
                        break
                    cp, i = self._char(s, i)
                    seq.append(("c", ((cp, cp),), False))
                if len(seq) == last_start:        # empty literal ""
                    last_start = None
            elif c == "[":
                i += 1
                neg = i < len(s) and s[i] == "^"
                if neg:
                    i += 1
                ranges = []
                while True:
                    if i >= len(s):
                        raise GrammarError(f"unterminated class in rule {name}")
                    if s[i] == "]":
                        i += 1
                        break
                    lo, i = self._char(s, i)
                    hi = lo
                    if i + 1 < len(s) and s[i] == "-" and s[i + 1] != "]":
                        hi, i = self._char(s, i + 1)
                    ranges.append((lo, hi))
                last_start = len(seq)
                seq.append(("c", tuple(ranges), neg))
            elif c == ".":
                i += 1
                last_start = len(seq)
                seq.append(("c", ((0, 0x10FFFF),), False))
            elif c == "(":
                alts, i = self.parse_alternates(s, i + 1, name, ")")
                last_start = len(seq)
                seq.append(("r", self.new_rule(name, alts)))
            elif c in "*+?{":
                if last_start is None:
                    raise GrammarError(f"repetition without an operand in rule {name}")
                atom = seq[last_start:]
                del seq[last_start:]
                if c == "{":
                    m = re.match(r"\{\s*(\d+)\s*(,\s*(\d*)\s*)?\}", s[i:])
                    if not m:
                        raise GrammarError(f"bad repetition in rule {name}")
                    lo = int(m.group(1))
                    hi = lo if m.group(2) is None else (int(m.group(3)) if m.group(3) else None)
                    i += m.end()
                else:
                    lo, hi = {"*": (0, None), "+": (1, None), "?": (0, 1)}[c]
                    i += 1
                seq.append(("r", self._repeat(name, atom, lo, hi)))
                last_start = len(seq) - 1
            else:
                m = _NAME.match(s, i)
                if not m:
                    raise GrammarError(f"unexpected {s[i]!r} in rule {name}")
                last_start = len(seq)
                seq.append(("r", self.rule_id(m.group(0))))
                i = m.end()

    def _repeat(self, name: str, atom: List[Elem], lo: int, hi: Optional[int]) -> int:
        """atom{lo,hi} as rules: lo copies, then (hi - lo) optional ones, or a star tail."""
        if hi is not None and hi < lo:
            raise GrammarError(f"bad repetition bounds in rule {name}")
        seq = list(atom) * lo
        if hi is None:
            star = self.new_rule(name, [])
            self.rules[star] = [list(atom) + [("r", star)], []]
            seq.append(("r", star))
        else:
            tail: Optional[int] = None
            for _ in range(hi - lo):       # nested optionals: (atom (atom (...)?)?)?
                body = list(atom) + ([("r", tail)] if tail is not None else [])
                tail = self.new_rule(name, [body, []])
            if tail is not None:
                seq.append(("r", tail))
        return self.new_rule(name, [seq])

    def parse(self, text: str) -> Tuple[List[List[List[Elem]]], Dict[str, int]]:
        text = _strip_comments(text)
        starts = list(_RULE_START.finditer(text))
        if not starts:
            raise GrammarError("no rules")
        if text[:starts[0].start()].strip():
            raise GrammarError("text before the first rule")
        for j, m in enumerate(starts):
            name = m.group(1)
            body = text[m.end(): starts[j + 1].start() if j + 1 < len(starts) else len(text)]
            alts, k = self.parse_alternates(body, 0, name, None)
            if body[k:].strip():
                raise GrammarError(f"unexpected {body[k:].strip()[:20]!r} in rule {name}")
            rid = self.rule_id(name)
            self.rules[rid] = alts
            self.defined.add(name)
        for n in self.names:
            if n not in self.defined:
                raise GrammarError(f"undefined rule {n!r}")
        if "root" not in self.names:
            raise GrammarError("grammar has no 'root' rule")
        return self.rules, self.names


class LlamaGrammar:
    """A compiled grammar (``llama_cpp.LlamaGrammar.from_string`` / ``from_file``)."""

    def __init__(self, rules, names, text: str = ""):
        self.rules = rules
        self.names = names
        self.text = text
        self.root = names["root"]
        self._accept_cache: Dict[Tuple[State, int], State] = {}
        self._check_left_recursion()
        self.initial: State = self._expand_all([((self.root, a, 0),) for a in range(len(rules[self.root]))])

    @classmethod
    def from_string(cls, grammar: str, verbose: bool = True) -> "LlamaGrammar":
        rules, names = _Parser().parse(grammar)
        return cls(rules, names, grammar)

    @classmethod
    def from_file(cls, file: str, verbose: bool = True) -> "LlamaGrammar":
        with open(file, encoding="utf-8") as f:
            return cls.from_string(f.read(), verbose)

    @classmethod
    def from_json_schema(cls, json_schema: str, verbose: bool = True) -> "LlamaGrammar":
        from .json_schema import json_schema_to_gbnf
        return cls.from_string(json_schema_to_gbnf(json_schema), verbose)

    # --- structure checks
    def _nullable(self) -> List[bool]:
        null = [False] * len(self.rules)
        changed = True
        while changed:
            changed = False
            for r, alts in enumerate(self.rules):
                if null[r]:
                    continue
                if any(all(e[0] == "r" and null[e[1]] for e in alt) for alt in alts):
                    null[r] = changed = True
        return null

    def _check_left_recursion(self):
        null = self._nullable()
        first: List[set] = [set() for _ in self.rules]   # rules reachable at position 0
        for r, alts in enumerate(self.rules):
            for alt in alts:
                for e in alt:
                    if e[0] != "r":
                        break
                    first[r].add(e[1])
                    if not null[e[1]]:
                        break
        for r in range(len(self.rules)):
            seen, todo = set(), list(first[r])
            while todo:
                x = todo.pop()
                if x == r:
                    name = next(n for n, i in self.names.items() if i == r)
                    raise GrammarError(f"left recursion in rule {name!r}")
                if x not in seen:
                    seen.add(x)
                    todo.extend(first[x])

    # --- pushdown matching
    def _expand(self, stack: Stack, out: set):
        if not stack:
            out.add(stack)
            return
        r, a, i = stack[-1]
        alt = self.rules[r][a]
        if i == len(alt):
            self._expand(stack[:-1], out)
            return
        el = alt[i]
        if el[0] == "c":
            out.add(stack)
            return
        base = stack[:-1] + (((r, a, i + 1),) if i + 1 < len(alt) else ())
        for ai in range(len(self.rules[el[1]])):
            self._expand(base + ((el[1], ai, 0),), out)

    def _expand_all(self, stacks) -> State:
        out: set = set()
        for st in stacks:
            self._expand(st, out)
        return frozenset(out)

    @staticmethod
    def _match(el: Elem, cp: int) -> bool:
        hit = any(lo <= cp <= hi for lo, hi in el[1])
        return hit != el[2]

    def accept(self, state: State, cp: int) -> State:
        key = (state, cp)
        got = self._accept_cache.get(key)
        if got is not None:
            return got
        nxt = []
        for st in state:
            if not st:
                continue
            r, a, i = st[-1]
            if self._match(self.rules[r][a][i], cp):
                alt = self.rules[r][a]
                nxt.append(st[:-1] + (((r, a, i + 1),) if i + 1 < len(alt) else ()))
        res = self._expand_all(nxt)
        if len(self._accept_cache) > 200000:
            self._accept_cache.clear()
        self._accept_cache[key] = res
        return res

    def accept_cps(self, state: State, cps: Sequence[int]) -> State:
        for cp in cps:
            state = self.accept(state, cp)
            if not state:
                break
        return state

    @staticmethod
    def can_end(state: State) -> bool:
        return () in state

    def partial_ok(self, state: State, pending: bytes) -> bool:
        """Whether an incomplete UTF-8 sequence can still become a code point that some
        stack accepts next (upstream ``match_partial_char``)."""
        if not pending:
            return True
        b0 = pending[0]
        total = 2 if 0xC0 <= b0 <= 0xDF else 3 if 0xE0 <= b0 <= 0xEF else 4 if 0xF0 <= b0 <= 0xF7 else 0
        if not total or len(pending) >= total or any(not 0x80 <= b <= 0xBF for b in pending[1:]):
            return False
        v = b0 & (0x7F >> total)
        for b in pending[1:]:
            v = (v << 6) | (b & 0x3F)
        miss = total - len(pending)
        lo, hi = v << (6 * miss), (v << (6 * miss)) | ((1 << (6 * miss)) - 1)
        lo = max(lo, (0, 0, 0x80, 0x800, 0x10000)[total])   # no overlong encodings
        if lo > hi:
            return False
        for st in state:
            if not st:
                continue
            r, a, i = st[-1]
            el = self.rules[r][a][i]
            if not el[2]:
                if any(x <= hi and lo <= y for x, y in el[1]):
                    return True
            elif not any(x <= lo and hi <= y for x, y in el[1]):
                return True
        return False


def _utf8_split(b: bytes) -> Tuple[List[int], bytes]:
    """Complete code points of ``b`` and the trailing incomplete UTF-8 bytes (if any)."""
    for cut in range(len(b), max(-1, len(b) - 4), -1):
        try:
            return [ord(c) for c in b[:cut].decode("utf-8")], b[cut:]
        except UnicodeDecodeError:
            continue
    return [ord(c) for c in b.decode("utf-8", errors="replace")], b""


class _Trie:
    __slots__ = ("children", "tokens")

    def __init__(self):
        self.children: Dict[int, "_Trie"] = {}
        self.tokens: List[int] = []


class GrammarVocab:
    """Token texts of a vocabulary, prepared once per model for grammar matching."""

    def __init__(self, token_bytes: Sequence[bytes], eog_ids: Sequence[int]):
        self.eog = set(int(t) for t in eog_ids)
        self.bytes = list(token_bytes)
        self.cps: List[Optional[List[int]]] = []
        self.tail: List[bytes] = []
        self._trie: Optional[_Trie] = None
        for b in self.bytes:
            cps, tail = _utf8_split(b) if b else ([], b"")
            self.cps.append(cps)
            self.tail.append(tail)

    def trie(self) -> _Trie:
        if self._trie is None:
            root = _Trie()
            for t, (cps, tail, b) in enumerate(zip(self.cps, self.tail, self.bytes)):
                if not b or tail or t in self.eog:
                    continue
                node = root
                for cp in cps:
                    node = node.children.setdefault(cp, _Trie())
                node.tokens.append(t)
            self._trie = root
        return self._trie


class GrammarState:
    """Per-request matcher: the current set of pushdown stacks plus any pending bytes of
    a code point split across tokens (byte-level BPE)."""

    def __init__(self, grammar: LlamaGrammar, vocab: GrammarVocab):
        self.g = grammar
        self.v = vocab
        self.state: State = grammar.initial
        self.pending = b""

    def _advance(self, tok: int) -> Tuple[State, bytes]:
        b = self.v.bytes[tok]
        if self.pending:
            cps, tail = _utf8_split(self.pending + b)
        else:
            cps, tail = self.v.cps[tok], self.v.tail[tok]
        return self.g.accept_cps(self.state, cps), tail

    def allows(self, tok: int) -> bool:
        if tok in self.v.eog:
            return LlamaGrammar.can_end(self.state) and not self.pending
        if not self.v.bytes[tok]:
            return False
        st, tail = self._advance(tok)
        return bool(st) and (not tail or self.g.partial_ok(st, tail))

    def accept_token(self, tok: int):
        if tok in self.v.eog:
            return
        self.state, self.pending = self._advance(tok)
        if not self.state:
            raise GrammarError("token not accepted by the grammar")

    def allowed_tokens(self) -> List[int]:
        """Every allowed token (trie walk; pending-byte and partial-UTF-8 tokens checked one by one)."""
        out = [t for t in self.v.eog if LlamaGrammar.can_end(self.state) and not self.pending]
        if self.pending:
            return out + [t for t in range(len(self.v.bytes)) if t not in self.v.eog and self.allows(t)]
        g = self.g
        todo = [(self.v.trie(), self.state)]
        while todo:
            node, st = todo.pop()
            out.extend(node.tokens)
            for cp, child in node.children.items():
                nst = g.accept(st, cp)
                if nst:
                    todo.append((child, nst))
        out.extend(t for t, (b, tail) in enumerate(zip(self.v.bytes, self.v.tail))
                   if b and tail and t not in self.v.eog and self.allows(t))
        return out


JSON_GBNF = r'''
root   ::= object
value  ::= object | array | string | number | ("true" | "false" | "null") ws

object ::=
  "{" ws (
            string ":" ws value
    ("," ws string ":" ws value)*
  )? "}" ws

array  ::=
  "[" ws (
            value
    ("," ws value)*
  )? "]" ws

string ::=
  "\"" (
    [^"\\\x7F\x00-\x1F] |
    "\\" (["\\bfnrt] | "u" [0-9a-fA-F]{4}) # escapes
  )* "\"" ws

number ::= ("-"? ([0-9] | [1-9] [0-9]{0,15})) ("." [0-9]+)? ([eE] [-+]? [0-9] [1-9]{0,15})? ws

# Optional space: by convention, applied in this grammar after literal chars when allowed
ws ::= | " " | "\n" [ \t]{0,20}
'''
