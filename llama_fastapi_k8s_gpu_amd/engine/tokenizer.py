"""Tokenizers built purely from GGUF metadata.

  * ``BPETokenizer``  - byte-level BPE (``tokenizer.ggml.model == "gpt2"``), the
    Llama-3 "llama-bpe" pre-tokenizer regex, merges ranked by
    ``tokenizer.ggml.merges`` order, special-token partitioning.
  * ``SPMTokenizer``  - SentencePiece-style BPE (``tokenizer.ggml.model ==
    "llama"``, TinyLlama/Mixtral): space -> U+2581, leading space prefix, greedy
    highest-score bigram merging, ``<0xXX>`` byte fallback.

Both expose ``encode(text, add_bos, special)``, ``decode(ids)`` and
``token_to_piece(id)`` - the subset of the llama.cpp vocab API that the
``Llama`` facade needs (reference reaches these through api.py:55-63).
"""
from __future__ import annotations

import heapq
from functools import lru_cache
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import regex

from ..gguf.constants import (TOKEN_TYPE_BYTE, TOKEN_TYPE_CONTROL, TOKEN_TYPE_NORMAL,
                              TOKEN_TYPE_UNUSED, TOKEN_TYPE_USER_DEFINED)

LLAMA3_PRETOKENIZE = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
                      r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2_PRETOKENIZE = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


@lru_cache(maxsize=1)
def bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


class _Base:
    tokens: List[str]
    types: List[int]
    bos_id: int
    eos_id: int

    def _init_specials(self):
        self.token_to_id: Dict[str, int] = {t: i for i, t in enumerate(self.tokens)}
        specials = [(t, i) for i, t in enumerate(self.tokens)
                    if self.types[i] in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED) and t]
        specials.sort(key=lambda x: -len(x[0]))
        self._special_ids = {i for _, i in specials}
        self._special_map = dict(specials)
        self._special_re = (regex.compile("|".join(regex.escape(t) for t, _ in specials))
                            if specials else None)

    @property
    def n_vocab(self) -> int:
        return len(self.tokens)

    def is_eog(self, tok: int) -> bool:
        return tok in self.eog_ids

    def _split_special(self, text: str, special: bool) -> Iterable[Tuple[bool, str]]:
        if not special or self._special_re is None:
            yield False, text
            return
        pos = 0
        for m in self._special_re.finditer(text):
            if m.start() > pos:
                yield False, text[pos:m.start()]
            yield True, m.group(0)
            pos = m.end()
        if pos < len(text):
            yield False, text[pos:]

    def encode(self, text: str, add_bos: bool = True, special: bool = True) -> List[int]:
        out: List[int] = [self.bos_id] if (add_bos and self.bos_id >= 0) else []
        first = True
        for is_special, seg in self._split_special(text, special):
            if is_special:
                out.append(self._special_map[seg])
            else:
                out.extend(self._encode_plain(seg, first))
            first = False
        return out

    def decode(self, ids: Sequence[int], special: bool = False) -> str:
        return self.detokenize_bytes(ids, special).decode("utf-8", errors="replace")


class BPETokenizer(_Base):
    def __init__(self, tokens: List[str], merges: List[str], types: Optional[List[int]] = None,
                 bos_id: int = -1, eos_id: int = -1, eot_id: int = -1, pre: str = "llama-bpe"):
        self.tokens = tokens
        self.types = list(types) if types is not None else [TOKEN_TYPE_NORMAL] * len(tokens)
        self.bos_id, self.eos_id = bos_id, eos_id
        self.eog_ids = {t for t in (eos_id, eot_id) if t >= 0}
        self.ranks: Dict[Tuple[str, str], int] = {}
        for r, m in enumerate(merges):
            a, b = m.split(" ", 1)
            self.ranks[(a, b)] = r
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        self.pre_re = regex.compile(LLAMA3_PRETOKENIZE if pre in ("llama-bpe", "llama3", "default")
                                    else GPT2_PRETOKENIZE)
        self._cache: Dict[str, List[int]] = {}
        self._init_specials()

    def _bpe(self, word: str) -> List[int]:
        cached = self._cache.get(word)
        if cached is not None:
            return cached
        parts = list(word)
        ranks = self.ranks
        while len(parts) > 1:
            best, best_i = None, -1
            for i in range(len(parts) - 1):
                r = ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best is None or r < best):
                    best, best_i = r, i
            if best is None:
                break
            parts[best_i:best_i + 2] = [parts[best_i] + parts[best_i + 1]]
        ids = []
        for p in parts:
            tid = self.token_to_id.get(p)
            if tid is None:  # unknown merge result: fall back to single byte tokens
                ids.extend(self.token_to_id[c] for c in p)
            else:
                ids.append(tid)
        if len(self._cache) < 100_000:
            self._cache[word] = ids
        return ids

    def _encode_plain(self, text: str, first: bool) -> List[int]:
        out: List[int] = []
        for piece in self.pre_re.findall(text):
            word = "".join(self.byte_encoder[b] for b in piece.encode("utf-8"))
            out.extend(self._bpe(word))
        return out

    def token_to_piece_bytes(self, tid: int, special: bool = False) -> bytes:
        if tid in self._special_ids or self.types[tid] in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_UNUSED):
            return self.tokens[tid].encode("utf-8") if special else b""
        tok = self.tokens[tid]
        try:
            return bytes(self.byte_decoder[c] for c in tok)
        except KeyError:
            return tok.encode("utf-8")

    def detokenize_bytes(self, ids: Sequence[int], special: bool = False) -> bytes:
        return b"".join(self.token_to_piece_bytes(int(i), special) for i in ids)


class SPMTokenizer(_Base):
    SPACE = "▁"

    def __init__(self, pieces: List[str], scores: List[float], types: List[int],
                 bos_id: int = 1, eos_id: int = 2, unk_id: int = 0, add_space_prefix: bool = True):
        self.tokens = pieces
        self.scores = scores
        self.types = list(types)
        self.bos_id, self.eos_id, self.unk_id = bos_id, eos_id, unk_id
        self.eog_ids = {eos_id} if eos_id >= 0 else set()
        self.add_space_prefix = add_space_prefix
        self._init_specials()
        self._byte_ids: Dict[int, int] = {}
        for i, t in enumerate(pieces):
            if self.types[i] == TOKEN_TYPE_BYTE and len(t) == 6 and t.startswith("<0x"):
                self._byte_ids[int(t[3:5], 16)] = i
        self._normal = {t: i for i, t in enumerate(pieces)
                        if self.types[i] in (TOKEN_TYPE_NORMAL, TOKEN_TYPE_USER_DEFINED)}

    def _encode_plain(self, text: str, first: bool) -> List[int]:
        if not text:
            return []
        if self.add_space_prefix and first:
            text = " " + text
        text = text.replace(" ", self.SPACE)
        syms = list(text)
        # doubly linked list of symbols + max-heap of candidate bigrams
        prev = list(range(-1, len(syms) - 1))
        nxt = list(range(1, len(syms) + 1))
        nxt[-1] = -1
        alive = [True] * len(syms)
        heap: List[Tuple[float, int, int, str]] = []

        def push(i: int):
            j = nxt[i]
            if j < 0:
                return
            merged = syms[i] + syms[j]
            tid = self._normal.get(merged)
            if tid is not None:
                heapq.heappush(heap, (-self.scores[tid], i, j, merged))

        for i in range(len(syms) - 1):
            push(i)
        while heap:
            _, i, j, merged = heapq.heappop(heap)
            if not alive[i] or not alive[j] or nxt[i] != j or syms[i] + syms[j] != merged:
                continue
            syms[i] = merged
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] >= 0:
                prev[nxt[j]] = i
            if prev[i] >= 0:
                push(prev[i])
            push(i)
        out: List[int] = []
        i = 0
        while i >= 0 and i < len(syms):
            if alive[i]:
                tid = self._normal.get(syms[i])
                if tid is not None:
                    out.append(tid)
                else:
                    for b in syms[i].encode("utf-8"):
                        out.append(self._byte_ids.get(b, self.unk_id))
            i = nxt[i]
        return out

    def token_to_piece_bytes(self, tid: int, special: bool = False) -> bytes:
        t = self.types[tid]
        piece = self.tokens[tid]
        if t == TOKEN_TYPE_BYTE:
            return bytes([int(piece[3:5], 16)])
        if t in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_UNUSED):
            return piece.encode("utf-8") if special else b""
        return piece.replace(self.SPACE, " ").encode("utf-8")

    def detokenize_bytes(self, ids: Sequence[int], special: bool = False) -> bytes:
        out = b"".join(self.token_to_piece_bytes(int(i), special) for i in ids)
        return out


def tokenizer_from_metadata(md: dict):
    model = md.get("tokenizer.ggml.model", "gpt2")
    tokens = md["tokenizer.ggml.tokens"]
    types = md.get("tokenizer.ggml.token_type") or [TOKEN_TYPE_NORMAL] * len(tokens)
    bos = int(md.get("tokenizer.ggml.bos_token_id", -1))
    eos = int(md.get("tokenizer.ggml.eos_token_id", -1))
    if model == "gpt2":
        eot = -1
        for name in ("<|eot_id|>", "<|im_end|>", "<|end|>"):
            if name in tokens:
                eot = tokens.index(name)
                break
        return BPETokenizer(tokens, md.get("tokenizer.ggml.merges", []), types, bos, eos, eot,
                            md.get("tokenizer.ggml.pre", "llama-bpe"))
    if model == "llama":
        return SPMTokenizer(tokens, md.get("tokenizer.ggml.scores", [0.0] * len(tokens)), types, bos, eos,
                            int(md.get("tokenizer.ggml.unknown_token_id", 0)),
                            bool(md.get("tokenizer.ggml.add_space_prefix", True)))
    raise NotImplementedError(f"tokenizer model {model!r}")
