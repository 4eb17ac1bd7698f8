"""T2 - tokenizers built from GGUF metadata vs HF `tokenizers` / `sentencepiece`
on the same synthetic vocabularies; chat template exactness."""
import json
import os

import pytest

from llama_fastapi_k8s_gpu_amd.engine.chat_format import format_llama3, get_formatter
from llama_fastapi_k8s_gpu_amd.engine.tokenizer import (LLAMA3_PRETOKENIZE, BPETokenizer,
                                                        tokenizer_from_metadata)
from llama_fastapi_k8s_gpu_amd.gguf.synthetic import ASSETS, SPECS, build_vocab

TEXTS = [
    "Hello world! How are you doing today?",
    "  leading spaces and\ttabs\nnew lines\n\n\nand 12345 numbers 3.14159",
    "Unicode: naïve café, 你好世界, emoji 🙂 and ÄÖÜ.",
    "def foo(x):\n    return x ** 2  # comment\n",
    "I'm sure they'll've DONE it; isn't it?",
    "",
    "a" * 300,
]


@pytest.fixture(scope="module")
def bpe_md():
    md, n = build_vocab(SPECS["tiny-llama3-q4_k_m"])
    return md


@pytest.fixture(scope="module")
def hf_tok(bpe_md):
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers
    tokens = bpe_md["tokenizer.ggml.tokens"]
    vocab = {t: i for i, t in enumerate(tokens)}
    merges = [tuple(m.split(" ", 1)) for m in bpe_md["tokenizer.ggml.merges"]]
    tok = Tokenizer(models.BPE(vocab=vocab, merges=merges, ignore_merges=False))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_PRETOKENIZE), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    return tok


@pytest.mark.parametrize("text", TEXTS)
def test_bpe_matches_hf_tokenizers(bpe_md, hf_tok, text):
    ours = tokenizer_from_metadata(bpe_md)
    ids = ours.encode(text, add_bos=False, special=False)
    assert ids == hf_tok.encode(text).ids
    assert ours.decode(ids) == text


def test_bpe_special_tokens(bpe_md):
    tok = tokenizer_from_metadata(bpe_md)
    s = "<|start_header_id|>user<|end_header_id|>\n\nhi<|eot_id|>"
    ids = tok.encode(s, add_bos=True, special=True)
    toks = bpe_md["tokenizer.ggml.tokens"]
    assert ids[0] == tok.bos_id and toks[ids[1]] == "<|start_header_id|>"
    assert toks[ids[-1]] == "<|eot_id|>" and tok.is_eog(ids[-1])
    assert tok.decode(ids) == "user\n\nhi"        # control tokens render empty
    assert tok.decode(ids, special=True).endswith("<|eot_id|>")
    # special=False: special strings are plain text
    assert toks[tok.encode(s, add_bos=False, special=False)[0]] != "<|start_header_id|>"


@pytest.mark.parametrize("text", [t for t in TEXTS if "  " not in t and "\t" not in t and "\n" not in t])
def test_spm_matches_sentencepiece(text):
    import sentencepiece as spm
    sp = spm.SentencePieceProcessor(model_file=os.path.join(ASSETS, "spm_model.bin"))
    md, n = build_vocab(SPECS["tiny-tinyllama-q8_0"])
    ours = tokenizer_from_metadata(md)
    ref = sp.encode(text)
    got = ours.encode(text, add_bos=False, special=False)
    assert got == ref
    assert ours.decode(got).lstrip(" ") == text


def test_llama3_prompt_exact():
    msgs = [{"role": "user", "content": "hi"}, {"role": "system", "content": "be nice"},
            {"role": "assistant", "content": "yo"}]
    r = format_llama3(msgs)
    assert r.prompt == ("<|start_header_id|>user<|end_header_id|>\n\nhi<|eot_id|>"
                        "<|start_header_id|>system<|end_header_id|>\n\nbe nice<|eot_id|>"
                        "<|start_header_id|>assistant<|end_header_id|>\n\nyo<|eot_id|>"
                        "<|start_header_id|>assistant<|end_header_id|>\n\n")
    assert r.stop == "<|eot_id|>"


def test_format_guessing(bpe_md):
    name, _ = get_formatter(bpe_md, None, "<|begin_of_text|>", "<|eot_id|>")
    assert name == "llama-3"
    md, _ = build_vocab(SPECS["tiny-tinyllama-q8_0"])
    name, fmt = get_formatter(md, None, "<s>", "</s>")
    assert name == "jinja"
    r = fmt([{"role": "user", "content": "hi"}, {"role": "system", "content": "s"}])
    assert r.prompt == "<|user|>\nhi</s>\n<|system|>\ns</s>\n<|assistant|>\n"
    md, _ = build_vocab(SPECS["tiny-mixtral-q4_k_m"])
    name, fmt = get_formatter(md, None, "<s>", "</s>")
    assert name == "mistral-instruct"
    r = fmt([{"role": "user", "content": "hi"}, {"role": "system", "content": "s"}])
    assert r.prompt == "<s>[INST] hi [/INST]"
