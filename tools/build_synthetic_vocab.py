"""Train the small synthetic tokenizer vocabularies shipped in
``llama_fastapi_k8s_gpu_amd/assets`` (no network: real Llama-3 / TinyLlama
vocabularies cannot be fetched).

  * bpe_vocab.json : byte-level BPE with the Llama-3 ("llama-bpe") pre-tokenizer
                     regex, trained with HF `tokenizers` -> used for Llama-3 shaped
                     synthetic GGUFs (tokenizer.ggml.model = "gpt2").
  * spm_vocab.json : SentencePiece BPE with byte fallback, trained with
                     `sentencepiece` -> used for TinyLlama/Mixtral shaped GGUFs
                     (tokenizer.ggml.model = "llama").

The corpus is English prose + code harvested from local text files (CPython's
stdlib docstrings and this repo's docs).
"""
import glob
import io
import json
import os
import random
import sys

LLAMA3_PRETOKENIZE = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
                      r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")


def corpus(limit_bytes=12_000_000):
    files = sorted(glob.glob("/usr/lib/python3.10/**/*.py", recursive=True))
    random.Random(0).shuffle(files)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = [os.path.join(root, "SURVEY.md"), os.path.join(root, "README.md")] + files
    out, n = [], 0
    for f in files:
        try:
            t = open(f, encoding="utf-8").read()
        except Exception:
            continue
        out.append(t)
        n += len(t)
        if n > limit_bytes:
            break
    return out


def main():
    from tokenizers import Regex, Tokenizer, models, pre_tokenizers, trainers
    texts = corpus()
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_PRETOKENIZE), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    trainer = trainers.BpeTrainer(vocab_size=16000, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  show_progress=False, min_frequency=2)
    tok.train_from_iterator(texts, trainer)
    spec = json.loads(tok.to_str())
    vocab = spec["model"]["vocab"]
    tokens = [None] * len(vocab)
    for s, i in vocab.items():
        tokens[i] = s
    merges = [m if isinstance(m, str) else " ".join(m) for m in spec["model"]["merges"]]
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "llama_fastapi_k8s_gpu_amd", "assets")
    with open(os.path.join(dst, "bpe_vocab.json"), "w") as f:
        json.dump({"pre": "llama-bpe", "tokens": tokens, "merges": merges}, f, ensure_ascii=False)

    import sentencepiece as spm
    buf = io.BytesIO()
    sents = []
    for t in texts[:400]:
        sents.extend(l for l in t.splitlines() if l.strip())
    spm.SentencePieceTrainer.train(sentence_iterator=iter(sents), model_writer=buf, vocab_size=8000,
                                   model_type="bpe", byte_fallback=True, character_coverage=1.0,
                                   unk_id=0, bos_id=1, eos_id=2, pad_id=-1, split_digits=True,
                                   num_threads=4, minloglevel=2)
    sp = spm.SentencePieceProcessor(model_proto=buf.getvalue())
    pieces, scores, types = [], [], []
    for i in range(sp.get_piece_size()):
        pieces.append(sp.id_to_piece(i))
        scores.append(sp.get_score(i))
        if sp.is_unknown(i):
            types.append(2)
        elif sp.is_control(i):
            types.append(3)
        elif sp.is_byte(i):
            types.append(6)
        else:
            types.append(1)
    with open(os.path.join(dst, "spm_vocab.json"), "w") as f:
        json.dump({"pieces": pieces, "scores": scores, "types": types}, f, ensure_ascii=False)
    with open(os.path.join(dst, "spm_model.bin"), "wb") as f:
        f.write(buf.getvalue())
    print("bpe", len(tokens), len(merges), "spm", len(pieces))


if __name__ == "__main__":
    sys.exit(main())
