"""Raw engine timing (no HTTP): prefill of P tokens, then graph-replayed decode
steps at a few KV lengths. Used for profiling (rocprofv3) and quick A/B."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--slots", type=int, default=1, help="KV slots (> 1: batching on, tile16 copies + tile16 prefill)")
    ap.add_argument("--gen", type=int, default=0, help="also time a full generate() of this many tokens")
    args = ap.parse_args()
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    t0 = time.time()
    path = cached_synthetic_gguf(args.model)
    t1 = time.time()
    hip = load_hip()
    eng = hip.Engine(path, n_ctx=args.n_ctx, n_batch=512, device=0, use_graph=not args.no_graph,
                     **({"n_slots": args.slots} if args.slots > 1 else {}))
    t2 = time.time()
    import numpy as np
    toks = [int(t) for t in np.random.default_rng(0).integers(0, eng.hparams["n_vocab"], args.prompt)]
    eng.eval_logits(toks, 0)
    t3 = time.time()
    eng.eval_logits(toks, 0)
    prefill_ms = (time.time() - t3) * 1e3
    res = {"model": args.model, "gen_s": round(t1 - t0, 1), "load_s": round(t2 - t1, 1),
           "device_GB": round(eng.device_bytes / 1e9, 2), "prefill_tokens": args.prompt,
           "prefill_ms": round(prefill_ms, 2), "prefill_t16": bool(getattr(eng, "prefill_t16", False)), "prefill_tok_s": round(args.prompt / prefill_ms * 1e3, 1)}
    for pos0 in (args.prompt, min(args.n_ctx - args.steps - 2, 768)):
        ms = eng.bench_decode(args.steps, pos0)
        res[f"decode_ms_at_{pos0}"] = round(ms, 4)
        res[f"decode_tok_s_at_{pos0}"] = round(1e3 / ms, 1)
    if args.gen:
        r = eng.generate(toks, 0, args.gen, {"temperature": 1.2, "top_p": 0.9, "frequency_penalty": 0.7,
                                             "presence_penalty": 0.8, "seed": 1}, [], None, None)
        res["generate_tokens"] = len(r["tokens"])
        res["generate_decode_tok_s"] = round((len(r["tokens"]) - 1) / r["decode_s"], 1)
        res["generate_prefill_ms"] = round(r["prefill_s"] * 1e3, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
