"""split_mode=layer decode rate: the native stage chain (Engine::chain_generate) vs the host loop
it replaced (per-token eval_stage chain + host sampling) vs one engine, on one model. On a one-GPU
box every stage sits on device 0 (`--devices 0,0`); on a node each stage gets its own GPU.

    python tools/layer_split_bench.py [--model llama3-8b-q4_k_m] [--split 1,1] [--devices 0,0] [--new 128]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--split", default="1,1")
    ap.add_argument("--devices", default="0,0")
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--host-new", type=int, default=32, help="tokens for the (slow) host-loop comparison")
    args = ap.parse_args()
    import numpy as np
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    from llama_fastapi_k8s_gpu_amd.runtime.layer_split_backend import LayerSplitBackend
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    path = cached_synthetic_gguf(args.model)
    hip = load_hip()
    split = [float(v) for v in args.split.split(",")]
    devs = [int(v) for v in args.devices.split(",")]
    hp = Llama(path, split_mode="layer", tensor_split=split, layer_devices=devs, n_gpu_layers=-1, n_ctx=1024,
               n_batch=512, verbose=False)
    be = hp._backend
    assert isinstance(be, LayerSplitBackend)
    V = hp.hparams.n_vocab
    prompt = [int(t) for t in np.random.default_rng(0).integers(3, V, args.prompt)]
    greedy = SamplingParams(temperature=0.0)
    res = {"model": args.model, "split": split, "devices": devs,
           "stages": [[s.layer_begin, s.layer_end, d] for s, d in zip(be.stages, be.devices)], "prompt": args.prompt}

    def run(fn, n):
        fn(prompt, n)  # warm (graph capture, first-use allocations)
        t0 = time.perf_counter()
        r = fn(prompt, n)
        dt = time.perf_counter() - t0
        return r, dt

    r0 = be.generate(prompt, 0, args.new, greedy, [])
    r, dt = run(lambda p, n: be.generate(p, 0, n, greedy, []), args.new)
    res["chain_runs_first_diff"] = next((i for i, (a, b) in enumerate(zip(r0.tokens, r.tokens)) if a != b), None)
    res["chain"] = {"tokens": len(r.tokens), "decode_ms_per_token": round(r.decode_s * 1e3 / max(1, len(r.tokens) - 1), 3),
                    "prefill_ms": round(r.prefill_s * 1e3, 2), "wall_s": round(dt, 3)}
    be._hip = None  # the host loop the chain replaced
    r2, dt2 = run(lambda p, n: be.generate(p, 0, n, greedy, []), args.host_new)
    res["host_loop"] = {"tokens": len(r2.tokens), "ms_per_token": round(dt2 * 1e3 / len(r2.tokens), 3)}
    res["same_greedy_prefix"] = r.tokens[:len(r2.tokens)] == r2.tokens
    del be, hp
    whole = hip.Engine(path, n_ctx=1024, n_batch=512, device=devs[0], use_graph=True)
    sp = {"temperature": 0.0}
    w0 = whole.generate(prompt, 0, args.new, sp, [])
    t0 = time.perf_counter()
    w = whole.generate(prompt, 0, args.new, sp, [])
    res["one_engine_repeatable"] = list(w0["tokens"]) == list(w["tokens"])
    res["one_engine"] = {"decode_ms_per_token": round(w["decode_s"] * 1e3 / max(1, len(w["tokens"]) - 1), 3),
                         "wall_s": round(time.perf_counter() - t0, 3)}
    res["chain_tokens_equal_one_engine"] = list(w["tokens"]) == list(r.tokens)
    res["chain_vs_one_engine_first_diff"] = next((i for i, (a, b) in enumerate(zip(w["tokens"], r.tokens)) if a != b), None)
    res["one_engine_runs_first_diff"] = next((i for i, (a, b) in enumerate(zip(w0["tokens"], w["tokens"])) if a != b), None)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
