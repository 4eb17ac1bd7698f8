"""Persistent decode step vs the launch-per-op decode on a BASELINE shape:
logit agreement after a prefill, then graph-replayed decode timing of both.

    LFK_PDECODE is set per engine here; run on the GPU box:
    python tools/pdecode_check.py --model llama3-8b-q4_k_m
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--only-on", action="store_true", help="skip the launch-path engine")
    args = ap.parse_args()
    import numpy as np

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = cached_synthetic_gguf(args.model)
    hip = load_hip()
    res = {"model": args.model}
    engines = {}
    for mode in (("1",) if args.only_on else ("1", "0")):
        os.environ["LFK_PDECODE"] = mode
        e = hip.Engine(path, n_ctx=args.n_ctx, n_batch=512, device=0, use_graph=True)
        engines[mode] = e
        res[f"status_{mode}"] = e.pdecode
        print(f"[pdecode_check] LFK_PDECODE={mode}: {e.pdecode}", file=sys.stderr, flush=True)
    rng = np.random.default_rng(0)
    toks = [int(t) for t in rng.integers(0, 1000, args.prompt + 8)]
    logits = {}
    for mode, e in engines.items():
        e.eval_logits(toks[:args.prompt], 0)
        logits[mode] = [np.asarray(e.decode_logits(toks[args.prompt + i], args.prompt + i)) for i in range(4)]
        res[f"healthy_{mode}"] = bool(e.healthy)
        res[f"error_{mode}"] = e.last_error
    if "0" in logits:
        errs = [float(np.linalg.norm(a - b) / np.linalg.norm(b)) for a, b in zip(logits["1"], logits["0"])]
        res["rel_err_vs_launch_path"] = [round(x, 5) for x in errs]
        res["argmax_equal"] = [int(np.argmax(a) == np.argmax(b)) for a, b in zip(logits["1"], logits["0"])]
    print(json.dumps(res), flush=True)
    for mode, e in engines.items():
        for pos0 in (args.prompt, min(args.n_ctx - args.steps - 2, 768)):
            ms = e.bench_decode(args.steps, pos0)
            res[f"decode_ms_{mode}_at_{pos0}"] = round(ms, 4)
        res[f"healthy_after_bench_{mode}"] = bool(e.healthy)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
